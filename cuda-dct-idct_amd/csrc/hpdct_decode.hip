// hpdct_decode.hip -- launcher of hpdct_decode_i8_f32 (kernel: hpdct_decode.hpp).
#include "hpdct_decode.hpp"

namespace hpdct {

// one wave per KiB, 256-thread workgroups (the round-4 A/B, tools/kb_decode.hip)
hipError_t launch_decode_i8_f32(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    constexpr int kB = 256, kU = 1;
    const uint64_t blocks = decode_blocks<kB, kU>(n, 0);
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((decode_i8_f32_kernel<kB, kU, false>), dim3(static_cast<uint32_t>(blocks)), dim3(kB), 0, s, in,
                       out, n);
    return hipGetLastError();
}

}  // namespace hpdct
