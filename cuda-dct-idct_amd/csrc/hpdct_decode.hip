// hpdct_decode.hip -- launcher of hpdct_decode_i8_f32 (kernel: hpdct_decode.hpp).
#include "hpdct_decode.hpp"
#include "hpdct_launch.hpp"

namespace hpdct {

// One wave per KiB in one-wave workgroups, at most kDecodeCapWaves resident
// per CU (the headline's dynamic-LDS reservation): like the forward's 1 B read
// + 4 B NT write mix, the DRAM serves this stream better with fewer waves.
// 16384^2: 206 us (0.81 of 8 TB/s) against 250-252 uncapped with 256-thread
// workgroups, 236 at 8 per CU (profiles/r04/b/kb_decode.log).
constexpr uint32_t kDecodeCapWaves = 12;

hipError_t launch_decode_i8_f32(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    constexpr int kB = 64, kU = 1;
    auto* kern = decode_i8_f32_kernel<kB, kU, false>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kDecodeCapWaves);
    const uint64_t blocks = decode_blocks<kB, kU>(n, 0);
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(static_cast<uint32_t>(blocks)), dim3(kB), dyn, s, in, out, n);
    return hipGetLastError();
}

}  // namespace hpdct
