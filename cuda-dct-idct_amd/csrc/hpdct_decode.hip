// hpdct_decode.hip -- int8 wire coefficients -> the reference's fp32
// coefficient plane (hpdct_decode_i8_f32): what a root does after the C4
// gather of int8 slabs to hand dct_all_blocks_cuda's fp32
// layout (main_newAppr.cu:252-291) to its consumer.  An HBM stream of
// 1 B read + 4 B written per coefficient.
//
// Per wave: 1 KiB of int8 in (four dword loads, each 256 B contiguous over the
// wave), 4 KiB of fp32 out (four non-temporal dwordx4 stores, each 1 KiB
// contiguous): lane l of store k writes floats [4(64k + l), 4(64k + l) + 4),
// so it loads exactly the dword of bytes it converts.
#include "hpdct_kernels.h"

namespace hpdct {
namespace {

constexpr uint32_t kDecodeBlock = 256;
constexpr uint64_t kDecodeWaveBytes = 1024;

__global__ __launch_bounds__(kDecodeBlock) void decode_i8_f32_kernel(const int8_t* __restrict__ in,
                                                                     float* __restrict__ out, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kDecodeBlock / 64u) + threadIdx.x / 64u;
    const uint64_t base = wave * kDecodeWaveBytes;
    if (base >= n) return;
    if (base + kDecodeWaveBytes <= n) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(in + base);
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = __builtin_nontemporal_load(src + 64 * k + lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float* dst = out + base + 4u * (64u * k + lane);
            __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>(w[k] & 0xffu)), dst + 0);
            __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>((w[k] >> 8) & 0xffu)), dst + 1);
            __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>((w[k] >> 16) & 0xffu)), dst + 2);
            __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>(w[k] >> 24)), dst + 3);
        }
        return;
    }
    for (uint64_t i = base + lane; i < n; i += 64u) out[i] = static_cast<float>(in[i]);  // ragged tail
}

}  // namespace

hipError_t launch_decode_i8_f32(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t waves = (n + kDecodeWaveBytes - 1) / kDecodeWaveBytes;
    const uint64_t blocks = (waves + kDecodeBlock / 64u - 1) / (kDecodeBlock / 64u);
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(decode_i8_f32_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kDecodeBlock), 0, s, in, out,
                       n);
    return hipGetLastError();
}

}  // namespace hpdct
