// hpdct_decode.hpp -- int8 wire coefficients -> the reference's fp32
// coefficient plane (hpdct_decode_i8_f32, launched by hpdct_decode.hip; A/B
// variants in tools/kb_decode.hip): what a root does after the C4 gather of
// int8 slabs to hand dct_all_blocks_cuda's fp32 layout
// (main_newAppr.cu:252-291) to its consumer.  An HBM stream of 1 B read +
// 4 B written per coefficient.
//
// Per wave and step: kUnits KiB of int8 in (four dword loads per KiB, each
// 256 B contiguous over the wave), 4 kUnits KiB of fp32 out (non-temporal
// dwordx4 stores, each 1 KiB contiguous): lane l of store k writes floats
// [4(64k + l), 4(64k + l) + 4), so it loads exactly the dword it converts.
#pragma once

#include "hpdct_kernels.h"

namespace hpdct {

template <int kUnits>
__device__ __forceinline__ void decode_units(const int8_t* __restrict__ in, float* __restrict__ out, uint32_t lane) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(in);
    uint32_t w[4 * kUnits];
#pragma unroll
    for (int k = 0; k < 4 * kUnits; ++k) w[k] = __builtin_nontemporal_load(src + 64 * k + lane);
#pragma unroll
    for (int k = 0; k < 4 * kUnits; ++k) {
        float* dst = out + 4u * (64u * k + lane);
        __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>(w[k] & 0xffu)), dst + 0);
        __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>((w[k] >> 8) & 0xffu)), dst + 1);
        __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>((w[k] >> 16) & 0xffu)), dst + 2);
        __builtin_nontemporal_store(static_cast<float>(static_cast<int8_t>(w[k] >> 24)), dst + 3);
    }
}

// kBlock threads per workgroup; each wave decodes kUnits KiB per step and
// walks the plane with a stride of the whole grid (kPersist) or takes one
// step (grid = one wave per kUnits KiB).  Ragged tail: per element.
template <int kBlock, int kUnits, bool kPersist>
__global__ __launch_bounds__(kBlock) void decode_i8_f32_kernel(const int8_t* __restrict__ in, float* __restrict__ out,
                                                               uint64_t n) {
    constexpr uint64_t kStep = 1024u * kUnits;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64u) + threadIdx.x / 64u;
    const uint64_t waves = kPersist ? static_cast<uint64_t>(gridDim.x) * (kBlock / 64u) : 1u;
    for (uint64_t base = wave * kStep; base < n; base += waves * kStep) {
        if (base + kStep <= n) {
            decode_units<kUnits>(in + base, out + base, lane);
        } else {
            for (uint64_t i = base + lane; i < n; i += 64u) out[i] = static_cast<float>(in[i]);
        }
        if constexpr (!kPersist) break;
    }
}

// grid for a launch: one wave per step, or at most `waves_cap` waves (persistent)
template <int kBlock, int kUnits>
inline uint64_t decode_blocks(uint64_t n, uint64_t waves_cap) {
    const uint64_t steps = (n + 1024u * kUnits - 1) / (1024u * kUnits);
    uint64_t waves = waves_cap && steps > waves_cap ? waves_cap : steps;
    return (waves + kBlock / 64u - 1) / (kBlock / 64u);
}

}  // namespace hpdct
