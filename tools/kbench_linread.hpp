// kbench_linread.hpp -- A/B variant of the headline kernel (uint8 -> fp32
// quantised, built-in T) whose INPUT is read linearly: the membench "pat"
// cases show the set-shaped reads (8 row pieces of 512 B per wave, 8 KiB
// apart) cost 3-4 % against every wave reading 4 KiB contiguous
// (profiles/r02/s4/membench_pat2.log).
//
// One 1024-thread workgroup = 16 waves = 16 consecutive 64-tile sets = a block
// of 8 pixel rows x 8192 px (frames whose width is a multiple of 8192 px).
//   1. wave k loads 4 KiB contiguous: row k/2 of the block, half k%2
//      (4 x global_load_dwordx4, 1 KiB per instruction), into a 64 KiB LDS
//      stage [8 rows][8192 B];
//   2. barrier; wave j reads its set's tile rows (8 x ds_read_b64, 512 B of
//      a row per instruction) -- the tile registers of the product kernel;
//   3. barrier; the stage becomes the waves' output re-staging slots (4 KiB
//      each), and the rest is the product kernel (fdct_tile, quotient, LDS
//      re-staged 1 KiB NT stores).
// 64 KiB of LDS per workgroup: two workgroups (8 waves/SIMD) per CU.
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {
namespace lin {

template <unsigned kVar>
__global__ __launch_bounds__(1024, 1) void fdct_linread_kernel(const uint8_t* __restrict__ img, float* __restrict__ out,
                                                               TileGrid g, QParams qp) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[8 * 8192];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t per_row = g.tiles_x / 1024u;  // blocks per tile row
    const uint32_t ty = blockIdx.x / per_row, part = blockIdx.x - ty * per_row;
    const uint64_t origin = static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(part) * 8192u;
    {
        const uint8_t* src = img + origin + static_cast<uint64_t>(w >> 1) * g.width + (w & 1u) * 4096u;
        uint4 v[4];
        unroll<4>([&](auto k) { v[k] = *reinterpret_cast<const uint4*>(src + 1024u * k + 16u * lane); });
        uint8_t* dst = stage + (w >> 1) * 8192u + (w & 1u) * 4096u + 16u * lane;
        unroll<4>([&](auto k) { *reinterpret_cast<uint4*>(dst + 1024u * k) = v[k]; });
    }
    __syncthreads();
    RawTile<uint8_t> raw;
    unroll<8>([&](auto i) { raw.r[i] = *reinterpret_cast<const uint2*>(stage + i * 8192u + 512u * w + 8u * lane); });
    __syncthreads();
    float4* const slots = reinterpret_cast<float4*>(stage) + w * 256u;
    const TSource<true, true> T(nullptr);
    float* const seg = out + origin + 512u * w;  // the set's first pixel, row 0
    float x[8][8];
    raw.to_float(x, 128.0f);
    fdct_tile(T, x, [&](auto v, float (&c)[8]) {
        unroll<8>([&](auto u) { c[u] = quantise<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
        store_row_lds<true>(slots + (v & 1) * 128, seg + v * g.width, lane, c);
    });
}

inline bool linread_ok(const TileGrid& g) { return g.tiles_x % 1024u == 0u && g.ntiles % 1024u == 0u; }

template <unsigned kVar>
void linread_go(const uint8_t* img, float* out, const TileGrid& g, const QParams& qp, hipStream_t s) {
    hipLaunchKernelGGL((fdct_linread_kernel<kVar>), dim3(g.ntiles / 1024u), dim3(1024), 0, s, img, out, g, qp);
}

}  // namespace lin
}  // namespace hpdct
