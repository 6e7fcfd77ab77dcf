// kbench_dma.hpp -- A/B variant of the headline kernel (uint8 -> fp32
// quantised, built-in T) whose INPUT is read linearly through an LDS-DMA
// double buffer, by persistent workgroups.
//
// Stage = one tile row's 8 pixel rows x (kWaves * 512) px = kWaves 64-tile
// sets, one per wave.  Per workgroup, stage k+1's pixels are in flight
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, each wave 4 KiB
// contiguous of the image) while stage k is transformed:
//
//   top:  s_waitcnt vmcnt(16)     own DMA of stage k landed (only the 16
//                                  output stores of stage k-1 may be younger)
//         s_barrier               everyone's DMA of stage k landed; everyone
//                                  is done with buffer (k+1)%2
//         DMA stage k+1 -> buffer (k+1)%2      (4 instructions per wave)
//         8 x ds_read_b64         the lane's tile rows from buffer k%2
//         fdct_tile + quotient, fp32 rows re-staged through the wave's own
//         4 KiB column slab of buffer k%2 (its tile rows are in VGPRs by
//         then) and stored as 2 x 1 KiB NT stores per row
//
// One raw s_barrier per stage, no vmcnt(0) in the loop: the next stage's DMA
// stays in flight across the barrier and under the arithmetic.
// LDS: 2 x kWaves x 4 KiB.
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {
namespace dma {

template <uint32_t kWaves>
constexpr uint32_t kRowBytes = kWaves * 512u;  // one pixel row of a stage (u8)
template <uint32_t kWaves>
constexpr uint32_t kBufBytes = 8u * kRowBytes<kWaves>;

// fp32 row through the wave's slab: slot s (row parity) = slab rows 4s..4s+3,
// float4 k of the slot at slab row 4s + k/32, byte 16 (k % 32); the slot
// holds the 2 KiB output row segment in order, stored as two 1 KiB runs.
template <uint32_t kRow>
__device__ __forceinline__ void store_row_slab(uint8_t* slab, uint32_t s, float* __restrict__ seg, uint32_t lane,
                                               const float (&c)[8]) {
    auto at = [&](uint32_t k) -> float4* {
        return reinterpret_cast<float4*>(slab + (4u * s + (k >> 5)) * kRow + (k & 31u) * 16u);
    };
    *at(2u * lane) = make_float4(c[0], c[1], c[2], c[3]);
    *at(2u * lane + 1u) = make_float4(c[4], c[5], c[6], c[7]);
    const float4 a = *at(lane);
    const float4 b = *at(64u + lane);
    st_at<true>(seg, 16u * lane, a);
    st_at<true>(seg, 16u * (64u + lane), b);
}

template <unsigned kVar, uint32_t kWaves>
__global__ __launch_bounds__(kWaves * 64u, 1) void fdct_dma_kernel(const uint8_t* __restrict__ img,
                                                                  float* __restrict__ out, TileGrid g, QParams qp,
                                                                  uint32_t nstages) {
    constexpr uint32_t kRow = kRowBytes<kWaves>, kBuf = kBufBytes<kWaves>;
    // the two buffers are separate objects and every access names one of them
    // at compile time (the loop is unrolled by two): hipcc then sees that the
    // ds_reads of one buffer do not alias the DMA in flight into the other and
    // does not wait for it
    __shared__ __attribute__((aligned(16))) uint8_t buf0[kBuf];
    __shared__ __attribute__((aligned(16))) uint8_t buf1[kBuf];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t per_row = static_cast<uint32_t>(g.width / kRow);  // stages per tile row
    auto origin = [&](uint32_t st) -> uint64_t {
        const uint32_t ty = st / per_row, part = st - ty * per_row;
        return static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(part) * kRow;
    };
    // wave w's 4 KiB of the stage: buffer bytes [4096w, 4096w + 4096), 1 KiB per instruction
    auto issue = [&](uint32_t st, uint8_t* buf) {
        const uint64_t o = origin(st);
        unroll<4>([&](auto k) {
            const uint32_t off = 4096u * w + 1024u * k;  // wave-uniform
            const uint32_t row = off / kRow, col = off - row * kRow;
            const uint8_t* src = img + o + static_cast<uint64_t>(row) * g.width + col + 16u * lane;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                             reinterpret_cast<__attribute__((address_space(3))) void*>(
                                                 reinterpret_cast<uintptr_t>(buf + off)),
                                             16, 0, 0);
        });
    };
    const TSource<true, true> T(nullptr);
    // one stage from `cur` while the next one lands in `nxt`
    // (kFirst: nothing but the stage's own DMA is outstanding yet)
    auto stage = [&](auto kFirst, uint32_t st, uint8_t* cur, uint8_t* nxt) {
        if constexpr (kFirst) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (st + gridDim.x < nstages) issue(st + gridDim.x, nxt);
        RawTile<uint8_t> raw;
        unroll<8>([&](auto i) { raw.r[i] = *reinterpret_cast<const uint2*>(cur + i * kRow + 512u * w + 8u * lane); });
        float x[8][8];
        raw.to_float_minus128(x);
        float* const seg = out + origin(st) + 512u * w;  // the wave's set, pixel row 0
        uint8_t* const slab = cur + 512u * w;
        fdct_tile(T, x, [&](auto v, float (&c)[8]) {
            unroll<8>([&](auto u) { c[u] = quantise<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
            store_row_slab<kRow>(slab, v & 1, seg + v * g.width, lane, c);
        });
    };
    uint32_t st = blockIdx.x;
    if (st >= nstages) return;
    issue(st, buf0);
    stage(std::true_type{}, st, buf0, buf1);
    for (;;) {
        st += gridDim.x;
        if (st >= nstages) break;
        stage(std::false_type{}, st, buf1, buf0);
        st += gridDim.x;
        if (st >= nstages) break;
        stage(std::false_type{}, st, buf0, buf1);
    }
}

template <uint32_t kWaves>
inline bool dma_ok(const TileGrid& g) {
    return g.width % kRowBytes<kWaves> == 0u;
}

// wgs_per_cu: resident workgroups per CU the grid is sized for (LDS 2 x kBuf each)
template <unsigned kVar, uint32_t kWaves>
hipError_t dma_go(const uint8_t* img, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                  uint32_t wgs_per_cu, hipStream_t s) {
    const uint32_t nstages = static_cast<uint32_t>((static_cast<uint64_t>(g.ntiles) * 64u) / (8u * kRowBytes<kWaves>));
    const uint32_t grid = std::min<uint32_t>(nstages, cus * wgs_per_cu);
    hipLaunchKernelGGL((fdct_dma_kernel<kVar, kWaves>), dim3(grid), dim3(kWaves * 64u), 0, s, img, out, g, qp,
                       nstages);
    return hipGetLastError();
}

}  // namespace dma
}  // namespace hpdct
