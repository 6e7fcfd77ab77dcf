// kbench_spec.hpp -- wave-specialised forward (round 3 probe): per CU one
// persistent workgroup of 4 STORE waves (one per SIMD) and kCompute compute
// waves.  Compute waves load their own 64-tile sets (walking the sets in bands,
// set = j * W + wave) and transform them; each fp32 output row (2 KiB) goes
// into a 2-slot LDS ring owned by the wave; the store wave of the same SIMD
// drains the rings of its compute waves with 1 KiB non-temporal stores.  So
// the write stream, 80 % of the bytes, is issued by only 4 waves per CU in band
// order -- the access shape that reached 0.77 of 8 TB/s as a pure pattern
// (kbench3 "pat": band 4 waves/CU) -- while the arithmetic keeps 2-3 waves per
// SIMD issuing VALU at the full rate.
//
// Ring protocol per (compute wave w, slot k), two LDS counters:
//   written[w][k]  rows the compute wave has put into slot k (its own count)
//   drained[w][k]  rows the store wave has taken out of slot k
// Compute: row j goes to slot k = j & 1; wait until drained == written for that
// slot, write the row (ds_write), s_waitcnt lgkmcnt(0), then written += 1.
// Store: when written > drained for a slot, read the row (ds_read), s_waitcnt
// lgkmcnt(0), drained += 1, then issue the two global stores from VGPRs.
// Row j of compute wave w is row j % 8 of its set j / 8; the store wave derives
// the destination from j.  LDS operations of one wave complete in order, and
// the counter is written only after the data write has completed, so a reader
// that sees the new count reads the new data.
//
// kMath == false: the arithmetic is replaced by an s_sleep of kSleep x 64
// cycles (a pattern probe, values not a transform).
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {
namespace spec {

constexpr uint32_t kStoreWaves = 4;

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <uint32_t kCompute, bool kMath, uint32_t kSleep, unsigned kVar>
__global__ __launch_bounds__((kStoreWaves + kCompute) * 64u, 1) void fdct_spec_kernel(const uint8_t* __restrict__ img,
                                                                                    float* __restrict__ out,
                                                                                    TileGrid g, QParams qp) {
    // one array: rings [kCompute][2 slots][128 float4] then the counters
    __shared__ __attribute__((aligned(16))) float4 ring[kCompute][2][128];
    __shared__ uint32_t written[kCompute][2], drained[kCompute][2];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t nsets = g.ntiles / 64u;  // whole 64-tile sets of one tile row each (tiles_x % 64 == 0)
    const uint32_t W = gridDim.x * kCompute;
    if (threadIdx.x < kCompute * 2) {
        (&written[0][0])[threadIdx.x] = 0u;
        (&drained[0][0])[threadIdx.x] = 0u;
    }
    __syncthreads();
    auto set_base = [&](uint32_t set) {  // element offset of the set's first pixel (row 0)
        const uint32_t t0 = set * 64u, ty = t0 / g.tiles_x, tx = t0 - ty * g.tiles_x;
        return static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(tx) * 8u;
    };
    if (wv < kStoreWaves) {
        // ---- store wave: serves compute waves c with c % 4 == wv (the same SIMD)
        constexpr uint32_t kMine = (kCompute + kStoreWaves - 1) / kStoreWaves;
        uint32_t taken[kMine][2], total[kMine];
        uint32_t left = 0;
#pragma unroll
        for (uint32_t m = 0; m < kMine; ++m) {
            const uint32_t c = wv + m * kStoreWaves;
            taken[m][0] = taken[m][1] = 0u;
            const uint32_t gc = blockIdx.x * kCompute + c;
            total[m] = (c < kCompute && gc < nsets) ? 8u * ((nsets - 1u - gc) / W + 1u) : 0u;
            left += total[m];
        }
        while (left) {
            bool any = false;
#pragma unroll
            for (uint32_t m = 0; m < kMine; ++m) {
                const uint32_t c = wv + m * kStoreWaves;
                if (c >= kCompute) continue;
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k) {
                    if (taken[m][k] >= lds_load(&written[c][k])) continue;
                    const float4 a = ring[c][k][lane], b = ring[c][k][64u + lane];
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const uint32_t j = 2u * taken[m][k] + k;  // the wave's row count
                    lds_store(&drained[c][k], ++taken[m][k]);
                    const uint32_t gc = blockIdx.x * kCompute + c;
                    float* row = out + set_base(gc + (j >> 3) * W) + static_cast<uint64_t>(j & 7u) * g.width;
                    st_at<true>(row, 16u * lane, a);
                    st_at<true>(row, 16u * (64u + lane), b);
                    --left;
                    any = true;
                }
            }
            if (!any) __builtin_amdgcn_s_sleep(1);
        }
        return;
    }
    // ---- compute wave
    const uint32_t c = wv - kStoreWaves;
    uint32_t put[2] = {0u, 0u};
    const TSource<true, true> T(nullptr);
    for (uint32_t s = blockIdx.x * kCompute + c; s < nsets; s += W) {
        const uint64_t base = set_base(s) + 8u * lane;
        RawTile<uint8_t> raw;
        raw.load(img + base, g.width);
        auto emit_row = [&](auto v, float (&r)[8]) {
            constexpr uint32_t k = v & 1;
            while (lds_load(&drained[c][k]) != put[k]) __builtin_amdgcn_s_sleep(1);
            ring[c][k][2u * lane] = make_float4(r[0], r[1], r[2], r[3]);
            ring[c][k][2u * lane + 1u] = make_float4(r[4], r[5], r[6], r[7]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_store(&written[c][k], ++put[k]);
        };
        if constexpr (kMath) {
            float x[8][8];
            raw.to_float(x, 128.0f);
            fdct_tile(T, x, [&](auto v, float (&cc)[8]) {
                unroll<8>([&](auto u) { cc[u] = quantise<kVar>(cc[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
                emit_row(v, cc);
            });
        } else {
            __builtin_amdgcn_s_sleep(kSleep);
            unroll<8>([&](auto v) {
                float r[8];
                unroll<8>([&](auto u) { r[u] = static_cast<float>((raw.r[v].x >> (4 * u)) & 15u); });
                emit_row(v, r);
            });
        }
    }
}

inline bool spec_ok(const TileGrid& g) { return g.tiles_x % 64u == 0u; }

template <uint32_t kCompute, bool kMath, uint32_t kSleep, unsigned kVar>
hipError_t spec_go(const uint8_t* img, float* out, const TileGrid& g, const QParams& qp, uint32_t cus, hipStream_t s) {
    hipLaunchKernelGGL((fdct_spec_kernel<kCompute, kMath, kSleep, kVar>), dim3(cus), dim3((kStoreWaves + kCompute) * 64u),
                       0, s, img, out, g, qp);
    return hipGetLastError();
}

}  // namespace spec
}  // namespace hpdct
