// kbench_band.hpp -- A/B variant of the tile-per-lane forward kernel with a
// persistent, banded schedule: W = kWavesPerCU x CUs resident waves, wave w
// takes sets w, w + W, w + 2W, ... so at any time all waves work on W
// consecutive 64-tile sets (the chip-wide write front is W x 16 KiB for
// fp32 output), and each wave's next set is loaded into registers before the
// current one is transformed and stored.  The access pattern alone runs at
// 0.77 of 8 TB/s with 4 waves per CU against 0.72 for one set per
// non-persistent wave (tools/kbench3 "pat" group, profiles/r03).
// Arithmetic, staging and stores are the product's (fdct_tile, quantise,
// RowSink), so the output is bit-identical.
// kPk: the packed-fp32 transform and quotient of tools/kbench_variants.hpp
// (ab::fdct_tile_pk, v_pk_fma_f32; bit-exact): at one wave per SIMD a wave
// issues a VALU instruction every 4 cycles at best, so two fmas per
// instruction may give back the rate the band schedule loses there.
#pragma once

#include "hpdct_kernels_impl.hpp"
#include "kbench_variants.hpp"

namespace hpdct {
namespace band {

template <unsigned kVar, typename TIn, typename Body>
__device__ __forceinline__ void walk_band(const TIn* __restrict__ src, const TileGrid& g, Body&& body) {
    constexpr uint32_t kWavesPerBlock = kBlock<kVar> / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t nsets = (g.ntiles + 63u) / 64u;
    uint32_t s = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + threadIdx.x / 64u);
    if (s >= nsets) return;
    TilePos p = tile_pos(g, s * 64u + lane);
    RawTile<TIn> cur;
    cur.load(src + p.base, g.width);
    for (;;) {
        const uint32_t sn = s + nw;
        const bool more = sn < nsets;
        TilePos pn{0, false};
        RawTile<TIn> nxt;
        if (more) {
            pn = tile_pos(g, sn * 64u + lane);
            nxt.load(src + pn.base, g.width);
        }
        const uint32_t t0 = s * 64u;
        const bool whole = t0 + 63u < g.ntiles && (t0 / g.tiles_x) == ((t0 + 63u) / g.tiles_x);
        const uint64_t seg = p.base - 8u * static_cast<uint64_t>(lane);
        if (p.valid) body(cur, p, whole ? 64u : 0u, seg);
        if (!more) break;
        s = sn;
        p = pn;
        cur = nxt;
    }
}

template <typename TOut, unsigned kVar, bool kPk = false>
__global__ __launch_bounds__(kBlock<kVar>, 1) void fdct_band_kernel(const uint8_t* __restrict__ img,
                                                                   TOut* __restrict__ out, TileGrid g, QParams qp) {
    const TSource<true, true> T(nullptr);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, TOut> sink{out, g.width, slots};
    walk_band<kVar>(img, g, [&](const RawTile<uint8_t>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
        if constexpr (kPk) {
            static_assert(std::is_same_v<TOut, float> && (kVar & kVarFastDiv) != 0, "packed: fp32 out, fast quotient");
            using ab::f32x2;
            float xs[8][8];
            raw.to_float(xs, 0.0f);
            f32x2 x2[8][4];
            unroll<8>([&](auto i) {
                unroll<4>([&](auto cp) { x2[i][cp] = f32x2{xs[i][2 * cp], xs[i][2 * cp + 1]} - f32x2{128.0f, 128.0f}; });
            });
            ab::fdct_tile_pk(x2, [&](auto v, f32x2(&c2)[4]) {
                float c[8];
                unroll<4>([&](auto k) {
                    constexpr int u0 = ab::kPairU[k][0], u1 = ab::kPairU[k][1];
                    const f32x2 q2 = {qp.q.v[v * 8 + u0], qp.q.v[v * 8 + u1]};
                    const f32x2 r2 = {qp.r.v[v * 8 + u0], qp.r.v[v * 8 + u1]};
                    const f32x2 q0 = c2[k] * r2;
                    const f32x2 e = ab::fma2(-q0, q2, c2[k]);
                    f32x2 d = ab::fma2(e, r2, q0);
                    d = d + f32x2{__builtin_copysignf(0.49999997f, d.x), __builtin_copysignf(0.49999997f, d.y)};
                    c[u0] = __builtin_truncf(d.x);
                    c[u1] = __builtin_truncf(d.y);
                });
                sink(v, p, ok, seg, c);
            });
            return;
        }
        float x[8][8];
        raw.to_float(x, 128.0f);
        fdct_tile(T, x, [&](auto v, float (&c)[8]) {
            if constexpr (std::is_same_v<TOut, int8_t> && (kVar & kVarI8Pack) != 0) {
                unroll<8>([&](auto u) { c[u] = quotient<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
                const uint2 w = make_uint2(pack_q_i8x4(c[0], c[1], c[2], c[3]), pack_q_i8x4(c[4], c[5], c[6], c[7]));
                st<(kVar & kVarNT) != 0>(reinterpret_cast<uint2*>(out + p.base + v * g.width), w);
                return;
            }
            unroll<8>([&](auto u) { c[u] = quantise<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
            sink(v, p, ok, seg, c);
        });
    });
}

// waves_per_cu resident waves per CU (the grid), kVar's workgroup size
template <typename TOut, unsigned kVar, bool kPk = false>
hipError_t band_go(const uint8_t* img, TOut* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                   uint32_t waves_per_cu, hipStream_t s) {
    const uint32_t per = kBlock<kVar> / 64u, sets = (g.ntiles + 63u) / 64u;
    const uint32_t grid = std::min<uint32_t>((sets + per - 1) / per, cus * waves_per_cu / per);
    hipLaunchKernelGGL((fdct_band_kernel<TOut, kVar, kPk>), dim3(grid), dim3(kBlock<kVar>), 0, s, img, out, g, qp);
    return hipGetLastError();
}

}  // namespace band
}  // namespace hpdct
