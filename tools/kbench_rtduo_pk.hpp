// kbench_rtduo_pk.hpp -- the C3 duo round trip with packed fp32 (tools only;
// round 5, rejected: 78.6 against 76.3 us with sums at 8192^2, 69.7 against
// 67.0 without, profiles/r05/b/kb_rt_8192.log).  Same arithmetic and sums as
// hpdct_rt_duo.hpp's rt_duo_body, bit-identical; fewer VALU instructions
// (733 against 1,002 per lane without sums) but no faster.
#pragma once

#include "hpdct_rt_duo.hpp"

namespace hpdct {

// The same round trip with both transforms, the quantiser, the dequantiser
// and the level shift in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32: two IEEE operations per instruction, each half rounded as
// the scalar one, so bit-identical).  Pass 1 of each transform pairs two
// columns of the lane's half (same T entry, broadcast); pass 2 pairs output
// columns (u, u+1) (T entries differ per half; a term whose T entry is zero
// in one half only adds fma(0, P, s) = s exactly: P is finite and a chain
// from +0 never holds -0).  The quantiser takes a column pair in one packed
// sequence: the short JPEG form when all four positions of the pair (two
// rows, the lanes' 2k and 2k+1, times two columns) have one, the verified
// 6-op quotient otherwise.
template <bool kStats, int kQMode, int kRecon, bool kRun>
__device__ __forceinline__ void rt_duo_body_pk(const uint8_t* __restrict__ img, float* __restrict__ coef,
                                               uint8_t* __restrict__ recon, const DuoAddr& a, uint32_t h,
                                               const float (&tab)[2][64], float4* __restrict__ slots, f32x2& acc_f2,
                                               uint32_t& acc_xx, uint32_t& acc_xr, uint32_t& acc_rr) {
    constexpr bool kNT = true;
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* const src = img + a.base;
    auto T = [](int v, int i) constexpr { return kBuiltinT.v[v * 8 + i]; };

    uint2 raw[4];
    unroll<4>([&](auto k) {
        raw[k] = make_uint2(0u, 0u);
        if (kRun || a.valid) raw[k] = *reinterpret_cast<const uint2*>(src + a.off(2u * k + h));
    });
    uint32_t lo[4], hi[4];
    unroll<4>([&](auto k) {
        lo[k] = raw[k].x ^ 0x80808080u, hi[k] = raw[k].y ^ 0x80808080u;
        xswap(lo[k], hi[k]);
    });
    // ---- forward pass 1, column pairs (2cp, 2cp+1) of the lane's half
    f32x2 pa[4][2], pb[4][2];
    unroll<2>([&](auto cp) {
        f32x2 x2[8];
        unroll<4>([&](auto k) {
            x2[2 * k] = f32x2{px_minus128(lo[k], 2 * cp), px_minus128(lo[k], 2 * cp + 1)};
            x2[2 * k + 1] = f32x2{px_minus128(hi[k], 2 * cp), px_minus128(hi[k], 2 * cp + 1)};
        });
        unroll<8>([&](auto v) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float c = T(v, i);
                if constexpr (c != 0.0f) s = fma2(f32x2{c, c}, x2[i], s);
            });
            if constexpr (v % 2 == 0) {
                pa[v / 2][cp] = s;
            } else {
                pb[v / 2][cp] = s;
            }
        });
    });
    auto swap2 = [](f32x2& x, f32x2& y) {
        float x0 = x.x, x1 = x.y, y0 = y.x, y1 = y.y;
        xswap(x0, y0), xswap(x1, y1);
        x = f32x2{x0, x1}, y = f32x2{y0, y1};
    };
    // ---- rows 2k+h: columns (0,1) (2,3) in pa[k][0..1], (4,5) (6,7) in pb[k][0..1]
    unroll<4>([&](auto k) { unroll<2>([&](auto cp) { swap2(pa[k][cp], pb[k][cp]); }); });

    // ---- forward pass 2 (output pairs (2j, 2j+1)), quantiser, coefficient rows, D = q * Q
    f32x2 da[4][2], db[4][2];
    unroll<4>([&](auto k) {
        const uint32_t row = 2u * k + h;
        const float4* const qrow = reinterpret_cast<const float4*>(&tab[0][row * 8u]);
        const float4* const rrow = reinterpret_cast<const float4*>(&tab[1][row * 8u]);
        const float4 q0 = qrow[0], q1 = qrow[1], r0 = rrow[0], r1 = rrow[1];
        const f32x2 q2[4] = {{q0.x, q0.y}, {q0.z, q0.w}, {q1.x, q1.y}, {q1.z, q1.w}};
        const f32x2 r2[4] = {{r0.x, r0.y}, {r0.z, r0.w}, {r1.x, r1.y}, {r1.z, r1.w}};
        const float prow[8] = {pa[k][0].x, pa[k][0].y, pa[k][1].x, pa[k][1].y,
                               pb[k][0].x, pb[k][0].y, pb[k][1].x, pb[k][1].y};
        f32x2 c2[4];
        unroll<4>([&](auto j) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float t0 = T(2 * j, i), t1 = T(2 * j + 1, i);
                if constexpr (t0 != 0.0f || t1 != 0.0f) s = fma2(f32x2{t0, t1}, f32x2{prow[i], prow[i]}, s);
            });
            constexpr int u0 = 2 * j, u1 = 2 * j + 1;
            constexpr int pl0 = 2 * k * 8 + u0, ph0 = (2 * k + 1) * 8 + u0;
            constexpr int pl1 = 2 * k * 8 + u1, ph1 = (2 * k + 1) * 8 + u1;
            constexpr bool kShort = kQMode == 2 && quantforms::jpeg_form(pl0) != quantforms::kFull &&
                                    quantforms::jpeg_form(ph0) != quantforms::kFull &&
                                    quantforms::jpeg_form(pl1) != quantforms::kFull &&
                                    quantforms::jpeg_form(ph1) != quantforms::kFull;
            f32x2 b;
            if constexpr (kShort) {
                auto mag = [&](auto pl, auto ph) {
                    if constexpr (quantforms::jpeg_bias(pl) == quantforms::jpeg_bias(ph)) {
                        return quantforms::jpeg_bias(pl);
                    } else {
                        return h ? quantforms::jpeg_bias(ph) : quantforms::jpeg_bias(pl);
                    }
                };
                const float m0 = mag(std::integral_constant<int, pl0>{}, std::integral_constant<int, ph0>{});
                const float m1 = mag(std::integral_constant<int, pl1>{}, std::integral_constant<int, ph1>{});
                b = fma2(s, r2[j], f32x2{signed_mag(m0, s.x), signed_mag(m1, s.y)});
            } else {
                const f32x2 qa = s * r2[j];
                const f32x2 e = fma2(-qa, q2[j], s);
                const f32x2 d = fma2(e, r2[j], qa);
                b = d + f32x2{signed_half(d.x), signed_half(d.y)};
            }
            c2[j] = f32x2{__builtin_truncf(b.x), __builtin_truncf(b.y)};
        });
        // coefficient row 2k+h
        if constexpr (kRun) {
            float4* const slot = slots + (k & 1) * 128;
            slot[2u * lane] = make_float4(c2[0].x, c2[0].y, c2[1].x, c2[1].y);
            slot[2u * lane + 1u] = make_float4(c2[2].x, c2[2].y, c2[3].x, c2[3].y);
            const float4 lo4 = slot[lane], hi4 = slot[64u + lane];
            float* const dst = coef + a.base;
            st<kNT>(reinterpret_cast<float4*>(dst + (2u * k * a.width + 4u * lane)), lo4);
            st<kNT>(reinterpret_cast<float4*>(dst + ((2u * k + 1u) * a.width + 4u * lane)), hi4);
        } else {
            const float c[8] = {c2[0].x, c2[0].y, c2[1].x, c2[1].y, c2[2].x, c2[2].y, c2[3].x, c2[3].y};
            if (a.valid) store_row<kNT>(coef + a.base + a.off(row), c);
        }
        unroll<2>([&](auto cp) {
            da[k][cp] = c2[cp] * q2[cp];
            db[k][cp] = c2[2 + cp] * q2[2 + cp];
        });
    });
    // ---- columns of D: row 2k in da[k][cp], row 2k+1 in db[k][cp]
    unroll<4>([&](auto k) { unroll<2>([&](auto cp) { swap2(da[k][cp], db[k][cp]); }); });
    // ---- inverse pass 1, column pairs: P[v][c] = chain_i T[i][v] D[i][c]
    unroll<2>([&](auto cp) {
        f32x2 d2[8];
        unroll<4>([&](auto k) { d2[2 * k] = da[k][cp], d2[2 * k + 1] = db[k][cp]; });
        unroll<8>([&](auto v) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float c = T(i, v);
                if constexpr (c != 0.0f) s = fma2(f32x2{c, c}, d2[i], s);
            });
            if constexpr (v % 2 == 0) {
                pa[v / 2][cp] = s;
            } else {
                pb[v / 2][cp] = s;
            }
        });
    });
    unroll<4>([&](auto k) { unroll<2>([&](auto cp) { swap2(pa[k][cp], pb[k][cp]); }); });
    // ---- inverse pass 2 (output pairs (2j, 2j+1)), + 128, uint8, sums
    unroll<4>([&](auto k) {
        const float prow[8] = {pa[k][0].x, pa[k][0].y, pa[k][1].x, pa[k][1].y,
                               pb[k][0].x, pb[k][0].y, pb[k][1].x, pb[k][1].y};
        float r[8];
        unroll<4>([&](auto j) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float t0 = T(i, 2 * j), t1 = T(i, 2 * j + 1);
                if constexpr (t0 != 0.0f || t1 != 0.0f) s = fma2(f32x2{t0, t1}, f32x2{prow[i], prow[i]}, s);
            });
            const f32x2 o = s + f32x2{128.0f, 128.0f};  // add_matrix_scalar (utils_kernels.cu:29)
            r[2 * j] = o.x, r[2 * j + 1] = o.y;
        });
        const uint2 r8 = make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
        if constexpr (kStats) rt_duo_row_sums(raw[k], r, r8, acc_f2, acc_xx, acc_xr, acc_rr);
        if constexpr (kRecon == kRtReconU8) {
            if (kRun || a.valid) st<kNT>(reinterpret_cast<uint2*>(recon + a.base + a.off(2u * k + h)), r8);
        }
    });
    if constexpr (kStats) {
        if (!(kRun || a.valid)) acc_f2 = f32x2{0.0f, 0.0f}, acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    }
}


// roundtrip_duo_kernel with the packed body (same launch shape and epilogue)
template <bool kStats, int kQMode, int kRecon, int kBlockT = 256, int kWaves = 6>
__global__ __launch_bounds__(kBlockT) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void roundtrip_duo_pk_kernel(
    const uint8_t* __restrict__ img, float* __restrict__ coef, uint8_t* __restrict__ recon, RtSums* __restrict__ sums,
    TileGrid g, QParams qp) {
    constexpr uint32_t kW = kBlockT / 64u;
    __shared__ __attribute__((aligned(16))) float tab[2][64];
    __shared__ __attribute__((aligned(16))) float4 stage[kW][2][128];
    if (threadIdx.x < 64u) tab[0][threadIdx.x] = qp.q.v[threadIdx.x], tab[1][threadIdx.x] = qp.r.v[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, t = lane & 31u, h = lane >> 5;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kW + wv);
    const uint32_t first = wave * kRtDuoTiles;
    f32x2 acc_f2 = {0.0f, 0.0f};
    uint32_t acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    if (first < g.ntiles) {
        const uint32_t by = first / g.tiles_x, bx = first - by * g.tiles_x;
        const DuoAddr a{static_cast<uint64_t>(by) * 8u * g.width + static_cast<uint64_t>(bx) * 8u, t * 8u,
                        static_cast<uint32_t>(g.width), true};
        rt_duo_body_pk<kStats, kQMode, kRecon, true>(img, coef, recon, a, h, tab, stage[wv][0], acc_f2, acc_xx, acc_xr,
                                                     acc_rr);
    }
    if constexpr (kStats) {
        bool ok = true;
        unsigned long long f = rt_sse_fix(acc_f2.x, ok) + rt_sse_fix(acc_f2.y, ok);
        const uint32_t e8 = acc_xx + acc_rr - 2u * acc_xr;
        unsigned long long ints = (static_cast<unsigned long long>(acc_xx) << 32) | e8;
        f = wave_sum_dpp(f), ints = wave_sum_dpp(ints);
        const bool bad = __builtin_amdgcn_ballot_w64(!ok) != 0;
        if (lane == 0u) {
            auto* const dst = reinterpret_cast<unsigned long long*>(sums) + (wave % kRtSpread) * kRtSpreadStride;
            if (f) atomicAdd(dst, f);
            if (bad) atomicOr(dst, kRtSseF32Invalid);
            if (ints & 0xffffffffull) atomicAdd(dst + 1, ints & 0xffffffffull);
            if (ints >> 32) atomicAdd(dst + 2, ints >> 32);
        }
    }
}

}  // namespace hpdct
