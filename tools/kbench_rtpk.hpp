// kbench_rtpk.hpp -- A/B variant of the C3 one-pass round trip
// (csrc/hpdct_roundtrip.hpp, kFast tables, uint8 reconstruction, sums with the
// pixels stashed in LDS) whose four transform passes, quotient, dequantiser
// and level shifts run as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32: two IEEE operations per instruction, each half rounded like
// the scalar one).  tools/kbench3 "issue": per fma the packed form issues
// ~1.65x faster at every occupancy.
//
// Pairing (zero terms of T skipped exactly as in the scalar chains; a term
// zero in one half only adds fma(0, P, s) = s):
//   forward  pass 1 pixel columns (2c, 2c+1), shared coefficient T[v][i]
//            pass 2 output columns kPairU (rows of T with matching zeros)
//   inverse  pass 1 coefficient columns (2c, 2c+1), shared T[i][v]
//            pass 2 output columns kPairInvU: columns of T with identical
//            zero patterns, (0,1) (6,7) (3,4) (2,5)
// Every chain keeps the scalar kernel's i = 0..7 order from +0, so the
// coefficients, reconstruction and sums are bit-identical to the product.
#pragma once

#include "hpdct_roundtrip.hpp"
#include "kbench_variants.hpp"

namespace hpdct {
namespace rtpk {

using ab::f32x2;
using ab::fma2;
inline constexpr int kPairInvU[4][2] = {{0, 1}, {6, 7}, {3, 4}, {2, 5}};

template <typename Emit2>
__device__ __forceinline__ void idct_tile_pk(const f32x2 (&d2)[8][4], Emit2&& emit2) {
    f32x2 p2[8][4];
    // P[v][col] = sum_i T[i][v] D[i][col]
    unroll<8>([&](auto v) {
        unroll<4>([&](auto cp) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float c = kBuiltinT.v[i * 8 + v];
                if constexpr (c != 0.0f) s = fma2(f32x2{c, c}, d2[i][cp], s);
            });
            p2[v][cp] = s;
        });
    });
    // R[v][u] = sum_i P[v][i] T[i][u]
    unroll<8>([&](auto v) {
        f32x2 r2[4];
        unroll<4>([&](auto k) {
            constexpr int u0 = kPairInvU[k][0], u1 = kPairInvU[k][1];
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float a = kBuiltinT.v[i * 8 + u0], b = kBuiltinT.v[i * 8 + u1];
                if constexpr (a != 0.0f || b != 0.0f) {
                    const float pv = p2[v][i / 2][i % 2];
                    s = fma2(f32x2{a, b}, f32x2{pv, pv}, s);
                }
            });
            r2[k] = s;
        });
        emit2(v, r2);
    });
}

template <bool kStats>
__global__ __launch_bounds__(512, 2) void roundtrip_pk_kernel(const uint8_t* __restrict__ img, float* __restrict__ coef,
                                                              uint8_t* __restrict__ recon, RtSums* __restrict__ sums,
                                                              TileGrid g, QParams qp) {
    constexpr unsigned kVar = (2u << 12) | kVarNT | kVarLdsStore | kVarFastDiv;
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, float> coef_sink{coef, g.width, slots};
    float acc_f = 0.0f;
    uint32_t acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    uint2* stash = nullptr;
    if constexpr (kStats) {
        __shared__ uint2 raw_lds[512 / 64][8 * 64];
        stash = raw_lds[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
    }
    const uint32_t lane = threadIdx.x & 63u;

    walk_sets<kVar>(img, g, slots, [&](const RawTile<uint8_t>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
        if constexpr (kStats) unroll<8>([&](auto i) { stash[i * 64u + lane] = raw.r[i]; });
        float xs[8][8];
        raw.to_float(xs, 0.0f);
        f32x2 x2[8][4];
        unroll<8>([&](auto i) {
            unroll<4>([&](auto cp) { x2[i][cp] = f32x2{xs[i][2 * cp], xs[i][2 * cp + 1]} - f32x2{128.0f, 128.0f}; });
        });
        // ---- forward: T.(X-128).T^T, round(C/Q) (verified 3-op quotient, 3-op roundf)
        uint2 q8[8];
        ab::fdct_tile_pk(x2, [&](auto v, f32x2(&c2)[4]) {
            float c[8];
            unroll<4>([&](auto k) {
                constexpr int u0 = ab::kPairU[k][0], u1 = ab::kPairU[k][1];
                const f32x2 q2 = {qp.q.v[v * 8 + u0], qp.q.v[v * 8 + u1]};
                const f32x2 r2 = {qp.r.v[v * 8 + u0], qp.r.v[v * 8 + u1]};
                const f32x2 q0 = c2[k] * r2;
                const f32x2 e = fma2(-q0, q2, c2[k]);
                f32x2 d = fma2(e, r2, q0);
                d = d + f32x2{__builtin_copysignf(0.49999997f, d.x), __builtin_copysignf(0.49999997f, d.y)};
                c[u0] = __builtin_truncf(d.x);
                c[u1] = __builtin_truncf(d.y);
            });
            coef_sink(v, p, ok, seg, c);
            uint32_t w0 = 0u, w1 = 0u;
            cvt_into_byte<0>(w0, c[0]), cvt_into_byte<1>(w0, c[1]), cvt_into_byte<2>(w0, c[2]),
                cvt_into_byte<3>(w0, c[3]);
            cvt_into_byte<0>(w1, c[4]), cvt_into_byte<1>(w1, c[5]), cvt_into_byte<2>(w1, c[6]),
                cvt_into_byte<3>(w1, c[7]);
            q8[v] = make_uint2(w0, w1);
        });
        // ---- inverse: D = q*Q, T^T.D.T + 128
        f32x2 d2[8][4];
        unroll<8>([&](auto i) {
            unroll<4>([&](auto cp) {
                const uint32_t w = cp < 2 ? q8[i].x : q8[i].y;
                constexpr int b0 = (2 * cp) & 3;
                const f32x2 qv = {static_cast<float>(static_cast<int8_t>((w >> (8 * b0)) & 0xffu)),
                                  static_cast<float>(static_cast<int8_t>((w >> (8 * (b0 + 1))) & 0xffu))};
                d2[i][cp] = qv * f32x2{qp.q.v[i * 8 + 2 * cp], qp.q.v[i * 8 + 2 * cp + 1]};
            });
        });
        idct_tile_pk(d2, [&](auto v, f32x2(&r2)[4]) {
            float r[8];
            unroll<4>([&](auto k) {
                const f32x2 t = r2[k] + f32x2{128.0f, 128.0f};
                r[kPairInvU[k][0]] = t.x;
                r[kPairInvU[k][1]] = t.y;
            });
            const uint2 r8 = make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
            if constexpr (kStats) {
                const uint2 w = stash[v * 64u + lane];
                acc_xx = __builtin_amdgcn_udot4(w.x, w.x, acc_xx, false);
                acc_xx = __builtin_amdgcn_udot4(w.y, w.y, acc_xx, false);
                acc_xr = __builtin_amdgcn_udot4(w.x, r8.x, acc_xr, false);
                acc_xr = __builtin_amdgcn_udot4(w.y, r8.y, acc_xr, false);
                acc_rr = __builtin_amdgcn_udot4(r8.x, r8.x, acc_rr, false);
                acc_rr = __builtin_amdgcn_udot4(r8.y, r8.y, acc_rr, false);
                unroll<8>([&](auto u) {
                    const float e = byte_f32(u < 4 ? w.x : w.y, u & 3) - r[u];
                    acc_f = __builtin_fmaf(e, e, acc_f);
                });
            }
            st<true>(reinterpret_cast<uint2*>(recon + p.base + v * g.width), r8);
        });
    });

    if constexpr (kStats) {  // the product's epilogue (hpdct_roundtrip.hpp)
        const float fx = __builtin_rintf(acc_f * kRtFixScale);
        const bool f_ok = fx < 0x1p40f;
        unsigned long long f = f_ok ? static_cast<unsigned long long>(fx) : 0ull;
        unsigned long long e8 = static_cast<unsigned long long>(acc_xx + acc_rr - 2u * acc_xr);
        unsigned long long xx = static_cast<unsigned long long>(acc_xx);
        auto wsum = [](unsigned long long x) {
            unroll<6>([&](auto s) { x += __shfl_xor(x, 1 << s, 64); });
            return x;
        };
        f = wsum(f), e8 = wsum(e8), xx = wsum(xx);
        if (__builtin_amdgcn_ballot_w64(!f_ok) != 0) f |= kRtSseF32Invalid;
        __shared__ unsigned long long part[512 / 64][3];
        const uint32_t w = threadIdx.x / 64u;
        if ((threadIdx.x & 63u) == 0u) part[w][0] = f, part[w][1] = e8, part[w][2] = xx;
        __syncthreads();
        if (threadIdx.x < 3u) {
            unsigned long long s = 0, bad = 0;
            for (uint32_t k = 0; k < 512u / 64u; ++k) {
                s += part[k][threadIdx.x] & ~kRtSseF32Invalid;
                bad |= part[k][threadIdx.x] & kRtSseF32Invalid;
            }
            auto* const dst = reinterpret_cast<unsigned long long*>(sums) + threadIdx.x;
            if (s) atomicAdd(dst, s);
            if (bad) atomicOr(dst, kRtSseF32Invalid);
        }
    }
}

}  // namespace rtpk
}  // namespace hpdct
