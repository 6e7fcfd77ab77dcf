// hpdct_rt_duo.hpp -- the C3 round trip (uint8 frame -> quantised fp32
// coefficients + uint8 reconstruction + PEEN/MSE sums) with TWO lanes per
// tile, for CDNA4 / gfx950.
//
// Why: the tile-per-lane round trip (hpdct_roundtrip.hpp) keeps a whole tile
// per lane through both transforms, 118-120 VGPRs, so only 4 waves fit a SIMD
// and the two transforms' latency per wave is exposed (bounded to 5 waves the
// compiler spills).  Here lane l of a wave works on tile t = l & 31 of the
// wave's 32 consecutive tiles, half h = l >> 5, so a lane holds 32 values of
// its tile, not 64.
//
// The two halves of a tile sit 32 lanes apart, so every change of layout
// between the reference's passes is ONE v_permlane32_swap_b32 per pair of
// registers (lanes 32..63 of one register trade places with lanes 0..31 of
// the other): no LDS, no select.  A lane's rows are 2k + h (k = 0..3), its
// columns 4h..4h+3.  Per lane:
//
//   load      rows 2k+h, one 8-byte load per row (the wave reads rows 2k and
//             2k+1 of its 32 tiles: two 256-B runs per instruction)
//   swap      -> columns 4h..4h+3 of all 8 rows
//   fwd 1     P[v][c] = chain_i T[v][i] (X[i][c] - 128)   main_newAppr.cu:193-197
//   swap      -> rows 2k+h of P, all 8 columns
//   fwd 2     C[v][u] = chain_i P[v][i] T[u][i]            main_newAppr.cu:206-209
//             q = round(C / Q[v][u])                        utils_kernels.cu:42
//             fp32 coefficient rows out (re-staged through LDS: 1 KiB
//             contiguous per store instruction)
//             D = q * Q[v][u]                               utils_kernels.cu:55
//   swap      -> columns 4h..4h+3 of D
//   inv 1     P[v][c] = chain_i T[i][v] D[i][c]            main_newAppr.cu:236-239
//   swap      -> rows 2k+h
//   inv 2     R[v][u] = chain_i P[v][i] T[i][u]; R + 128  main_newAppr.cu:246-248,
//             uint8 pixels (convertToUnsignedChar)         utils_kernels.cu:29, utils.cu:21
//             and the sums against the loaded rows (the lane's own rows again)
//
// The quantised rows stay fp32 between the transforms (32 VGPRs), so the
// int8 packing and unpacking of the tile kernel (128 conversions per tile)
// are gone.  Chains, quotient forms, rounding and sums are those of the tile
// kernel, so coefficients, reconstruction and all three sums are
// bit-identical to it (tools/kbench3 group rtduo checks that on the GPU;
// tests/test_gpu_roundtrip.py against the oracle).
//
// The lanes of one instruction quantise two table positions, (2k, u) and
// (2k+1, u): Q and RN(1/Q) come per lane from a copy of the table in LDS
// (broadcast reads), and a short JPEG form (hpdct_quant_forms.h) is used at a
// column when BOTH positions have one, the verified 6-op quotient otherwise.
//
// sse_f32 is the tile kernel's per-tile fp32 chain over the 64 pixels in row
// order: row 2k in lanes 0..31, its sum moved to lanes 32..63 for row 2k+1,
// and back for row 2k+2 (two swaps per row pair).
#pragma once

#include "hpdct_octet.hpp"
#include "hpdct_roundtrip.hpp"

namespace hpdct {

namespace {

constexpr uint32_t kRtDuoTiles = 32;  // tiles per wave

// lanes 0..31 keep a and take b's old value from lane + 32 into b;
// lanes 32..63 keep b and take a's old value from lane - 32 into a
__device__ __forceinline__ void xswap(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0], b = r[1];
}
__device__ __forceinline__ void xswap(float& a, float& b) {
    uint32_t x = __float_as_uint(a), y = __float_as_uint(b);
    xswap(x, y);
    a = __uint_as_float(x), b = __uint_as_float(y);
}

// signed magnitude as one v_bitop3_b32 (magnitude bits from m, sign from x)
__device__ __forceinline__ float signed_mag(float m, float x) {
    return __uint_as_float(__builtin_amdgcn_bitop3_b32(0x7fffffffu, __float_as_uint(m), __float_as_uint(x), 0xca));
}

// (-128 + byte k of w) exactly: the sign-extended byte of w ^ 0x80808080
__device__ __forceinline__ float px_minus128(uint32_t w_xor, int k) {
    return static_cast<float>(static_cast<int32_t>(static_cast<int8_t>(w_xor >> (8 * k))));
}

// Sum over the wave in DPP steps (row_shr 1, 2, 4, 8 inside each 16-lane row,
// then row_bcast 15 and 31 across rows): lane 63 ends with the total, read
// back with one readlane.  No LDS traffic, unlike __shfl_xor.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), kCtrl, kRowMask, 0xf, false));
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void dpp_add(uint32_t& v) {
    v += dpp_u32<kCtrl, kRowMask>(v);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void dpp_add(unsigned long long& v) {
    const uint32_t lo = dpp_u32<kCtrl, kRowMask>(static_cast<uint32_t>(v));
    const uint32_t hi = dpp_u32<kCtrl, kRowMask>(static_cast<uint32_t>(v >> 32));
    v += (static_cast<unsigned long long>(hi) << 32) | lo;
}
template <typename U>
__device__ __forceinline__ U wave_sum_dpp(U v) {
    dpp_add<0x111, 0xf>(v);  // row_shr:1
    dpp_add<0x112, 0xf>(v);  // row_shr:2
    dpp_add<0x114, 0xf>(v);  // row_shr:4
    dpp_add<0x118, 0xf>(v);  // row_shr:8
    dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    if constexpr (sizeof(U) == 8) {
        const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v)), 63));
        const uint32_t hi =
            static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v >> 32)), 63));
        return (static_cast<unsigned long long>(hi) << 32) | lo;
    } else {
        return static_cast<U>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
    }
}

// Where a duo wave's rows live: the wave's first tile's top-left pixel (a
// wave-uniform base, SGPRs) plus a 32-bit per-lane offset.  A wave's 32 tiles
// are consecutive in row-major tile order, so every offset is >= 0 (tiles in
// the next tile row start 8 * width further on); it stays below 2^32 bytes of
// fp32 for widths below 4 Mi pixels.  So every access is the saddr + voffset
// form, also in a wave whose tiles straddle tile rows (ragged widths).
struct DuoAddr {
    uint64_t base;      // element index of the wave's first tile's top-left pixel
    uint32_t lane_off;  // element offset of this lane's tile from base
    uint32_t width;     // elements per image row
    bool valid;         // this lane's tile exists
    __device__ __forceinline__ uint32_t off(uint32_t r) const { return lane_off + r * width; }
};

}  // namespace

// One wave's 32 tiles (kQMode, kRecon: as roundtrip_duo_kernel).  kRun:
// every wave's 32 tiles are one run of a tile row (tiles_x a multiple of 32),
// all valid; the coefficient rows are re-staged for 1 KiB-contiguous stores.
// Otherwise (ragged widths) per-lane validity and 32-B row stores.  Two
// kernels, not a branch per wave: a runtime branch around the staging costs
// the whole body ~16 VGPRs (94 against 78).
template <bool kStats, int kQMode, int kRecon, bool kRun>
__device__ __forceinline__ void rt_duo_body(const uint8_t* __restrict__ img, float* __restrict__ coef,
                                            uint8_t* __restrict__ recon, const DuoAddr& a, uint32_t h,
                                            const float (&tab)[2][64], float4* __restrict__ slots, float& acc_f,
                                            uint32_t& acc_xx, uint32_t& acc_xr, uint32_t& acc_rr) {
    constexpr bool kNT = true;
    const TSource<true, true> T(nullptr);  // built-in T, zero terms skipped (finite operands)
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* const src = img + a.base;

    // ---- load rows 2k+h (kept for the sums: the inverse ends on the same rows)
    uint2 raw[4];
    unroll<4>([&](auto k) {
        raw[k] = make_uint2(0u, 0u);
        if (kRun || a.valid) raw[k] = *reinterpret_cast<const uint2*>(src + a.off(2u * k + h));
    });
    // ---- columns 4h..4h+3: row 2k in lo[k], row 2k+1 in hi[k] (bytes ^ 0x80)
    uint32_t lo[4], hi[4];
    unroll<4>([&](auto k) {
        lo[k] = raw[k].x ^ 0x80808080u, hi[k] = raw[k].y ^ 0x80808080u;
        xswap(lo[k], hi[k]);
    });
    // ---- forward pass 1: P[v][c], chain over the rows i (T[v][i])
    float pa[4][4], pb[4][4];  // P rows 2k (pa) and 2k+1 (pb), columns c of this lane's half
    unroll<4>([&](auto c) {
        float x[8];
        unroll<4>([&](auto k) {
            x[2 * k] = px_minus128(lo[k], c);
            x[2 * k + 1] = px_minus128(hi[k], c);
        });
        unroll<8>([&](auto v) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(x[i], s); });
            if constexpr (v % 2 == 0) {
                pa[v / 2][c] = s;
            } else {
                pb[v / 2][c] = s;
            }
        });
    });
    // ---- rows: lane h holds row 2k+h of P, columns 0..3 in pa[k], 4..7 in pb[k]
    unroll<4>([&](auto k) { unroll<4>([&](auto c) { xswap(pa[k][c], pb[k][c]); }); });

    // ---- forward pass 2, quantiser, coefficient rows, D = q * Q
    float da[4][4], db[4][4];  // D row 2k+h: columns 0..3 (da), 4..7 (db)
    unroll<4>([&](auto k) {
        const uint32_t row = 2u * k + h;
        const float4* const qrow = reinterpret_cast<const float4*>(&tab[0][row * 8u]);
        const float4* const rrow = reinterpret_cast<const float4*>(&tab[1][row * 8u]);
        const float4 q0 = qrow[0], q1 = qrow[1], r0 = rrow[0], r1 = rrow[1];
        const float qv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const float rv[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        const float prow[8] = {pa[k][0], pa[k][1], pa[k][2], pa[k][3], pb[k][0], pb[k][1], pb[k][2], pb[k][3]};
        float c[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(prow[i], s); });
            constexpr int pl = 2 * k * 8 + u, ph = (2 * k + 1) * 8 + u;
            constexpr int fl = quantforms::jpeg_form(pl), fh = quantforms::jpeg_form(ph);
            if constexpr (kQMode == 2 && fl != quantforms::kFull && fh != quantforms::kFull) {
                float m;
                if constexpr (fl == fh) {
                    m = quantforms::jpeg_bias(pl);
                } else {
                    m = h ? quantforms::jpeg_bias(ph) : quantforms::jpeg_bias(pl);
                }
                c[u] = __builtin_truncf(__builtin_fmaf(s, rv[u], signed_mag(m, s)));
            } else {
                const float q0v = s * rv[u];
                const float e = __builtin_fmaf(-q0v, qv[u], s);
                const float d = __builtin_fmaf(e, rv[u], q0v);
                c[u] = __builtin_truncf(d + signed_half(d));
            }
        });
        // coefficient row 2k+h
        if constexpr (kRun) {
            float4* const slot = slots + (k & 1) * 128;
            slot[2u * lane] = make_float4(c[0], c[1], c[2], c[3]);
            slot[2u * lane + 1u] = make_float4(c[4], c[5], c[6], c[7]);
            const float4 lo4 = slot[lane], hi4 = slot[64u + lane];
            // [0, 1 KiB): row 2k of the 32 tiles; [1 KiB, 2 KiB): row 2k+1
            float* const dst = coef + a.base;
            st<kNT>(reinterpret_cast<float4*>(dst + (2u * k * a.width + 4u * lane)), lo4);
            st<kNT>(reinterpret_cast<float4*>(dst + ((2u * k + 1u) * a.width + 4u * lane)), hi4);
        } else {
            if (a.valid) store_row<kNT>(coef + a.base + a.off(row), c);
        }
        unroll<4>([&](auto u) {
            da[k][u] = c[u] * qv[u];
            db[k][u] = c[4 + u] * qv[4 + u];
        });
    });
    // ---- columns 4h..4h+3 of D: row 2k in da[k], row 2k+1 in db[k]
    unroll<4>([&](auto k) { unroll<4>([&](auto c) { xswap(da[k][c], db[k][c]); }); });
    // ---- inverse pass 1: P[v][c] = chain_i T[i][v] D[i][c]
    unroll<4>([&](auto c) {
        float d[8];
        unroll<4>([&](auto k) { d[2 * k] = da[k][c], d[2 * k + 1] = db[k][c]; });
        unroll<8>([&](auto v) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + v>(d[i], s); });
            if constexpr (v % 2 == 0) {
                pa[v / 2][c] = s;
            } else {
                pb[v / 2][c] = s;
            }
        });
    });
    unroll<4>([&](auto k) { unroll<4>([&](auto c) { xswap(pa[k][c], pb[k][c]); }); });
    // ---- inverse pass 2: R[v][u] = chain_i P[v][i] T[i][u], + 128, uint8, sums
    float chain = 0.0f;  // lanes 0..31: the tile's sse_f32 chain so far (rows < 2k)
    unroll<4>([&](auto k) {
        const float prow[8] = {pa[k][0], pa[k][1], pa[k][2], pa[k][3], pb[k][0], pb[k][1], pb[k][2], pb[k][3]};
        float r[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + u>(prow[i], s); });
            r[u] = s + 128.0f;  // add_matrix_scalar (utils_kernels.cu:29)
        });
        const uint2 r8 = make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
        if constexpr (kStats) {
            const uint2 w = raw[k];
            acc_xx = __builtin_amdgcn_udot4(w.x, w.x, acc_xx, false);
            acc_xx = __builtin_amdgcn_udot4(w.y, w.y, acc_xx, false);
            acc_xr = __builtin_amdgcn_udot4(w.x, r8.x, acc_xr, false);
            acc_xr = __builtin_amdgcn_udot4(w.y, r8.y, acc_xr, false);
            acc_rr = __builtin_amdgcn_udot4(r8.x, r8.x, acc_rr, false);
            acc_rr = __builtin_amdgcn_udot4(r8.y, r8.y, acc_rr, false);
            float e[8];
            unroll<8>([&](auto u) { e[u] = byte_f32(u < 4 ? w.x : w.y, u & 3) - r[u]; });
            // row 2k continues the chain in lanes 0..31; its sum moves to
            // lanes 32..63 for row 2k+1, whose sum comes back for row 2k+2
            float s = chain;
            unroll<8>([&](auto u) { s = __builtin_fmaf(e[u], e[u], s); });
            float to_hi = s, keep = s;
            xswap(to_hi, keep);  // lanes 32..63: to_hi = lane - 32's s
            float s2 = to_hi;
            unroll<8>([&](auto u) { s2 = __builtin_fmaf(e[u], e[u], s2); });
            float back = s2, to_lo = s2;
            xswap(back, to_lo);  // lanes 0..31: to_lo = lane + 32's s2
            chain = to_lo;
        }
        if constexpr (kRecon == kRtReconU8) {
            if (kRun || a.valid) st<kNT>(reinterpret_cast<uint2*>(recon + a.base + a.off(2u * k + h)), r8);
        }
    });
    if constexpr (kStats) {
        // lanes 0..31 hold the tile's full chain; a tile is counted once
        acc_f = (h == 0u && (kRun || a.valid)) ? chain : 0.0f;
        if (!(kRun || a.valid)) acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    }
}

// kQMode 1: the verified 3-op quotient at every position; 2: the default JPEG
// table's short forms where both of an instruction's positions have one.
// kRecon: kRtReconU8 or kRtReconNone.  kWaves: waves per SIMD the register
// allocation must allow.
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
                                               const float (&tab)[2][64], float4* __restrict__ slots, float& acc_f,
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
    float chain = 0.0f;
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
        if constexpr (kStats) {
            const uint2 w = raw[k];
            acc_xx = __builtin_amdgcn_udot4(w.x, w.x, acc_xx, false);
            acc_xx = __builtin_amdgcn_udot4(w.y, w.y, acc_xx, false);
            acc_xr = __builtin_amdgcn_udot4(w.x, r8.x, acc_xr, false);
            acc_xr = __builtin_amdgcn_udot4(w.y, r8.y, acc_xr, false);
            acc_rr = __builtin_amdgcn_udot4(r8.x, r8.x, acc_rr, false);
            acc_rr = __builtin_amdgcn_udot4(r8.y, r8.y, acc_rr, false);
            float e[8];
            unroll<8>([&](auto u) { e[u] = byte_f32(u < 4 ? w.x : w.y, u & 3) - r[u]; });
            float s = chain;
            unroll<8>([&](auto u) { s = __builtin_fmaf(e[u], e[u], s); });
            float to_hi = s, keep = s;
            xswap(to_hi, keep);
            float s2 = to_hi;
            unroll<8>([&](auto u) { s2 = __builtin_fmaf(e[u], e[u], s2); });
            float back = s2, to_lo = s2;
            xswap(back, to_lo);
            chain = to_lo;
        }
        if constexpr (kRecon == kRtReconU8) {
            if (kRun || a.valid) st<kNT>(reinterpret_cast<uint2*>(recon + a.base + a.off(2u * k + h)), r8);
        }
    });
    if constexpr (kStats) {
        acc_f = (h == 0u && (kRun || a.valid)) ? chain : 0.0f;
        if (!(kRun || a.valid)) acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    }
}

// Sums epilogue.  One 64-bit atomic add per field per workgroup into ONE
// struct serialises once the workgroups are many: 8192^2 in 256-thread duo
// workgroups (8,192 of them) took 117.5 us against 66.9 without sums, in
// 64-thread workgroups 406 us (tools/kb_rt, profiles/r05/).  So workgroup b
// adds into sub-slot b % kRtSpread of a spread slot (kRtSpread lines of
// 256 B), and rt_spread_finish_kernel folds the sub-slots into the caller's
// struct and zeroes them.  kSpread: 0 one struct, > 0 spread sub-slots,
// -1 (A/B only) a plain store per workgroup, no atomics.
constexpr int kRtSpread = 64;
constexpr uint32_t kRtSpreadStride = 32;  // u64 words between sub-slots (256 B)

template <bool kStats, int kQMode, int kRecon, bool kRun, int kBlockT = 256, int kWaves = 6, int kSpread = kRtSpread,
          bool kPk = false>
__global__ __launch_bounds__(kBlockT) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void roundtrip_duo_kernel(
    const uint8_t* __restrict__ img, float* __restrict__ coef, uint8_t* __restrict__ recon, RtSums* __restrict__ sums,
    TileGrid g, QParams qp) {
    static_assert(kQMode == 1 || kQMode == 2, "duo round trip: verified quotient only");
    static_assert(kRecon == kRtReconU8 || kRecon == kRtReconNone, "duo round trip: uint8 reconstruction");
    constexpr uint32_t kW = kBlockT / 64u;

    // Q and RN(1/Q) for per-lane reads (the lanes of one instruction use rows 2k and 2k+1)
    __shared__ __attribute__((aligned(16))) float tab[2][64];
    __shared__ __attribute__((aligned(16))) float4 stage[kW][2][128];  // coefficient re-staging, 2 x 2 KiB per wave
    if (threadIdx.x < 64u) tab[0][threadIdx.x] = qp.q.v[threadIdx.x], tab[1][threadIdx.x] = qp.r.v[threadIdx.x];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u, t = lane & 31u, h = lane >> 5;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kW + wv);
    const uint32_t first = wave * kRtDuoTiles;
    float acc_f = 0.0f;
    uint32_t acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;

    if (first < g.ntiles) {
        float4* const slots = stage[wv][0];
        const uint32_t by = first / g.tiles_x, bx = first - by * g.tiles_x;
        const uint32_t w32 = static_cast<uint32_t>(g.width);
        uint32_t lane_off = t * 8u;  // kRun: the tiles of one tile row
        if constexpr (!kRun) {
            const uint32_t tile = first + t, ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
            lane_off = (ty - by) * 8u * w32 + tx * 8u - bx * 8u;
        }
        const DuoAddr a{static_cast<uint64_t>(by) * 8u * g.width + static_cast<uint64_t>(bx) * 8u, lane_off, w32,
                        first + t < g.ntiles};
        if constexpr (kPk) {
            rt_duo_body_pk<kStats, kQMode, kRecon, kRun>(img, coef, recon, a, h, tab, slots, acc_f, acc_xx, acc_xr,
                                                         acc_rr);
        } else {
            rt_duo_body<kStats, kQMode, kRecon, kRun>(img, coef, recon, a, h, tab, slots, acc_f, acc_xx, acc_xr,
                                                      acc_rr);
        }
    }

    if constexpr (kStats && kSpread == -2) {  // A/B: the sums computed, no reduction (kept alive)
        if ((acc_xx ^ acc_rr ^ acc_xr ^ __float_as_uint(acc_f)) == 0x9e3779b9u)
            reinterpret_cast<unsigned long long*>(sums)[threadIdx.x] = 1ull;
    } else if constexpr (kStats && (kSpread == -3 || kSpread == -4)) {
        // per-wave: wave sums, lane 0 adds into sub-slot (wave % kRtSpread); no LDS, no barrier
        const float fx = __builtin_rintf(acc_f * kRtFixScale);
        const bool f_ok = fx < 0x1p40f;  // false for NaN
        unsigned long long f = f_ok ? static_cast<unsigned long long>(fx) : 0ull;
        unsigned long long e8, xx;
        if constexpr (kSpread == -4) {
            f = wave_sum_dpp(f);
            e8 = wave_sum_dpp(acc_xx + acc_rr - 2u * acc_xr), xx = wave_sum_dpp(acc_xx);
        } else {
            f = wave_sum_u64(f);
            e8 = wave_sum_u64(acc_xx + acc_rr - 2u * acc_xr), xx = wave_sum_u64(acc_xx);
        }
        const bool bad = __builtin_amdgcn_ballot_w64(!f_ok) != 0;
        if (lane == 0u) {
            auto* const dst = reinterpret_cast<unsigned long long*>(sums) + (wave % kRtSpread) * kRtSpreadStride;
            if (f) atomicAdd(dst, f);
            if (bad) atomicOr(dst, kRtSseF32Invalid);
            if (e8) atomicAdd(dst + 1, e8);
            if (xx) atomicAdd(dst + 2, xx);
        }
    } else if constexpr (kStats) {
        const float fx = __builtin_rintf(acc_f * kRtFixScale);
        const bool f_ok = fx < 0x1p40f;  // false for NaN
        unsigned long long f = f_ok ? static_cast<unsigned long long>(fx) : 0ull;
        unsigned long long e8 = static_cast<unsigned long long>(acc_xx + acc_rr - 2u * acc_xr);
        unsigned long long xx = static_cast<unsigned long long>(acc_xx);
        f = wave_sum_u64(f), e8 = wave_sum_u64(e8), xx = wave_sum_u64(xx);
        if (__builtin_amdgcn_ballot_w64(!f_ok) != 0) f |= kRtSseF32Invalid;
        __shared__ unsigned long long part[kW][3];
        if (lane == 0u) part[wv][0] = f, part[wv][1] = e8, part[wv][2] = xx;
        __syncthreads();
        if (threadIdx.x < 3u) {
            unsigned long long s = 0, bad = 0;
            for (uint32_t k = 0; k < kW; ++k) {
                s += part[k][threadIdx.x] & ~kRtSseF32Invalid;
                bad |= part[k][threadIdx.x] & kRtSseF32Invalid;
            }
            auto* const words = reinterpret_cast<unsigned long long*>(sums);
            if constexpr (kSpread < 0) {
                words[blockIdx.x * 4u + threadIdx.x] = s | bad;
            } else {
                auto* const dst = words + (kSpread > 0 ? (blockIdx.x % kSpread) * kRtSpreadStride : 0u) + threadIdx.x;
                if (s) atomicAdd(dst, s);
                if (bad) atomicOr(dst, kRtSseF32Invalid);
            }
        }
    }
}

// Folds the kRtSpread sub-slots of a spread slot into *dst (overwriting it,
// or adding to it when accumulate) and zeroes them: one wave, lane i reads
// sub-slot i.
__global__ __launch_bounds__(64) void rt_spread_finish_kernel(RtSums* __restrict__ dst,
                                                              unsigned long long* __restrict__ slot, int accumulate) {
    static_assert(kRtSpread <= 64, "one wave folds the sub-slots");
    const uint32_t l = threadIdx.x;
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    if (l < static_cast<uint32_t>(kRtSpread)) {
        unroll<3>([&](auto f) {
            v[f] = slot[l * kRtSpreadStride + f];
            slot[l * kRtSpreadStride + f] = 0ull;
        });
    }
    unroll<3>([&](auto f) {
        const unsigned long long sum = wave_sum_u64(v[f] & ~kRtSseF32Invalid);
        const bool bad = __builtin_amdgcn_ballot_w64((v[f] & kRtSseF32Invalid) != 0ull) != 0ull;
        if (l == 0u) {
            auto* const d = reinterpret_cast<unsigned long long*>(dst) + f;
            unsigned long long out = accumulate ? *d + sum : sum;
            if (bad) out |= kRtSseF32Invalid;
            *d = out;
        }
    });
}

inline dim3 roundtrip_duo_grid(const TileGrid& g, uint32_t block = 256) {
    const uint32_t waves = (g.ntiles + kRtDuoTiles - 1u) / kRtDuoTiles, per = block / 64u;
    return dim3((waves + per - 1u) / per);
}

}  // namespace hpdct
