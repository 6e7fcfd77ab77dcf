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
// sse_f32 is the tile kernel's: four fp32 chains per tile, one per (row
// parity, column parity) class in row-major order (hpdct_roundtrip.hpp).  A
// lane owns rows of one parity (2k + h), so it keeps two of them, even and odd
// columns in the halves of one packed register: no cross-lane hand-off.
#pragma once

#include "hpdct_octet.hpp"
#include "hpdct_residency.hpp"
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

// sse_f32 of one chain in fixed point (rt_sse_fix), added to the lane's
// 32-bit halves split at 2^22: fx = hi * 2^22 + lo exactly (fx is an integer
// below 2^40, hi = floor(fx / 2^22) < 2^18, lo = fx - hi * 2^22 < 2^22 by
// one exact fma).  Over a wave (64 lanes, 2 chains, <= 8 runs) both sums
// stay below 2^32.
__device__ __forceinline__ void rt_sse_split(float chain, bool& ok, uint32_t& hi, uint32_t& lo) {
    const float fx = __builtin_rintf(chain * kRtFixScale);
    const bool good = fx < 0x1p40f;  // false for NaN
    ok = ok && good;
    const float h = __builtin_floorf(fx * 0x1p-22f);
    const float l = __builtin_fmaf(-h, 0x1p22f, fx);
    hi += good ? static_cast<uint32_t>(h) : 0u;
    lo += good ? static_cast<uint32_t>(l) : 0u;
}

}  // namespace

// The quality sums of one reconstructed row (8 pixels) of a lane: the exact
// integer sums on the packed bytes (v_dot4_u32_u8: x.x, x.r8, r8.r8) and the
// row's terms of the lane's two sse_f32 chains, (x - r)^2 for the even
// columns into acc_f2.x and the odd ones into acc_f2.y, in column order (one
// v_pk_add_f32 and one v_pk_fma_f32 per column pair).  With the rows a lane
// owns (2k + h, in order), its two chains are the (row parity h, column
// parity) classes of the tile's sse_f32 definition (hpdct_roundtrip.hpp).
__device__ __forceinline__ void rt_duo_row_sums(uint2 w, const float (&r)[8], uint2 r8, f32x2& acc_f2,
                                                uint32_t& acc_xx, uint32_t& acc_xr, uint32_t& acc_rr) {
    acc_xx = __builtin_amdgcn_udot4(w.x, w.x, acc_xx, false);
    acc_xx = __builtin_amdgcn_udot4(w.y, w.y, acc_xx, false);
    acc_xr = __builtin_amdgcn_udot4(w.x, r8.x, acc_xr, false);
    acc_xr = __builtin_amdgcn_udot4(w.y, r8.y, acc_xr, false);
    acc_rr = __builtin_amdgcn_udot4(r8.x, r8.x, acc_rr, false);
    acc_rr = __builtin_amdgcn_udot4(r8.y, r8.y, acc_rr, false);
    unroll<4>([&](auto j) {
        const uint32_t word = j < 2 ? w.x : w.y;
        const f32x2 x2 = {byte_f32(word, (2 * j) & 3), byte_f32(word, (2 * j + 1) & 3)};
        const f32x2 e2 = x2 - f32x2{r[2 * j], r[2 * j + 1]};
        acc_f2 = fma2(e2, e2, acc_f2);
    });
}

// One wave's 32 tiles (kQMode, kRecon: as roundtrip_duo_kernel).  kRun:
// every wave's 32 tiles are one run of a tile row (tiles_x a multiple of 32),
// all valid; the coefficient rows are re-staged for 1 KiB-contiguous stores.
// Otherwise (ragged widths) per-lane validity and 32-B row stores.  Two
// kernels, not a branch per wave: a runtime branch around the staging costs
// the whole body ~16 VGPRs (94 against 78).
// TC: the coefficient plane's type, float (the reference's) or int8_t (the
// wire format; forward only: no reconstruction, no sums).
template <bool kStats, int kQMode, int kRecon, bool kRun, typename TC = float>
__device__ __forceinline__ void rt_duo_body(const uint8_t* __restrict__ img, TC* __restrict__ coef,
                                            void* __restrict__ recon, const DuoAddr& a, uint32_t h,
                                            const float (&tab)[2][64], float4* __restrict__ slots, f32x2& acc_f2,
                                            uint32_t& acc_xx, uint32_t& acc_xr, uint32_t& acc_rr) {
    constexpr bool kNT = true;
    constexpr bool kI8 = std::is_same_v<TC, int8_t>;
    // int8 coefficients hold the quantiser's values before the final trunc (the
    // truncating convert does it), so D below is only right for fp32: the int8
    // kernel must be forward only (the compiler then drops the inverse)
    static_assert(!kI8 || (kRecon == kRtReconNone && !kStats), "int8 coefficients: forward only");
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
                const float b = __builtin_fmaf(s, rv[u], signed_mag(m, s));
                c[u] = kI8 ? b : __builtin_truncf(b);
            } else {
                const float q0v = s * rv[u];
                const float e = __builtin_fmaf(-q0v, qv[u], s);
                const float d = __builtin_fmaf(e, rv[u], q0v);
                const float b = d + signed_half(d);
                c[u] = kI8 ? b : __builtin_truncf(b);
            }
        });
        // coefficient row 2k+h
        if constexpr (kI8) {
            // the truncating convert straight into each byte; 8 B per lane: the
            // wave's rows 2k and 2k+1 of its 32 tiles, two 256-B runs
            const uint2 w = make_uint2(pack_biased_i8x4(c[0], c[1], c[2], c[3]), pack_biased_i8x4(c[4], c[5], c[6], c[7]));
            if (kRun || a.valid) st<kNT>(reinterpret_cast<uint2*>(coef + a.base + a.off(row)), w);
        } else if constexpr (kRun) {
            float4* const slot = slots + (k & 1) * 128;
            slot[2u * lane] = make_float4(c[0], c[1], c[2], c[3]);
            slot[2u * lane + 1u] = make_float4(c[4], c[5], c[6], c[7]);
            const float4 lo4 = slot[lane], hi4 = slot[64u + lane];
            // [0, 1 KiB): row 2k of the 32 tiles; [1 KiB, 2 KiB): row 2k+1
            // byte offsets in 32 bits (< 32 * width bytes from the wave's
            // base), so both stores take the SGPR-base + VGPR-offset form
            char* const dst = reinterpret_cast<char*>(coef + a.base);
            const uint32_t o_lo = (2u * k * a.width + 4u * lane) * 4u, o_hi = o_lo + a.width * 4u;
            st<kNT>(reinterpret_cast<float4*>(dst + o_lo), lo4);
            st<kNT>(reinterpret_cast<float4*>(dst + o_hi), hi4);
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
    unroll<4>([&](auto k) {
        const float prow[8] = {pa[k][0], pa[k][1], pa[k][2], pa[k][3], pb[k][0], pb[k][1], pb[k][2], pb[k][3]};
        float r[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + u>(prow[i], s); });
            r[u] = s + 128.0f;  // add_matrix_scalar (utils_kernels.cu:29)
        });
        const uint2 r8 = make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
        if constexpr (kStats) rt_duo_row_sums(raw[k], r, r8, acc_f2, acc_xx, acc_xr, acc_rr);
        if constexpr (kRecon == kRtReconU8) {
            if (kRun || a.valid)
                st<kNT>(reinterpret_cast<uint2*>(static_cast<uint8_t*>(recon) + a.base + a.off(2u * k + h)), r8);
        } else if constexpr (kRecon == kRtReconF32) {
            // fp32 R + 128 (the reference's float output), re-staged like the
            // coefficient rows: 1 KiB contiguous per store instruction
            if constexpr (kRun) {
                float4* const slot = slots + (k & 1) * 128;
                slot[2u * lane] = make_float4(r[0], r[1], r[2], r[3]);
                slot[2u * lane + 1u] = make_float4(r[4], r[5], r[6], r[7]);
                const float4 lo4 = slot[lane], hi4 = slot[64u + lane];
                char* const dst = reinterpret_cast<char*>(static_cast<float*>(recon) + a.base);
                const uint32_t o_lo = (2u * k * a.width + 4u * lane) * 4u, o_hi = o_lo + a.width * 4u;
                st<kNT>(reinterpret_cast<float4*>(dst + o_lo), lo4);
                st<kNT>(reinterpret_cast<float4*>(dst + o_hi), hi4);
            } else {
                if (a.valid) store_row<kNT>(static_cast<float*>(recon) + a.base + a.off(2u * k + h), r);
            }
        }
    });
    if constexpr (kStats) {
        if (!(kRun || a.valid)) acc_f2 = f32x2{0.0f, 0.0f}, acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;
    }
}

// kQMode 1: the verified 3-op quotient at every position; 2: the default JPEG
// table's short forms where both of an instruction's positions have one.
// kRecon: kRtReconU8, kRtReconF32 or kRtReconNone.  kWaves: waves per SIMD the register
// allocation must allow.
// Sums epilogue.  One 64-bit atomic add per field per workgroup into ONE
// struct serialises once the workgroups are many: 8192^2 in 256-thread duo
// workgroups (8,192 of them) took 117.5 us against 66.9 without sums, in
// 64-thread workgroups 406 us (tools/kb_rt, profiles/r05/a/).  So each wave
// adds its sums into sub-slot (wave % kRtSpread) of a spread slot (kRtSpread
// lines of 256 B; DPP wave sums keep it free of LDS and of a workgroup
// barrier: 78.6 us against 81.2 with __shfl_xor sums and 80.9 with a
// workgroup reduction, profiles/r05/a/kb_rt_8192_epilogue.log), and
// rt_spread_finish_kernel folds the sub-slots into the caller's struct and
// zeroes them.  Four 32-bit DPP sums instead of two 64-bit ones (sse_f32
// split at 2^22, rt_sse_split): 1,096 VALU per wave instead of 1,163 and
// 73.7-74.0 us against 74.5-75.2 (profiles/r05/f/).

// The sums of one wave after its runs: four 32-bit DPP sums (each add takes
// its DPP operand directly; every one stays below 2^32 over a wave: 32 pixels
// per lane and run, kSets <= 8), wave-uniform; sse_f32 rebuilt as 64 bits.
struct DuoWaveSums {
    unsigned long long fs;  // sse_f32 in fixed point (2^-16)
    uint32_t se, sx;        // sse_u8, sum_x2
    bool bad;               // some chain was non-finite or too large (kRtSseF32Invalid)
};

// The body both round-trip kernels share: the Q tables to LDS, the wave's
// kSets runs of 32 tiles (a grid apart), and the wave's sums (kStats).
// kSets: 32-tile runs per wave.
template <bool kStats, int kQMode, int kRecon, bool kRun, int kBlockT, int kSets, typename TC = float>
__device__ __forceinline__ DuoWaveSums rt_duo_waves(const uint8_t* __restrict__ img, TC* __restrict__ coef,
                                                    void* __restrict__ recon, const TileGrid& g, const QParams& qp,
                                                    uint32_t& wave_out) {
    static_assert(kQMode == 1 || kQMode == 2, "duo round trip: verified quotient only");
    constexpr uint32_t kW = kBlockT / 64u;

    // Q and RN(1/Q) for per-lane reads (the lanes of one instruction use rows 2k and 2k+1)
    __shared__ __attribute__((aligned(16))) float tab[2][64];
    __shared__ __attribute__((aligned(16))) float4 stage[kW][2][128];  // coefficient re-staging, 2 x 2 KiB per wave
    if (threadIdx.x < 64u) tab[0][threadIdx.x] = qp.q.v[threadIdx.x], tab[1][threadIdx.x] = qp.r.v[threadIdx.x];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u, t = lane & 31u, h = lane >> 5;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kW + wv);
    wave_out = wave;
    uint32_t f_hi = 0u, f_lo = 0u;  // this lane's sse_f32 chains in fixed point over its runs, split at 2^22
    bool ok = true;
    uint32_t acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;

    unroll<kSets>([&](auto it) {
        const uint32_t first = (wave + static_cast<uint32_t>(it) * gridDim.x * kW) * kRtDuoTiles;
        if (first >= g.ntiles) return;
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
        f32x2 acc_f2 = {0.0f, 0.0f};  // the run's tile: this lane's two chains
        rt_duo_body<kStats, kQMode, kRecon, kRun, TC>(img, coef, recon, a, h, tab, slots, acc_f2, acc_xx, acc_xr,
                                                      acc_rr);
        if constexpr (kStats) {
            rt_sse_split(acc_f2.x, ok, f_hi, f_lo);
            rt_sse_split(acc_f2.y, ok, f_hi, f_lo);
        }
    });

    DuoWaveSums out{0ull, 0u, 0u, false};
    if constexpr (kStats) {
        static_assert(kSets <= 8, "32-bit wave sums");
        const uint32_t e8 = acc_xx + acc_rr - 2u * acc_xr;
        const uint32_t sh = wave_sum_dpp(f_hi), sl = wave_sum_dpp(f_lo);
        out.sx = wave_sum_dpp(acc_xx), out.se = wave_sum_dpp(e8);
        out.fs = (static_cast<unsigned long long>(sh) << 22) + sl;
        out.bad = __builtin_amdgcn_ballot_w64(!ok) != 0;
    }
    return out;
}

// kSpreadN: sub-slots of the spread slot.  Two more kSpreadN values exist for
// tools/kb_rt's decomposition of the sums' cost only: 0 writes one plain 32-B
// record per wave (no atomics), < 0 computes the sums and skips the atomics
// when sums is null.
template <bool kStats, int kQMode, int kRecon, bool kRun, int kBlockT = 256, int kWaves = 6, int kSets = 1,
          int kSpreadN = kRtSpread>
__global__ __launch_bounds__(kBlockT) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void roundtrip_duo_kernel(
    const uint8_t* __restrict__ img, float* __restrict__ coef, void* __restrict__ recon, RtSums* __restrict__ sums,
    TileGrid g, QParams qp) {
    uint32_t wave;
    const DuoWaveSums w = rt_duo_waves<kStats, kQMode, kRecon, kRun, kBlockT, kSets>(img, coef, recon, g, qp, wave);
    if constexpr (kStats) {
        // lane 0 adds into sub-slot (wave % kSpreadN) of the spread slot: no
        // LDS, no barrier.  Its atomics take a per-lane zero offset, so they
        // stay single atomics (no uniform-address rewrite).
        if ((threadIdx.x & 63u) == 0u && (kSpreadN > 0 || sums)) {
            uint32_t z = 0u;
            asm volatile("" : "+v"(z));
            if constexpr (kSpreadN == 0) {
                auto* const dst = reinterpret_cast<unsigned long long*>(sums) + wave * 4u + z;
                dst[0] = w.bad ? (w.fs | kRtSseF32Invalid) : w.fs, dst[1] = w.se, dst[2] = w.sx;
            } else {
                constexpr uint32_t kN = kSpreadN < 0 ? -kSpreadN : kSpreadN;
                auto* const dst = reinterpret_cast<unsigned long long*>(sums) + (wave % kN) * kRtSpreadStride + z;
                if (w.fs) atomicAdd(dst, w.fs);
                if (w.bad) atomicOr(dst, kRtSseF32Invalid);
                if (w.se) atomicAdd(dst + 1, static_cast<unsigned long long>(w.se));
                if (w.sx) atomicAdd(dst + 2, static_cast<unsigned long long>(w.sx));
            }
        }
    }
}

// The forward alone on the duo mapping (round 6): uint8 frame -> quantised
// fp32 coefficients.  It is the round trip's body without a reconstruction or
// sums, whose inverse the compiler then drops (583 VALU and 20 lane swaps per
// 32-tile wave, 58 VGPRs, against 992 and 52 for the round trip with a uint8
// reconstruction): same loads, chains, quotient forms and re-staged 1 KiB
// stores, so the same bits as the tile kernel's forward.  Launched in
// kDuoFwdBlock-thread workgroups at most kDuoFwdCapWgs resident per CU
// (launch_fdct_duo_u8): 8192^2 53.0 us against 56.1 for the tile kernel at its
// cap, 2048 x 16384 (the C4 8-way slab) 28.4 against 32.8, 2048^2 5.3 against
// 7.8 (octet), 1024^2 equal (tools/kb_rt groups fwdduo / fwdcap,
// profiles/r06/kb_rt_fwdcap_*.log).
// TC int8_t: the int8 wire format, 8 B row stores (no LDS re-staging);
// bit-exact but slower than the int8 tile kernel (8192^2 36.3 against 31.8 us,
// tools/kb_rt group i8duo, profiles/r06/kb_rt_i8duo_*.log), so only the A/B
// harness instantiates it.
template <int kQMode, typename TC = float>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void fdct_duo_u8_kernel(
    const uint8_t* __restrict__ img, TC* __restrict__ coef, TileGrid g, QParams qp) {
    uint32_t wave;
    (void)rt_duo_waves<false, kQMode, kRtReconNone, true, 256, 1, TC>(img, coef, nullptr, g, qp, wave);
}

// The same forward over a list of frames of one shape (hpdct_forward_frames):
// blockIdx.y picks the frame, whose pointers travel in the kernel arguments.
template <int kQMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void fdct_duo_u8_frames_kernel(
    FrameTable<float> ft, TileGrid g, QParams qp) {
    uint32_t wave;
    const uint32_t f = blockIdx.y;
    (void)rt_duo_waves<false, kQMode, kRtReconNone, true, 256, 1>(ft.in[f], ft.out[f], nullptr, g, qp, wave);
}

inline dim3 roundtrip_duo_grid(const TileGrid& g, uint32_t block = 256, uint32_t sets = 1) {
    const uint32_t runs = (g.ntiles + kRtDuoTiles - 1u) / kRtDuoTiles, per = block / 64u;
    const uint32_t waves = (runs + sets - 1u) / sets;
    return dim3((waves + per - 1u) / per);
}

namespace rt_duo_detail {
// 256-thread workgroups, 6 waves per SIMD (74 VGPRs, no spills; 7 and 8
// spill and run slower, tools/kb_rt, profiles/r05/a/).  Whole runs only
// (tiles_x a multiple of 32, launch_roundtrip checks): the kRun = false kernel
// (ragged widths, 92 VGPRs) is slower than the tile kernel there (4096 x 4104:
// 36.9 against 31.9 us with sums, profiles/r05/b/kb_rt_ragged.log).
// Round 6: at most kDuoRtCapWgs workgroups (16 waves) per CU, by the
// dynamic-LDS reservation, for the fp32 reconstruction and for every round
// trip without sums: 8192^2 fp32 reconstruction + sums 100.2-100.3 against
// 106.6-106.7 us uncapped, without sums 98.9 against 102.4; uint8
// reconstruction without sums 67.2 against 68.4 (tools/kb_rt group f32cap,
// profiles/r06/kb_rt_f32cap.log).  The uint8 reconstruction with sums (the C3
// one pass) gains nothing from it (group rtcap) and stays uncapped.
constexpr int kDuoRtBlock = 256, kDuoRtWaves = 6;
constexpr uint32_t kDuoRtCapWgs = 4;
template <bool kStats, int kQMode, int kRecon>
hipError_t go(const uint8_t* img, float* coef, void* recon, unsigned long long* spread, const TileGrid& g,
              const QParams& qp, hipStream_t s) {
    auto* const kern = roundtrip_duo_kernel<kStats, kQMode, kRecon, true, kDuoRtBlock, kDuoRtWaves>;
    size_t dyn = 0;
    if constexpr (kRecon == kRtReconF32 || !kStats) {
        static const size_t st = static_lds_of(kern);
        dyn = residency_cap_lds(st, kDuoRtCapWgs);
    }
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(g, kDuoRtBlock), dim3(kDuoRtBlock), dyn, s, img, coef, recon,
                       reinterpret_cast<RtSums*>(spread), g, qp);
    return hipGetLastError();
}
template <int kRecon>
hipError_t go_r(const uint8_t* img, float* coef, void* recon, unsigned long long* spread, const TileGrid& g,
                const QParams& qp, int qmode, hipStream_t s) {
    if (spread) {
        return qmode == 2 ? go<true, 2, kRecon>(img, coef, recon, spread, g, qp, s)
                          : go<true, 1, kRecon>(img, coef, recon, spread, g, qp, s);
    }
    return qmode == 2 ? go<false, 2, kRecon>(img, coef, recon, nullptr, g, qp, s)
                      : go<false, 1, kRecon>(img, coef, recon, nullptr, g, qp, s);
}
}  // namespace rt_duo_detail

}  // namespace hpdct
