// kbench_mfma.hpp -- TOOLS ONLY (tools/kbench2.hip group "mfma"): a measured
// and rejected design, kept for re-measurement.  Bit-exact with the library's
// int8 forward at 8192^2, 2048x16384 and 16384^2, but slower: 41.2-41.9 us
// against 32.6 us per 8192^2 frame (profiles/r02/kbench2_mfma_r02.log,
// kbench2_mfma2_r02.log), also with the groups processed in pairs (4 MFMA
// chains in flight) and a bank-padded exchange.  The 128 MFMAs per set with
// their 40-cycle dependent latency, 64 single-byte LDS reads and the LDS
// exchange per group cost more than the ~400 VALU instructions they remove.
//
// uint8 -> int8 forward DCT + quantisation with the first
// pass of T.X.T^T on the matrix cores (CDNA4 v_mfma_f32_4x4x1_16b_f32) and the
// second pass, the quotient and the byte pack on the VALU.  Same arithmetic as
// every other kernel of the library, bit for bit:
//   * the f32 MFMA of one k-step is D = fma(A, B, C) with one rounding, and a
//     chain of 8 such steps from +0 is the scalar fmaf chain over k = 0..7
//     (tools/mfma_probe.hip: 102,400 single steps and 51,200 8-step chains
//     bit-identical on gfx950, subnormals, signed zeros and huge values
//     included), i.e. P[v][x] = chain_i T[v][i] X'[i][x]  (main_newAppr.cu:193-197);
//     the zero entries of T are multiplied in, fma(0, x, s) = s exactly for
//     finite x and a chain from +0 never holds -0;
//   * C[v][u] = chain_i P[v][i] T[u][i] (main_newAppr.cu:206-209) on the VALU
//     with T in immediates and its zero terms skipped, as in hpdct_tile.hpp;
//   * q = roundf(C / Q) (utils_kernels.cu:42): the verified 3-op quotient where
//     the launcher proved it legal, else IEEE division; round half away folded
//     into the truncating conversion, each value converted into its byte.
//
// Why: the one-lane-per-tile int8 kernel issues ~1,240 VALU instructions per
// 64-tile set (352 of them the first pass) and is VALU-bound (math alone 26.5 us
// against a 25.7 us HBM floor for 2 B/px at 8192^2; profiles/r02).  Here the
// first pass is 128 MFMAs per set on the matrix pipe, which runs beside the
// VALU of the other waves, and the VALU keeps ~830 instructions per set.
//
// Work mapping (one wave = one 64-tile set of one tile row; launched for widths
// that are a multiple of 512 px):
//   1. lane L loads tile L's 8 rows (8 x global_load_dwordx2, 512 B contiguous
//      per instruction) and deposits them, XOR 0x80 per byte, into the wave's
//      4 KiB LDS slot in the frame's own row order;
//   2. the set is processed as 8 groups of 8 tiles.  In group g lane l = 8t + c
//      reads byte (k, 64g + l) for k = 0..7 with a sign-extending LDS load:
//      (int8)(b ^ 0x80) = b - 128 = X'[k][c] of tile 8g + t, exact in fp32;
//   3. MFMA block b = l / 4 = (tile t, column half C): A = X'[k][4C + i] (lane
//      4b + i), B = T[4V + j][k] (lane 4b + j, a per-lane constant), 8 k-steps
//      per V half: D_V (VGPR i, lane 4b + j) = P[4V + j][4C + i];
//   4. D_0, D_1 go through a 2 KiB LDS exchange so that lane l = 8t + r picks up
//      row r = l % 8 of P for its tile (columns 0-3 from lane 8t + j, 4-7 from
//      lane 8t + 4 + j of D_{r / 4});
//   5. the lane runs the 8 second-pass chains of that row, quantises with
//      Q[r][u] (per-lane constants, staged once per workgroup through LDS) and
//      stores the tile row as 8 int8 values (one dwordx2 per lane: the 8 lanes
//      of a row cover 64 contiguous bytes).
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {

typedef float mf32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kMfmaBlock = 256;  // 4 waves = 4 sets per workgroup

template <bool kFast>
__global__ __launch_bounds__(kMfmaBlock, 1) void fdct_mfma_i8_kernel(const uint8_t* __restrict__ img,
                                                                     int8_t* __restrict__ out, TileGrid g,
                                                                     QParams qp) {
    __shared__ float tab[3][64];                          // T, Q, RN(1/Q)
    __shared__ uint2 stage[kMfmaBlock / 64][8][64];       // per wave: 8 rows x 64 tiles x 8 B
    // per wave: D_0, D_1 of a pair of groups; D_1 rows start 4 entries (64 B)
    // later so the row pick-up of 16 lanes spans all 64 banks once
    __shared__ mf32x4 xch[kMfmaBlock / 64][2][2 * 64 + 4];
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        tab[0][tid] = kBuiltinT.v[tid];
        tab[1][tid] = qp.q.v[tid];
        tab[2][tid] = qp.r.v[tid];
    }
    __syncthreads();
    const uint32_t lane = tid & 63u, w = tid >> 6;
    const uint32_t set = __builtin_amdgcn_readfirstlane(blockIdx.x * (kMfmaBlock / 64u) + w);
    if (set * 64u >= g.ntiles) return;

    // per-lane constants: B operands T[4V + j][k] (j = lane % 4), Q / RN(1/Q) of row r = lane % 8
    const uint32_t j = lane & 3u, r = lane & 7u;
    float tb[2][8], qv[8], rv[8];
    unroll<8>([&](auto k) {
        tb[0][k] = tab[0][j * 8u + k];
        tb[1][k] = tab[0][(4u + j) * 8u + k];
        qv[k] = tab[1][r * 8u + k];
        rv[k] = tab[2][r * 8u + k];
    });

    // the set: 64 tiles of tile row ty0 starting at tile column tx0 (tiles_x % 64 == 0)
    const uint32_t t0 = set * 64u;
    const uint32_t ty0 = t0 / g.tiles_x, tx0 = t0 - ty0 * g.tiles_x;
    const uint64_t base = static_cast<uint64_t>(ty0) * 8u * g.width + static_cast<uint64_t>(tx0) * 8u;
    {
        uint2 raw[8];
        unroll<8>([&](auto k) { raw[k] = *reinterpret_cast<const uint2*>(img + base + k * g.width + 8u * lane); });
        unroll<8>([&](auto k) {
            stage[w][k][lane] = make_uint2(raw[k].x ^ 0x80808080u, raw[k].y ^ 0x80808080u);
        });
    }
    const int8_t* sb = reinterpret_cast<const int8_t*>(&stage[w][0][0]);
    const uint32_t t = lane >> 3;
    int8_t* const orow = out + base + static_cast<uint64_t>(r) * g.width + 8u * t;
    const TSource<true, true> T(nullptr);

    // groups in pairs: 4 independent MFMA chains in flight per wave
    unroll<4>([&](auto gp) {
        mf32x4 d[2][2];
        unroll<2>([&](auto h) {
            d[h][0] = mf32x4{0.0f, 0.0f, 0.0f, 0.0f};
            d[h][1] = mf32x4{0.0f, 0.0f, 0.0f, 0.0f};
        });
        // first pass on the matrix cores: P (rows 4V + j, columns 4C + i) of the groups' 8 tiles
        unroll<8>([&](auto k) {
            unroll<2>([&](auto h) {
                constexpr uint32_t grp = 2 * gp + h;
                const float a = static_cast<float>(sb[k * 512u + grp * 64u + lane]);  // X'[k][c] of tile 8g + t
                d[h][0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, tb[0][k], d[h][0], 0, 0, 0);
                d[h][1] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, tb[1][k], d[h][1], 0, 0, 0);
            });
        });
        // lane 8t + r takes row r of P: columns 0-3 from lane 8t + j, 4-7 from lane 8t + 4 + j of D_{r/4}
        unroll<2>([&](auto h) {
            xch[w][h][lane] = d[h][0];
            xch[w][h][64u + 4u + lane] = d[h][1];
        });
        unroll<2>([&](auto h) {
            constexpr uint32_t grp = 2 * gp + h;
            const uint32_t row0 = (r >> 2) * (64u + 4u) + 8u * t + j;
            const mf32x4 lo = xch[w][h][row0];
            const mf32x4 hi = xch[w][h][row0 + 4u];
            float p[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            // second pass, quotient, byte pack: C[r][u] = chain_i P[r][i] T[u][i]
            float c[8];
            unroll<8>([&](auto u) {
                float s = 0.0f;
                unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(p[i], s); });
                c[u] = quotient<kFast ? kVarFastDiv : 0u>(s, qv[u], rv[u]);
            });
            const uint2 wv = make_uint2(pack_q_i8x4(c[0], c[1], c[2], c[3]), pack_q_i8x4(c[4], c[5], c[6], c[7]));
            st<true>(reinterpret_cast<uint2*>(orow + grp * 64u), wv);
        });
    });
}

inline dim3 mfma_grid(const TileGrid& g) {
    const uint32_t sets = (g.ntiles + 63u) / 64u;
    return dim3((sets + kMfmaBlock / 64u - 1u) / (kMfmaBlock / 64u));
}

// eligible: whole 64-tile sets inside one tile row
inline bool mfma_ok(const TileGrid& g) { return g.tiles_x % 64u == 0u && g.ntiles % 64u == 0u; }

template <bool kFast>
hipError_t fdct_mfma_i8_go(const uint8_t* img, int8_t* out, const TileGrid& g, const QParams& q, hipStream_t s) {
    hipLaunchKernelGGL((fdct_mfma_i8_kernel<kFast>), mfma_grid(g), dim3(kMfmaBlock), 0, s, img, out, g, q);
    return hipGetLastError();
}

}  // namespace hpdct
