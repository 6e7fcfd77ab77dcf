// hpdct_tile.hpp -- device-side building blocks of the 8x8 block DCT/IDCT
// (HpApprDCT arithmetic) for CDNA4 / gfx950.
//
// Arithmetic contract (must match the reference bit for bit; see
// oracle/hpdct_oracle.c and DESIGN.md "Arithmetic contract"):
//   forward  (main_newAppr.cu:177-211, utils_kernels.cu:8-18,34-44)
//     X' = X - 128                                   fp32 subtract
//     P[v][x] = fma chain over i=0..7 of T[v][i]*X'[i][x], from +0
//     C[v][u] = fma chain over i=0..7 of P[v][i]*T[u][i], from +0
//     q = roundf(C / Q[v][u])                         IEEE division, half away
//   inverse  (utils_kernels.cu:47-57, main_newAppr.cu:220-250, utils_kernels.cu:21-31)
//     D = q * Q[v][u]
//     P[v][x] = fma chain over i of T[i][v]*D[i][x]
//     R[v][u] = fma chain over i of P[v][i]*T[i][u];  out = R + 128
// The whole library is compiled with -ffp-contract=off: every fused
// multiply-add is an explicit __builtin_fmaf, nothing else may fuse.
//
// Zero terms of the built-in T are skipped only where the operand is known
// finite (uint8 pixels, int8 coefficients): a chain that starts at +0 never
// holds -0 under round-to-nearest, so fma(0, x, s) == s for finite x and the
// skip is bit-exact.  fp32 inputs keep every term (an Inf/NaN input must
// poison the same outputs as in the reference).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "hpdct_kernels.h"
#include "hpdct_tables.h"

namespace hpdct {

// ---------------------------------------------------------------------------
// Tables: the built-in T (its entries become instruction immediates) and the
// default Q, both from the one shared copy in hpdct_tables.h
// (main_newAppr.cu:60-81, pinned to the reference's text by the tests).
// ---------------------------------------------------------------------------
constexpr Mat64 mat64_of(const float (&a)[64]) {
    Mat64 m{};
    for (int i = 0; i < 64; ++i) m.v[i] = a[i];
    return m;
}
inline constexpr Mat64 kBuiltinT = mat64_of(tables::kT);
inline constexpr Mat64 kDefaultQ = mat64_of(tables::kQ);

// ---------------------------------------------------------------------------
// Compile-time loop: f(integral_constant<int, I>) for I in [0, N).
// Every tile index below is a template constant, so table lookups and the
// zero-term skips fold away at compile time.
// ---------------------------------------------------------------------------
template <typename F, int... I>
__device__ __forceinline__ void unroll_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void unroll(F&& f) {
    unroll_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------
// Transform source: the built-in matrix (immediates, optional zero skipping)
// or a caller-provided device matrix (64 wave-uniform scalar loads -> SGPRs).
// ---------------------------------------------------------------------------
template <bool kBuiltin, bool kSkipZero>
struct TSource {
    float t[kBuiltin ? 1 : 64];

    __device__ __forceinline__ explicit TSource(const float* __restrict__ dev) {
        if constexpr (!kBuiltin) {
            unroll<64>([&](auto i) { t[i] = dev[i]; });
        } else {
            (void)dev;
        }
    }
    // s + T[IDX] * a, one rounding (the reference's contracted `sums += a*b`)
    template <int IDX>
    __device__ __forceinline__ float mac(float a, float s) const {
        if constexpr (kBuiltin) {
            constexpr float c = kBuiltinT.v[IDX];
            if constexpr (kSkipZero && c == 0.0f) {
                return s;
            } else {
                return __builtin_fmaf(c, a, s);
            }
        } else {
            return __builtin_fmaf(t[IDX], a, s);
        }
    }
};

// Forward tile transform on registers: x[i][j] level-shifted pixels,
// returns P via the column pass, then calls emit(v, c[8]) for each output row
// (so each row can be quantised and stored while the next is computed).
template <typename TS, typename Emit>
__device__ __forceinline__ void fdct_tile(const TS& T, float (&x)[8][8], Emit&& emit) {
    float p[8][8];
    // P = T . X   (main_newAppr.cu:193-197): P[v][col] = sum_i T[v][i] X[i][col]
    unroll<8>([&](auto col) {
        unroll<8>([&](auto v) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(x[i][col], s); });
            p[v][col] = s;
        });
    });
    // C = P . T^T (main_newAppr.cu:206-209): C[v][u] = sum_i P[v][i] T[u][i]
    unroll<8>([&](auto v) {
        float c[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(p[v][i], s); });
            c[u] = s;
        });
        emit(v, c);
    });
}

// Packed-fp32 forward (v_pk_fma_f32: two IEEE fmas per instruction, each half
// rounded exactly like the scalar v_fma_f32; round 3), built-in T, finite
// inputs only (uint8 pixels).  Same chains as fdct_tile: pass 1 pairs the
// columns (x, x+1) of one P row; pass 2 pairs output columns whose zero
// patterns in T coincide, (0,2) (4,6) (1,5) (3,7), so a term that is zero in
// one half only adds fma(0, P, s) = s exactly (P finite, s never -0).
// emit2(v, c2): c2[k] = {C[v][pair_u(k, 0)], C[v][pair_u(k, 1)]}.
typedef float f32x2 __attribute__((ext_vector_type(2)));
// (a function, not a table: indexing a namespace-scope table here made hipcc
// keep the quotient operands in scratch memory)
constexpr int pair_u(int k, int h) {
    return k == 0 ? (h ? 2 : 0) : k == 1 ? (h ? 6 : 4) : k == 2 ? (h ? 5 : 1) : (h ? 7 : 3);
}

__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename Emit2>
__device__ __forceinline__ void fdct_tile_pk(const f32x2 (&x2)[8][4], Emit2&& emit2) {
    f32x2 p2[8][4];
    // P = T . X, two columns per instruction (main_newAppr.cu:193-197)
    unroll<8>([&](auto v) {
        unroll<4>([&](auto cp) {
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float c = kBuiltinT.v[v * 8 + i];
                if constexpr (c != 0.0f) s = fma2(f32x2{c, c}, x2[i][cp], s);
            });
            p2[v][cp] = s;
        });
    });
    // C = P . T^T, two output columns per instruction (main_newAppr.cu:206-209)
    unroll<8>([&](auto v) {
        f32x2 c2[4];
        unroll<4>([&](auto k) {
            constexpr int u0 = pair_u(k, 0), u1 = pair_u(k, 1);
            f32x2 s = {0.0f, 0.0f};
            unroll<8>([&](auto i) {
                constexpr float a = kBuiltinT.v[u0 * 8 + i], b = kBuiltinT.v[u1 * 8 + i];
                if constexpr (a != 0.0f || b != 0.0f) {
                    const float pv = p2[v][i / 2][i % 2];
                    s = fma2(f32x2{a, b}, f32x2{pv, pv}, s);
                }
            });
            c2[k] = s;
        });
        emit2(v, c2);
    });
}

// cublasDCTv2 pass order (main_cublass_2.cu:228-235): R = X.T^T (row pass,
// temp1) first, then C = T.R, each a sequential FMA chain over the 8
// non-trivial terms of the block-diagonal GEMM's k range.
template <typename TS, typename Emit>
__device__ __forceinline__ void fdct_tile_rowfirst(const TS& T, float (&x)[8][8], Emit&& emit) {
    float r[8][8];
    unroll<8>([&](auto i) {
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto j) { s = T.template mac<u * 8 + j>(x[i][j], s); });
            r[i][u] = s;
        });
    });
    unroll<8>([&](auto v) {
        float c[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(r[i][u], s); });
            c[u] = s;
        });
        emit(v, c);
    });
}

// cublasDCTv2 inverse order (main_cublass_2.cu:288-295): R = D.T, then T^T.R.
template <typename TS, typename Emit>
__device__ __forceinline__ void idct_tile_rowfirst(const TS& T, float (&d)[8][8], Emit&& emit) {
    float r[8][8];
    unroll<8>([&](auto i) {
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto j) { s = T.template mac<j * 8 + u>(d[i][j], s); });
            r[i][u] = s;
        });
    });
    unroll<8>([&](auto v) {
        float c[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + v>(r[i][u], s); });
            c[u] = s;
        });
        emit(v, c);
    });
}

// Inverse tile transform: d[i][j] dequantised coefficients.
template <typename TS, typename Emit>
__device__ __forceinline__ void idct_tile(const TS& T, float (&d)[8][8], Emit&& emit) {
    float p[8][8];
    // P = T^T . D (main_newAppr.cu:236-239): P[v][col] = sum_i T[i][v] D[i][col]
    unroll<8>([&](auto col) {
        unroll<8>([&](auto v) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + v>(d[i][col], s); });
            p[v][col] = s;
        });
    });
    // R = P . T (main_newAppr.cu:246-248): R[v][u] = sum_i P[v][i] T[i][u]
    unroll<8>([&](auto v) {
        float r[8];
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + u>(p[v][i], s); });
            r[u] = s;
        });
        emit(v, r);
    });
}

}  // namespace hpdct
