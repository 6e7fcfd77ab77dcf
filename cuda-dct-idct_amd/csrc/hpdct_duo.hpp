// hpdct_duo.hpp -- the "duo" work mapping for fp32 planes: 2 lanes per tile.
//
// Lane (t, h) = (lane >> 1, lane & 1) of a wave owns columns 4h..4h+3 of tile
// t; a wave owns 32 consecutive tiles.  Row i of the wave's tiles is 256
// consecutive floats, so each of the 8 row loads is ONE dwordx4 instruction
// covering 1 KiB contiguous -- the copy kernel's access pattern -- where the
// tile-per-lane kernel needs two half-dense instructions per row and the
// octet kernel 4-byte loads.
//
//   phase 1  P[v][c] for the lane's 4 columns: the reference's first chain
//            (over rows i, fixed column: main_newAppr.cu:193-197 forward,
//            :236-239 inverse), lane-local.
//   exchange P (and later the output rows) through a wave-private LDS slot,
//            16-byte accesses only.
//   phase 2  lane (t, h) finishes rows 4h..4h+3: the second chain
//            (:206-209 / :246-248), quantise (utils_kernels.cu:42) or +128.
//   store    rows re-staged so that each store instruction writes one row of
//            the wave's 32 tiles: 1 KiB contiguous.
//
// Same chains, division and rounding as every other mapping: bit-identical.
#pragma once

#include "hpdct_octet.hpp"

namespace hpdct {

namespace {

enum : unsigned {
    kDuoTight = 1u << 21,  // unpadded slot (64 floats per tile): 8 KiB per wave, 5 waves/SIMD by LDS
};
constexpr uint32_t kDuoTiles = 32;  // tiles per wave
template <unsigned kVar>
constexpr uint32_t kDuoStride = (kVar & kDuoTight) ? 64u : 72u;  // floats per tile in the slot (64 + pad)

template <unsigned kVar>
__device__ __forceinline__ float* duo_slot() {
    __shared__ __attribute__((aligned(16))) float xchg[kBlock<kVar> / 64u][kDuoTiles * kDuoStride<kVar>];
    return xchg[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
}

__device__ __forceinline__ bool duo_run(const TileGrid& g, uint32_t first_tile) {
    return first_tile + kDuoTiles - 1u < g.ntiles &&
           (first_tile / g.tiles_x) == ((first_tile + kDuoTiles - 1u) / g.tiles_x);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void lds4(float* p, float a, float b, float c, float d) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}

// Second half of both duo kernels: P (x[v][c], the lane's 4 columns of every
// row v) -> LDS -> rows 4h..4h+3 -> finish(row, k, vals[8]) -> staged stores.
template <unsigned kVar, typename Finish>
__device__ __forceinline__ void duo_rows(float (&p)[8][4], float* slot_all, uint32_t t, uint32_t h,
                                         Finish&& finish, float (&o)[4][8]) {
    float* const slot = slot_all + t * kDuoStride<kVar>;
    unroll<8>([&](auto v) { lds4(slot + v * 8u + 4u * h, p[v][0], p[v][1], p[v][2], p[v][3]); });
    wave_lds_order();
    unroll<4>([&](auto k) {
        const uint32_t r = 4u * h + k;
        const float4 a = ld4(slot + r * 8u), b = ld4(slot + r * 8u + 4u);
        float row[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        finish(r, k, row, o[k]);
    });
    wave_lds_order();
}

template <unsigned kVar>
__device__ __forceinline__ void duo_store(float* __restrict__ plane, const TileGrid& g, bool run, uint64_t run_base,
                                          uint64_t base, bool valid, float* slot_all, uint32_t t, uint32_t h,
                                          const float (&o)[4][8]) {
    constexpr bool kNT = (kVar & kVarNT) != 0;
    if (run) {
        const uint32_t lane = threadIdx.x & 63u;
        float* const slot = slot_all + t * kDuoStride<kVar>;
        unroll<4>([&](auto k) {
            const uint32_t r = 4u * h + k;
            lds4(slot + r * 8u, o[k][0], o[k][1], o[k][2], o[k][3]);
            lds4(slot + r * 8u + 4u, o[k][4], o[k][5], o[k][6], o[k][7]);
        });
        wave_lds_order();
        // row k of the 32 tiles: lane l stores floats [4l, 4l+4) = tile l>>1, half l&1
        const float* src = slot_all + (lane >> 1) * kDuoStride<kVar> + 4u * (lane & 1u);
        unroll<8>([&](auto k) {
            st<kNT>(reinterpret_cast<float4*>(plane + run_base + k * g.width) + lane, ld4(src + k * 8u));
        });
        return;
    }
    if (valid) {
        unroll<4>([&](auto k) {
            float4* dst = reinterpret_cast<float4*>(plane + base + (4u * h + k) * g.width);
            st<kNT>(dst, make_float4(o[k][0], o[k][1], o[k][2], o[k][3]));
            st<kNT>(dst + 1, make_float4(o[k][4], o[k][5], o[k][6], o[k][7]));
        });
    }
}

}  // namespace

// Forward, duo mapping, fp32 image -> fp32 coefficients.  Arguments as fdct_kernel.
template <bool kQuant, bool kBuiltinT, bool kWriteback, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>) void fdct_duo_kernel(const float* __restrict__ img, float* __restrict__ out,
                                                                float* __restrict__ shifted, TileGrid g,
                                                                const float* __restrict__ t_dev, QParams qp,
                                                                float shift) {
    const TSource<kBuiltinT, false> T(t_dev);
    const uint32_t lane = threadIdx.x & 63u, t = lane >> 1, h = lane & 1u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
    const uint32_t first = wave * kDuoTiles;
    if (first >= g.ntiles) return;
    const OctetPos p = octet_pos(g, first + t);
    const bool run = duo_run(g, first);
    const uint64_t run_base = octet_pos(g, first).base;
    float* const slot_all = duo_slot<kVar>();

    // phase 1: columns 4h..4h+3, level shift (sub_matrix_scalar, utils_kernels.cu:16)
    float x[8][4];
    unroll<8>([&](auto i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.valid) v = ld4(img + p.base + i * g.width + 4u * h);
        x[i][0] = v.x - shift, x[i][1] = v.y - shift, x[i][2] = v.z - shift, x[i][3] = v.w - shift;
    });
    if constexpr (kWriteback) {  // X - 128 left in the caller's image (main_newAppr.cu:273)
        if (p.valid)
            unroll<8>([&](auto i) {
                *reinterpret_cast<float4*>(shifted + p.base + i * g.width + 4u * h) =
                    make_float4(x[i][0], x[i][1], x[i][2], x[i][3]);
            });
    }
    float pp[8][4];
    unroll<8>([&](auto v) {
        unroll<4>([&](auto c) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(x[i][c], s); });
            pp[v][c] = s;
        });
    });
    float o[4][8];
    duo_rows<kVar>(pp, slot_all, t, h, [&](uint32_t, auto k, const float (&row)[8], float (&dst)[8]) {
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(row[i], s); });
            dst[u] = s;
        });
        if constexpr (kQuant) {  // row 4h+k of Q: two kernel-argument values, one select
            unroll<8>([&](auto u) {
                const float qv = h ? qp.q.v[(4 + k) * 8 + u] : qp.q.v[k * 8 + u];
                dst[u] = quantise<kVar>(dst[u], qv, 0.0f);
            });
        }
    }, o);
    duo_store<kVar>(out, g, run, run_base, p.base, p.valid, slot_all, t, h, o);
}

// Inverse, duo mapping, fp32 coefficients -> fp32 pixels.  Arguments as idct_kernel.
template <bool kDequant, bool kBuiltinT, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>) void idct_duo_kernel(const float* __restrict__ coef, float* __restrict__ out,
                                                                float* __restrict__ dq_out, TileGrid g,
                                                                const float* __restrict__ t_dev, Mat64 q,
                                                                float shift) {
    const TSource<kBuiltinT, false> T(t_dev);
    const uint32_t lane = threadIdx.x & 63u, t = lane >> 1, h = lane & 1u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
    const uint32_t first = wave * kDuoTiles;
    if (first >= g.ntiles) return;
    const OctetPos p = octet_pos(g, first + t);
    const bool run = duo_run(g, first);
    const uint64_t run_base = octet_pos(g, first).base;
    float* const slot_all = duo_slot<kVar>();

    // phase 1: D = q * Q (multiply_matrices, utils_kernels.cu:55), columns 4h..4h+3
    float d[8][4];
    unroll<8>([&](auto i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.valid) v = ld4(coef + p.base + i * g.width + 4u * h);
        d[i][0] = v.x, d[i][1] = v.y, d[i][2] = v.z, d[i][3] = v.w;
        if constexpr (kDequant) {  // columns 4h..4h+3 of Q row i: one select per value
            unroll<4>([&](auto c) { d[i][c] = d[i][c] * (h ? q.v[i * 8 + 4 + c] : q.v[i * 8 + c]); });
        }
    });
    if constexpr (kDequant && (kVar & kVarWbDequant) != 0) {
        if (p.valid)
            unroll<8>([&](auto i) {
                *reinterpret_cast<float4*>(dq_out + p.base + i * g.width + 4u * h) =
                    make_float4(d[i][0], d[i][1], d[i][2], d[i][3]);
            });
    }
    float pp[8][4];
    unroll<8>([&](auto v) {
        unroll<4>([&](auto c) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + v>(d[i][c], s); });
            pp[v][c] = s;
        });
    });
    float o[4][8];
    duo_rows<kVar>(pp, slot_all, t, h, [&](uint32_t, auto, const float (&row)[8], float (&dst)[8]) {
        unroll<8>([&](auto u) {
            float s = 0.0f;
            unroll<8>([&](auto i) { s = T.template mac<i * 8 + u>(row[i], s); });
            dst[u] = s + shift;  // add_matrix_scalar (utils_kernels.cu:29), no clamp
        });
    }, o);
    duo_store<kVar>(out, g, run, run_base, p.base, p.valid, slot_all, t, h, o);
}

inline dim3 duo_grid(const TileGrid& g, uint32_t block) {
    const uint32_t waves = (g.ntiles + kDuoTiles - 1u) / kDuoTiles;
    const uint32_t per = block / 64u;
    return dim3((waves + per - 1u) / per);
}

}  // namespace hpdct
