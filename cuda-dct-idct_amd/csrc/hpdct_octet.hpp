// hpdct_octet.hpp -- the "octet" work mapping: 8 lanes per 8x8 tile.
//
// The tile-per-lane kernels (hpdct_kernels_impl.hpp) give each lane a whole
// tile: ideal for the 1-byte-per-pixel input (4 KiB per wave load, 1 KiB
// contiguous stores via LDS), but a wave then owns 64 tiles, so a small frame
// has few, long waves (C2 1024^2 = 256 waves), and the fp32 planes need
// 64 VGPRs of raw tile per lane.  Here a wave owns 8 consecutive tiles:
//
//   phase 1  lane (t, x) = (lane >> 3, lane & 7) holds COLUMN x of tile t.
//            Row i of the 8 tiles is 64 consecutive pixels, so each of the 8
//            loads is one contiguous 64-element run.  The first pass of the
//            reference chains over the rows i for a fixed column -- P = T.X
//            (main_newAppr.cu:193-197), P = T^T.D (:236-239) -- so it is
//            lane-local and keeps the reference's summation order.
//   exchange P goes through a wave-private LDS slot (8 tiles x 72 floats,
//            the pad makes the eight ds_write_b32 conflict-free).
//   phase 2  lane (t, r) holds ROW r of P and runs the second chain,
//            C[r][u] = sum_i P[r][i] T[u][i] (:206-209) or
//            R[r][u] = sum_i P[r][i] T[i][u] (:246-248), then quantises with
//            Q[r][u] (divide_matrices, utils_kernels.cu:42) and stores its
//            output row (8 contiguous values).
//
// Same FMA chains from +0, same IEEE division and roundf as the tile-per-lane
// kernels, hence bit-identical output.  Q / reciprocals are indexed by the
// lane's row, so they are staged once per workgroup in LDS.
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {

enum : unsigned {
    kOctRestage = 1u << 20,  // octet output rows re-staged through LDS: each store instruction writes
                             // four 256-B runs (a whole row of the wave's 8 tiles each) instead of
                             // 16-B pieces at a 32-B stride
};

namespace {

constexpr uint32_t kOctStride = 72;  // floats per tile in the exchange slot

// Lanes of one wave exchanging data through LDS: the hardware executes a
// wave's LDS instructions in order, so only the compiler must not move LDS
// accesses across this point (wave_barrier alone is not a memory barrier in IR).
__device__ __forceinline__ void wave_lds_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

template <unsigned kVar>
__device__ __forceinline__ float* octet_slot() {
    __shared__ __attribute__((aligned(16))) float xchg[kBlock<kVar> / 64u][8 * kOctStride];
    return xchg[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
}

// 64-entry table (+ optional second table) copied to LDS once per workgroup.
template <unsigned kVar, int kTables>
__device__ __forceinline__ const float* stage_tables(const Mat64& a, const Mat64* b) {
    // threads 64..127 stage the second table
    static_assert(kTables == 1 || kBlock<kVar> >= 128, "two tables need workgroups of at least 128 threads");
    __shared__ __attribute__((aligned(16))) float tab[kTables * 64];
    const uint32_t t = threadIdx.x;
    if (t < 64u) tab[t] = a.v[t];
    if constexpr (kTables > 1) {
        if (t >= 64u && t < 128u) tab[t] = b->v[t - 64u];
    }
    __syncthreads();
    return tab;
}

struct OctetPos {
    uint64_t base;  // element index of the tile's top-left pixel
    bool valid;
};

__device__ __forceinline__ OctetPos octet_pos(const TileGrid& g, uint32_t tile) {
    OctetPos p{0, tile < g.ntiles};
    if (p.valid) {
        const uint32_t by = tile / g.tiles_x, bx = tile - by * g.tiles_x;
        p.base = static_cast<uint64_t>(by) * 8u * g.width + static_cast<uint64_t>(bx) * 8u;
    }
    return p;
}

// Whole wave = 8 valid tiles of one tile row: their rows are 64-element runs.
__device__ __forceinline__ bool octet_run(const TileGrid& g, uint32_t first_tile) {
    return first_tile + 7u < g.ntiles && (first_tile / g.tiles_x) == ((first_tile + 7u) / g.tiles_x);
}

// Emit the lane's output row r (8 values) of tile t: straight from the lane,
// or (kOctRestage, whole runs only) via the slot so that instruction h stores
// rows 4h..4h+3 of all 8 tiles, 16 B per lane, 256 B contiguous per row.
template <unsigned kVar, typename TOut>
__device__ __forceinline__ void octet_store(TOut* __restrict__ plane, const TileGrid& g, const OctetPos& p,
                                            uint32_t r, bool run, uint64_t run_base, float* slot_all,
                                            const float (&c)[8]) {
    constexpr bool kNT = (kVar & kVarNT) != 0;
    if constexpr ((kVar & kOctRestage) != 0 && std::is_same_v<TOut, float>) {
        if (run) {
            const uint32_t lane = threadIdx.x & 63u;
            float* mine = slot_all + (lane >> 3) * kOctStride + r * 8u;
            reinterpret_cast<float4*>(mine)[0] = make_float4(c[0], c[1], c[2], c[3]);
            reinterpret_cast<float4*>(mine)[1] = make_float4(c[4], c[5], c[6], c[7]);
            wave_lds_order();
            const uint32_t chunk = lane & 15u, t = chunk >> 1, half = chunk & 1u;
            unroll<2>([&](auto h) {
                const uint32_t row = h * 4u + (lane >> 4);
                const float4 v = reinterpret_cast<const float4*>(slot_all + t * kOctStride + row * 8u)[half];
                st<kNT>(reinterpret_cast<float4*>(plane + run_base + row * g.width) + chunk, v);
            });
            return;
        }
    }
    if (p.valid) store_row<kNT>(plane + p.base + r * g.width, c);
}

}  // namespace

// Forward, octet mapping.  Arguments as fdct_kernel.
template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>) void fdct_octet_kernel(const TIn* __restrict__ img, TOut* __restrict__ out,
                                                                  float* __restrict__ shifted, TileGrid g,
                                                                  const float* __restrict__ t_dev, QParams qp,
                                                                  float shift) {
    constexpr bool kSkipZero = std::is_same_v<TIn, uint8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    const float* qtab = kQuant ? stage_tables<kVar, 2>(qp.q, &qp.r) : nullptr;
    const uint32_t lane = threadIdx.x & 63u, t = lane >> 3, x = lane & 7u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
    const uint32_t first = wave * 8u;
    if (first >= g.ntiles) return;
    const OctetPos p = octet_pos(g, first + t);
    const bool run = octet_run(g, first);
    const uint64_t run_base = octet_pos(g, first).base;
    float* const slot_all = octet_slot<kVar>();
    float* const slot = slot_all + t * kOctStride;

    // phase 1: column x, level shift (sub_matrix_scalar, utils_kernels.cu:16)
    float col[8];
    unroll<8>([&](auto i) { col[i] = p.valid ? static_cast<float>(img[p.base + i * g.width + x]) - shift : 0.0f; });
    if constexpr (kWriteback) {
        if (p.valid) unroll<8>([&](auto i) { shifted[p.base + i * g.width + x] = col[i]; });
    }
    unroll<8>([&](auto v) {
        float s = 0.0f;
        unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(col[i], s); });
        slot[v * 8u + x] = s;
    });
    wave_lds_order();
    // phase 2: row r = x of P
    const uint32_t r = x;
    float prow[8];
    const float4 a = reinterpret_cast<const float4*>(slot + r * 8u)[0];
    const float4 b = reinterpret_cast<const float4*>(slot + r * 8u)[1];
    prow[0] = a.x, prow[1] = a.y, prow[2] = a.z, prow[3] = a.w;
    prow[4] = b.x, prow[5] = b.y, prow[6] = b.z, prow[7] = b.w;
    float c[8];
    unroll<8>([&](auto u) {
        float s = 0.0f;
        unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(prow[i], s); });
        c[u] = s;
    });
    if constexpr (kQuant) {
        const float4* qr = reinterpret_cast<const float4*>(qtab + r * 8u);
        const float4* rr = reinterpret_cast<const float4*>(qtab + 64u + r * 8u);
        const float4 q0 = qr[0], q1 = qr[1], r0 = rr[0], r1 = rr[1];
        const float qv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const float rv[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        unroll<8>([&](auto u) { c[u] = quantise<kVar>(c[u], qv[u], rv[u]); });
    }
    wave_lds_order();
    octet_store<kVar>(out, g, p, r, run, run_base, slot_all, c);
}

// Inverse, octet mapping.  Arguments as idct_kernel.
template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>) void idct_octet_kernel(const TIn* __restrict__ coef, TOut* __restrict__ out,
                                                                  float* __restrict__ dq_out, TileGrid g,
                                                                  const float* __restrict__ t_dev, Mat64 q,
                                                                  float shift) {
    constexpr bool kSkipZero = std::is_same_v<TIn, int8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    const float* qtab = kDequant ? stage_tables<kVar, 1>(q, nullptr) : nullptr;
    const uint32_t lane = threadIdx.x & 63u, t = lane >> 3, x = lane & 7u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
    const uint32_t first = wave * 8u;
    if (first >= g.ntiles) return;
    const OctetPos p = octet_pos(g, first + t);
    const bool run = octet_run(g, first);
    const uint64_t run_base = octet_pos(g, first).base;
    float* const slot_all = octet_slot<kVar>();
    float* const slot = slot_all + t * kOctStride;

    // phase 1: column x of D = q * Q (multiply_matrices, utils_kernels.cu:55)
    float col[8];
    unroll<8>([&](auto i) {
        col[i] = p.valid ? static_cast<float>(coef[p.base + i * g.width + x]) : 0.0f;
        if constexpr (kDequant) col[i] = col[i] * qtab[i * 8u + x];
    });
    if constexpr (kDequant && (kVar & kVarWbDequant) != 0) {
        if (p.valid) unroll<8>([&](auto i) { dq_out[p.base + i * g.width + x] = col[i]; });
    }
    unroll<8>([&](auto v) {
        float s = 0.0f;
        unroll<8>([&](auto i) { s = T.template mac<i * 8 + v>(col[i], s); });
        slot[v * 8u + x] = s;
    });
    wave_lds_order();
    const uint32_t r = x;
    float prow[8];
    const float4 a = reinterpret_cast<const float4*>(slot + r * 8u)[0];
    const float4 b = reinterpret_cast<const float4*>(slot + r * 8u)[1];
    prow[0] = a.x, prow[1] = a.y, prow[2] = a.z, prow[3] = a.w;
    prow[4] = b.x, prow[5] = b.y, prow[6] = b.z, prow[7] = b.w;
    float o[8];
    unroll<8>([&](auto u) {
        float s = 0.0f;
        unroll<8>([&](auto i) { s = T.template mac<i * 8 + u>(prow[i], s); });
        o[u] = s + shift;  // add_matrix_scalar (utils_kernels.cu:29), no clamp
    });
    wave_lds_order();
    octet_store<kVar>(out, g, p, r, run, run_base, slot_all, o);
}

inline dim3 octet_grid(const TileGrid& g, uint32_t block) {
    const uint32_t waves = (g.ntiles + 7u) / 8u;
    const uint32_t per = block / 64u;
    return dim3((waves + per - 1u) / per);
}

}  // namespace hpdct
