// hpdct_kernels_impl.hpp -- fused 8x8 block DCT/IDCT + quantisation kernels for
// CDNA4 (gfx950).  Replaces the three-launch chains of dct_all_blocks_cuda /
// idct_all_blocks_cuda (main_newAppr.cu:252-332) with one HBM pass each.
//
// Mapping ("tile per lane"): lane L of the grid owns tile L of the image in
// row-major tile order and keeps the whole 8x8 tile in VGPRs, so both passes
// of T.X.T^T run in registers in the reference's exact FMA order with no
// LDS traffic, no barrier and no cross-lane shuffles.  64 consecutive lanes
// own 64 horizontally adjacent tiles, so
//   - each u8 row load is one global_load_dwordx2 covering 512 contiguous
//     bytes per wave (8 per tile row set),
//   - each fp32 row store is two global_store_dwordx4 that together cover
//     2 KiB contiguous per wave.
// Why not one wavefront per tile: a lane-per-pixel mapping needs 7 cross-lane
// operands per output per pass (14 DPP/ds_bpermute per pixel), which on its
// own costs as much LDS-crossbar time as the whole HBM stream; see DESIGN.md.
#pragma once

#include "hpdct_kernels.h"
#include "hpdct_tile.hpp"

namespace hpdct {

namespace {

__device__ __forceinline__ float byte_f32(uint32_t w, int k) {
    return static_cast<float>((w >> (8 * k)) & 0xffu);  // v_cvt_f32_ubyteK
}

__device__ __forceinline__ uint32_t pack_i8x4(float a, float b, float c, float d) {
    const uint32_t ia = static_cast<uint32_t>(static_cast<int32_t>(a)) & 0xffu;
    const uint32_t ib = static_cast<uint32_t>(static_cast<int32_t>(b)) & 0xffu;
    const uint32_t ic = static_cast<uint32_t>(static_cast<int32_t>(c)) & 0xffu;
    const uint32_t id = static_cast<uint32_t>(static_cast<int32_t>(d)) & 0xffu;
    return ia | (ib << 8) | (ic << 16) | (id << 24);
}

// convertToUnsignedChar (utils.cu:21): (unsigned char)fminf(fmaxf(x, 0), 255)
__device__ __forceinline__ uint32_t to_u8(float x) {
    return static_cast<uint32_t>(__builtin_fminf(__builtin_fmaxf(x, 0.0f), 255.0f));
}
__device__ __forceinline__ uint32_t pack_u8x4(float a, float b, float c, float d) {
    return to_u8(a) | (to_u8(b) << 8) | (to_u8(c) << 16) | (to_u8(d) << 24);
}

__device__ __forceinline__ bool tile_coords(const TileGrid& g, uint32_t& tile, uint64_t& base) {
    tile = blockIdx.x * kBlockThreads + threadIdx.x;
    if (tile >= g.ntiles) return false;
    const uint32_t ty = tile / g.tiles_x;
    const uint32_t tx = tile - ty * g.tiles_x;
    base = static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(tx) * 8u;
    return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// Forward: image -> (quantised) coefficients.
// ---------------------------------------------------------------------------
template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
__global__ __launch_bounds__(kBlockThreads) void fdct_kernel(const TIn* __restrict__ img, TOut* __restrict__ out,
                                                             float* __restrict__ shifted, TileGrid g,
                                                             const float* __restrict__ t_dev, Mat64 q, float shift) {
    uint32_t tile;
    uint64_t base;
    if (!tile_coords(g, tile, base)) return;

    // finite inputs (u8) may skip the zero terms of the built-in T
    constexpr bool kSkipZero = std::is_same_v<TIn, uint8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);

    float x[8][8];
    if constexpr (std::is_same_v<TIn, uint8_t>) {
        uint2 raw[8];
        unroll<8>([&](auto i) { raw[i] = *reinterpret_cast<const uint2*>(img + base + i * g.width); });
        unroll<8>([&](auto i) {
            unroll<4>([&](auto j) {
                x[i][j] = byte_f32(raw[i].x, j) - shift;
                x[i][j + 4] = byte_f32(raw[i].y, j) - shift;
            });
        });
    } else {
        float4 raw[8][2];
        unroll<8>([&](auto i) {
            const float4* src = reinterpret_cast<const float4*>(img + base + i * g.width);
            raw[i][0] = src[0];
            raw[i][1] = src[1];
        });
        unroll<8>([&](auto i) {
            x[i][0] = raw[i][0].x - shift;
            x[i][1] = raw[i][0].y - shift;
            x[i][2] = raw[i][0].z - shift;
            x[i][3] = raw[i][0].w - shift;
            x[i][4] = raw[i][1].x - shift;
            x[i][5] = raw[i][1].y - shift;
            x[i][6] = raw[i][1].z - shift;
            x[i][7] = raw[i][1].w - shift;
        });
        if constexpr (kWriteback) {
            // the reference leaves X-128 in its input (main_newAppr.cu:273)
            unroll<8>([&](auto i) {
                float4* dst = reinterpret_cast<float4*>(shifted + base + i * g.width);
                dst[0] = make_float4(x[i][0], x[i][1], x[i][2], x[i][3]);
                dst[1] = make_float4(x[i][4], x[i][5], x[i][6], x[i][7]);
            });
        }
    }

    fdct_tile(T, x, [&](auto v, float (&c)[8]) {
        if constexpr (kQuant) {
            // divide_matrices (utils_kernels.cu:42): round(C / Q[v][u])
            unroll<8>([&](auto u) { c[u] = __builtin_roundf(c[u] / q.v[v * 8 + u]); });
        }
        TOut* row = out + base + v * g.width;
        if constexpr (std::is_same_v<TOut, float>) {
            float4* dst = reinterpret_cast<float4*>(row);
            dst[0] = make_float4(c[0], c[1], c[2], c[3]);
            dst[1] = make_float4(c[4], c[5], c[6], c[7]);
        } else {
            *reinterpret_cast<uint2*>(row) = make_uint2(pack_i8x4(c[0], c[1], c[2], c[3]),
                                                        pack_i8x4(c[4], c[5], c[6], c[7]));
        }
    });
}

// ---------------------------------------------------------------------------
// Inverse: (quantised) coefficients -> image.
// ---------------------------------------------------------------------------
template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
__global__ __launch_bounds__(kBlockThreads) void idct_kernel(const TIn* __restrict__ coef, TOut* __restrict__ out,
                                                             TileGrid g, const float* __restrict__ t_dev, Mat64 q,
                                                             float shift) {
    uint32_t tile;
    uint64_t base;
    if (!tile_coords(g, tile, base)) return;

    constexpr bool kSkipZero = std::is_same_v<TIn, int8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);

    float d[8][8];
    if constexpr (std::is_same_v<TIn, int8_t>) {
        uint2 raw[8];
        unroll<8>([&](auto i) { raw[i] = *reinterpret_cast<const uint2*>(coef + base + i * g.width); });
        unroll<8>([&](auto i) {
            unroll<4>([&](auto j) {
                d[i][j] = static_cast<float>(static_cast<int8_t>((raw[i].x >> (8 * j)) & 0xffu));
                d[i][j + 4] = static_cast<float>(static_cast<int8_t>((raw[i].y >> (8 * j)) & 0xffu));
            });
        });
    } else {
        float4 raw[8][2];
        unroll<8>([&](auto i) {
            const float4* src = reinterpret_cast<const float4*>(coef + base + i * g.width);
            raw[i][0] = src[0];
            raw[i][1] = src[1];
        });
        unroll<8>([&](auto i) {
            d[i][0] = raw[i][0].x;
            d[i][1] = raw[i][0].y;
            d[i][2] = raw[i][0].z;
            d[i][3] = raw[i][0].w;
            d[i][4] = raw[i][1].x;
            d[i][5] = raw[i][1].y;
            d[i][6] = raw[i][1].z;
            d[i][7] = raw[i][1].w;
        });
    }
    if constexpr (kDequant) {
        // multiply_matrices (utils_kernels.cu:55): D = q * Q[i][j]
        unroll<8>([&](auto i) { unroll<8>([&](auto j) { d[i][j] = d[i][j] * q.v[i * 8 + j]; }); });
    }

    idct_tile(T, d, [&](auto v, float (&r)[8]) {
        // add_matrix_scalar (utils_kernels.cu:29): R + 128, no clamp
        unroll<8>([&](auto u) { r[u] = r[u] + shift; });
        TOut* row = out + base + v * g.width;
        if constexpr (std::is_same_v<TOut, float>) {
            float4* dst = reinterpret_cast<float4*>(row);
            dst[0] = make_float4(r[0], r[1], r[2], r[3]);
            dst[1] = make_float4(r[4], r[5], r[6], r[7]);
        } else {
            *reinterpret_cast<uint2*>(row) =
                make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
        }
    });
}

// ---------------------------------------------------------------------------
// Synthetic frame generator (config C4): 16 pixels per lane.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hash_px(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return static_cast<uint32_t>((z ^ (z >> 31)) & 255u);
}

static __global__ __launch_bounds__(kBlockThreads) void fill_hash_kernel(uint8_t* __restrict__ out, uint64_t n,
                                                                  uint64_t seed, uint64_t first) {
    const uint64_t i0 = (static_cast<uint64_t>(blockIdx.x) * kBlockThreads + threadIdx.x) * 16u;
    if (i0 >= n) return;
    if (i0 + 16 <= n) {
        uint32_t w[4];
        unroll<4>([&](auto k) {
            uint32_t acc = 0;
            unroll<4>([&](auto b) { acc |= hash_px(seed, first + i0 + k * 4 + b) << (8 * b); });
            w[k] = acc;
        });
        *reinterpret_cast<uint4*>(out + i0) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (uint64_t i = i0; i < n; ++i) out[i] = static_cast<uint8_t>(hash_px(seed, first + i));
    }
}

// ---------------------------------------------------------------------------
// Launchers (host side).  Shapes are validated by the caller (hpdct_api.hip).
// ---------------------------------------------------------------------------
namespace {
inline dim3 grid_for(const TileGrid& g) { return dim3((g.ntiles + kBlockThreads - 1) / kBlockThreads); }
}  // namespace

template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t launch_fdct(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                       const Mat64& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((fdct_kernel<TIn, TOut, kQuant, kBuiltinT, kWriteback>), grid_for(g), dim3(kBlockThreads), 0,
                       s, img, out, shifted, g, t_dev, q, shift);
    return hipGetLastError();
}

template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
hipError_t launch_idct(const TIn* coef, TOut* out, const TileGrid& g, const float* t_dev, const Mat64& q, float shift,
                       hipStream_t s) {
    hipLaunchKernelGGL((idct_kernel<TIn, TOut, kDequant, kBuiltinT>), grid_for(g), dim3(kBlockThreads), 0, s, coef,
                       out, g, t_dev, q, shift);
    return hipGetLastError();
}

inline hipError_t launch_fill_hash_impl(uint8_t* out, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    const uint64_t lanes = (n + 15) / 16;
    const dim3 grid(static_cast<uint32_t>((lanes + kBlockThreads - 1) / kBlockThreads));
    hipLaunchKernelGGL(fill_hash_kernel, grid, dim3(kBlockThreads), 0, s, out, n, seed, first);
    return hipGetLastError();
}

}  // namespace hpdct
