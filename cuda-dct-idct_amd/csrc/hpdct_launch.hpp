// hpdct_launch.hpp -- launch geometry and the product's kernel choice for
// every (input, output, flags) combination of the path.  Included by the
// explicit-instantiation units (hpdct_fwd_*.hip, hpdct_inv.hip) and tools.
#pragma once

#include "hpdct.h"
#include "hpdct_kernels_impl.hpp"
#include "hpdct_octet.hpp"
#include "hpdct_duo.hpp"

namespace hpdct {

// ---------------------------------------------------------------------------
// Launch geometry.
// ---------------------------------------------------------------------------
// Resident waves per CU the persistent kernels are sized for (4 waves/SIMD at
// <= 128 VGPRs); 256 CUs on MI355X.  The grid never exceeds the set count.
constexpr uint32_t kPersistWavesPerCU = 16;

inline dim3 grid_for(const TileGrid& g, bool persist, uint32_t cus, uint32_t block = kBlockThreads) {
    const uint32_t sets = (g.ntiles + 63u) / 64u;
    const uint32_t waves_per_block = block / 64u;
    uint32_t blocks = (sets + waves_per_block - 1) / waves_per_block;
    if (persist) {
        const uint32_t cap = cus * kPersistWavesPerCU / waves_per_block;
        if (blocks > cap) blocks = cap;
    }
    return dim3(blocks);
}

inline uint32_t device_cus() {
    static thread_local int cached_dev = -1;
    static thread_local uint32_t cached_cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev != cached_dev) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            cached_cus = static_cast<uint32_t>(cus);
        cached_dev = dev;
    }
    return cached_cus;
}

// Product variant choice (measured on MI355X, tools/kbench.hip).
//
// Tile-per-lane kernels (hpdct_kernels_impl.hpp), for frames of >= 8 tile
// sets (64 tiles each) per CU: fp32 planes are stored through the LDS
// re-staging with non-temporal stores (1 KiB contiguous per store
// instruction), 8-bit planes with non-temporal stores; the int8 output with
// the SDWA byte-pack conversion; the fast quotient where the caller proved it
// legal.  512-thread workgroups (1-3 % faster than 256 on every kernel).
template <typename TIn, typename TOut>
constexpr unsigned kProdVar = (2u << 12) | kVarNT | (std::is_same_v<TOut, float> ? kVarLdsStore : 0u) |
                              (std::is_same_v<TOut, int8_t> ? kVarI8Pack : 0u);
// Octet kernels (hpdct_octet.hpp, 8 lanes per tile) for smaller frames,
// where the tile-per-lane grid is too short to fill 256 CUs (1024^2: 6.2 ->
// 3.7 us).  256-thread workgroups; fp32 rows re-staged for 256-B runs.
template <typename TOut>
constexpr unsigned kOctVar = kVarNT | (std::is_same_v<TOut, float> ? kOctRestage : 0u);
constexpr uint32_t kOctetSetsPerCU = 8;
// Duo kernels (hpdct_duo.hpp, 2 lanes per tile, 1 KiB row loads and stores)
// for fp32 -> fp32 at the other sizes (8192^2: forward 102.4 -> 89.6 us,
// inverse 93.3 -> 88.0 us, compat forward with write-back 159 -> 136 us).
constexpr unsigned kDuoVar = kVarNT;

enum class Mapping { kTile, kOctet, kDuo };

// f32: an fp32 -> fp32 kernel in the reference's pass order (duo-capable)
inline Mapping pick_mapping(const TileGrid& g, bool f32) {
    const int m = mapping_mode();
    if (m == HPDCT_MAPPING_TILE) return Mapping::kTile;
    if (m == HPDCT_MAPPING_OCTET) return Mapping::kOctet;
    if (m == HPDCT_MAPPING_DUO && f32) return Mapping::kDuo;
    if ((g.ntiles + 63u) / 64u < kOctetSetsPerCU * device_cus()) return Mapping::kOctet;
    return f32 ? Mapping::kDuo : Mapping::kTile;
}

template <unsigned kV, typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_go(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev, const QParams& q,
                   float shift, hipStream_t s) {
    hipLaunchKernelGGL((fdct_kernel<TIn, TOut, kQuant, kBuiltinT, kWriteback, kV>), grid_for(g, false, 0, kBlock<kV>),
                       dim3(kBlock<kV>), 0, s, img, out, shifted, g, t_dev, q, shift);
    return hipGetLastError();
}

// uint8 -> fp32 tile kernels: 1024-thread workgroups for frames of at most
// kBigWgSetsPerCU sets per CU, where the whole grid is about one round of
// resident waves (with inputs from HBM: 2048 x 16384 35.2 -> 32.3 us,
// 4096 x 8192 34.2 -> 31.2 us; neutral at 8192^2 (64 sets per CU), 5 % slower
// at 16384^2; profiles/r02/kbench2_wide_hbm_r02.log, kbench2_wide_r02.log),
// the product's 512 otherwise.
constexpr uint32_t kBigWgSetsPerCU = 32;

template <unsigned kV, typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_tile_go(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                        const QParams& q, float shift, hipStream_t s) {
    if constexpr (std::is_same_v<TIn, uint8_t> && std::is_same_v<TOut, float>) {
        if ((g.ntiles + 63u) / 64u <= kBigWgSetsPerCU * device_cus())
            return fdct_go<(kV & ~(3u << 12)) | (3u << 12), TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                img, out, shifted, g, t_dev, q, shift, s);
    }
    return fdct_go<kV, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev, q, shift, s);
}

template <unsigned kV, typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_octet_go(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                         const QParams& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((fdct_octet_kernel<TIn, TOut, kQuant, kBuiltinT, kWriteback, kV>), octet_grid(g, kBlock<kV>),
                       dim3(kBlock<kV>), 0, s, img, out, shifted, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_duo_go(const float* img, float* out, float* shifted, const TileGrid& g, const float* t_dev,
                       const QParams& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((fdct_duo_kernel<kQuant, kBuiltinT, kWriteback, kV>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>),
                       0, s, img, out, shifted, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, bool kDequant, bool kBuiltinT, typename TOut>
hipError_t idct_duo_go(const float* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev,
                       const Mat64& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((idct_duo_kernel<kDequant, kBuiltinT, kV, TOut>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>), 0,
                       s, coef, out, dq_out, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, bool kInv, bool kQ, bool kBuiltinT, bool kWb>
hipError_t rowfirst_duo_go(const float* src, float* out, float* wb, const TileGrid& g, const float* t_dev,
                           const Mat64& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((rowfirst_duo_kernel<kInv, kQ, kBuiltinT, kWb, kV>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>),
                       0, s, src, out, wb, g, t_dev, q, shift);
    return hipGetLastError();
}

template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t launch_fdct_impl(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                            const QParams& q, float shift, bool fastdiv, bool row_first, hipStream_t s) {
    constexpr unsigned kBase = kProdVar<TIn, TOut>;
    constexpr unsigned kOct = kOctVar<TOut>;
    constexpr bool kFastDivOk = std::is_same_v<TIn, uint8_t> && kQuant && kBuiltinT && !kWriteback;
    if constexpr (std::is_same_v<TIn, float> && std::is_same_v<TOut, float>) {
        if (row_first) {  // cublasDCTv2 pass order: duo (rows first), or tile when forced
            if (mapping_mode() != HPDCT_MAPPING_TILE)
                return rowfirst_duo_go<kDuoVar, false, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev,
                                                                                      q.q, shift, s);
            return fdct_go<kBase | kVarRowFirst, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g,
                                                                                           t_dev, q, shift, s);
        }
    }
    (void)row_first;
    constexpr bool kF32 = std::is_same_v<TIn, float> && std::is_same_v<TOut, float>;
    const Mapping map = pick_mapping(g, kF32);
    if constexpr (kF32) {
        if (map == Mapping::kDuo)
            return fdct_duo_go<kDuoVar, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev, q, shift, s);
    }
    if (map == Mapping::kOctet) {
        if constexpr (kFastDivOk) {
            if (fastdiv)
                return fdct_octet_go<kOct | kVarFastDiv, TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                    img, out, shifted, g, t_dev, q, shift, s);
        }
        return fdct_octet_go<kOct, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev, q, shift,
                                                                             s);
    }
    // uint8 -> fp32 rows at a width that is not a multiple of 512 px: the
    // straddle-capable variant (two-run staged stores, kVarStraddle)
    constexpr bool kStraddleOk = std::is_same_v<TIn, uint8_t> && std::is_same_v<TOut, float> && kBuiltinT;
    if constexpr (kStraddleOk) {
        if (g.tiles_x % 64u != 0u) {
            if constexpr (kFastDivOk) {
                if (fastdiv)
                    return fdct_tile_go<kBase | kVarFastDiv | kVarStraddle, TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                        img, out, shifted, g, t_dev, q, shift, s);
            }
            return fdct_tile_go<kBase | kVarStraddle, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g,
                                                                                           t_dev, q, shift, s);
        }
    }
    if constexpr (kFastDivOk) {
        if (fastdiv)
            return fdct_tile_go<kBase | kVarFastDiv, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev,
                                                                                          q, shift, s);
    }
    (void)fastdiv;
    return fdct_tile_go<kBase, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev, q, shift, s);
}

template <unsigned kV, typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
hipError_t idct_go(const TIn* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev, const Mat64& q,
                   float shift, hipStream_t s) {
    hipLaunchKernelGGL((idct_kernel<TIn, TOut, kDequant, kBuiltinT, kV>), grid_for(g, false, 0, kBlock<kV>),
                       dim3(kBlock<kV>), 0, s, coef, out, dq_out, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
hipError_t idct_octet_go(const TIn* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev,
                         const Mat64& q, float shift, hipStream_t s) {
    hipLaunchKernelGGL((idct_octet_kernel<TIn, TOut, kDequant, kBuiltinT, kV>), octet_grid(g, kBlock<kV>),
                       dim3(kBlock<kV>), 0, s, coef, out, dq_out, g, t_dev, q, shift);
    return hipGetLastError();
}

template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
hipError_t launch_idct_impl(const TIn* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev,
                            const Mat64& q, float shift, bool row_first, hipStream_t s) {
    constexpr unsigned kV = kProdVar<TIn, TOut>;
    constexpr unsigned kOct = kOctVar<TOut>;
    constexpr bool kF32 = std::is_same_v<TIn, float> && std::is_same_v<TOut, float>;
    if constexpr (kF32) {
        if (row_first) {  // cublasDCTv2 pass order: duo (rows first), or tile when forced
            if (mapping_mode() != HPDCT_MAPPING_TILE) {
                if constexpr (kDequant) {
                    if (dq_out)
                        return rowfirst_duo_go<kDuoVar, true, kDequant, kBuiltinT, true>(coef, out, dq_out, g, t_dev,
                                                                                         q, shift, s);
                }
                return rowfirst_duo_go<kDuoVar, true, kDequant, kBuiltinT, false>(coef, out, nullptr, g, t_dev, q,
                                                                                  shift, s);
            }
            if constexpr (kDequant) {
                if (dq_out)
                    return idct_go<kV | kVarRowFirst | kVarWbDequant, TIn, TOut, kDequant, kBuiltinT>(
                        coef, out, dq_out, g, t_dev, q, shift, s);
            }
            return idct_go<kV | kVarRowFirst, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift,
                                                                              s);
        }
    }
    (void)row_first;
    // fp32 coefficients -> fp32 or uint8 pixels: the duo kernel's 1 KiB row loads
    // (8192^2 -> uint8: 61.8 -> 56.7 us, profiles/r01/mappings/kbench2_inv_i8.log)
    constexpr bool kDuoIn = std::is_same_v<TIn, float> && (kF32 || std::is_same_v<TOut, uint8_t>);
    const Mapping map = pick_mapping(g, kDuoIn);
    if constexpr (kDuoIn) {
        // uint8 output: 512-thread workgroups (56.7 vs 57.6 us with 256)
        constexpr unsigned kDV = std::is_same_v<TOut, uint8_t> ? (kDuoVar | (2u << 12)) : kDuoVar;
        if (map == Mapping::kDuo) {
            if constexpr (kDequant) {
                if (dq_out)
                    return idct_duo_go<kDV | kVarWbDequant, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q,
                                                                               shift, s);
            }
            return idct_duo_go<kDV, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift, s);
        }
    }
    if (map == Mapping::kOctet) {
        if constexpr (kF32 && kDequant) {
            if (dq_out)
                return idct_octet_go<kOct | kVarWbDequant, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g,
                                                                                          t_dev, q, shift, s);
        }
        return idct_octet_go<kOct, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift, s);
    }
    if constexpr (kF32 && kDequant) {
        if (dq_out)
            return idct_go<kV | kVarWbDequant, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift,
                                                                               s);
    }
    if constexpr (std::is_same_v<TIn, int8_t> && std::is_same_v<TOut, float> && kBuiltinT) {
        if (g.tiles_x % 64u != 0u)  // straddling sets: two-run staged stores (kVarStraddle)
            return idct_go<kV | kVarStraddle, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift,
                                                                              s);
    }
    return idct_go<kV, TIn, TOut, kDequant, kBuiltinT>(coef, out, dq_out, g, t_dev, q, shift, s);
}

// Frame lists: the tile kernel's product variant per frame (512-thread
// workgroups), the straddle-capable stores for fp32 rows at widths that are
// not a multiple of 512 px; grid (workgroups per frame, frames).
template <unsigned kV, typename TOut>
hipError_t fdct_frames_go(const FrameTable<TOut>& ft, int n, const TileGrid& g, const QParams& q, hipStream_t s) {
    const dim3 grid(grid_for(g, false, 0, kBlock<kV>).x, static_cast<uint32_t>(n));
    hipLaunchKernelGGL((fdct_frames_kernel<TOut, kV>), grid, dim3(kBlock<kV>), 0, s, ft, g, q);
    return hipGetLastError();
}

template <typename TOut>
hipError_t launch_fdct_frames_impl(const FrameTable<TOut>& ft, int n, const TileGrid& g, const QParams& q,
                                   bool fastdiv, hipStream_t s) {
    constexpr unsigned kBase = kProdVar<uint8_t, TOut>;
    if constexpr (std::is_same_v<TOut, float>) {
        if (g.tiles_x % 64u != 0u)
            return fastdiv ? fdct_frames_go<kBase | kVarFastDiv | kVarStraddle>(ft, n, g, q, s)
                           : fdct_frames_go<kBase | kVarStraddle>(ft, n, g, q, s);
    }
    return fastdiv ? fdct_frames_go<kBase | kVarFastDiv>(ft, n, g, q, s) : fdct_frames_go<kBase>(ft, n, g, q, s);
}

inline hipError_t launch_fill_hash_impl(uint8_t* out, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    const uint64_t lanes = (n + 15) / 16;
    const dim3 grid(static_cast<uint32_t>((lanes + kBlockThreads - 1) / kBlockThreads));
    hipLaunchKernelGGL(fill_hash_kernel, grid, dim3(kBlockThreads), 0, s, out, n, seed, first);
    return hipGetLastError();
}

}  // namespace hpdct
