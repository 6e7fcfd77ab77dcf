// hpdct_launch.hpp -- launch geometry and the product's kernel choice for
// every (input, output, flags) combination of the path.  Included by the
// explicit-instantiation units (hpdct_fwd_*.hip, hpdct_inv.hip) and tools.
#pragma once

#include "hpdct.h"
#include "hpdct_kernels_impl.hpp"
#include "hpdct_octet.hpp"
#include "hpdct_duo.hpp"
#include "hpdct_residency.hpp"

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

// Residency caps (round 3).  The DRAM serves the headline's mix of 1 B/px
// reads and 4 B/px non-temporal writes best with few concurrent streams: its
// access pattern alone runs at 0.72 of 8 TB/s with the hardware's default
// residency and at 0.75-0.80 with 12-4 waves per CU (tools/kbench3 "occpat",
// profiles/r03/m/).  The arithmetic needs more than one wave per SIMD to issue
// at full rate, so the u8 -> fp32 tile kernel runs in one-wave workgroups with
// at most kF32CapWavesPerCU resident per CU.  The cap is a
// dynamic-LDS reservation (hpdct_residency.hpp).
// 10 in round 3; 7 since round 4: 56.9-57.1 against 57.7-58.4 us at 8192^2
// with the per-position quantiser (profiles/r04/b/kb3_jqcap_8192.log; 6 waves
// per CU: 64.8 us, profiles/r04/a/kb3_jqf_8192.log)
constexpr uint32_t kF32CapWavesPerCU = 7;

// Product variant choice (measured on MI355X, tools/kbench.hip).
//
// Tile-per-lane kernels (hpdct_kernels_impl.hpp), for frames of >= 8 tile
// sets (64 tiles each) per CU: fp32 planes are stored through the LDS
// re-staging with non-temporal stores (1 KiB contiguous per store
// instruction), 8-bit planes with non-temporal stores; the int8 output with
// the SDWA byte-pack conversion; the fast quotient where the caller proved it
// legal.  512-thread workgroups (1-3 % faster than 256 on every kernel in
// round 1), except the int8 output: 256-thread workgroups since its JPEG-form
// quantiser (round 4: 8192^2 28.9 against 29.8-30.0 us with 512,
// profiles/r04/a/kb3_jqi8_8192.log), and with the JPEG forms one-wave
// workgroups under a residency cap (fdct_tile_go, kI8CapWavesPerCU).
template <typename TIn, typename TOut>
constexpr unsigned kProdVar = (std::is_same_v<TOut, int8_t> ? 0u : (2u << 12)) | kVarNT |
                              (std::is_same_v<TOut, float> ? kVarLdsStore : 0u) |
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

// cap_waves: at most that many resident waves per CU (0: the hardware's default)
template <unsigned kV, typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_go(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev, const QParams& q,
                   float shift, hipStream_t s, uint32_t cap_waves = 0) {
    auto* kern = fdct_kernel<TIn, TOut, kQuant, kBuiltinT, kWriteback, kV>;
    size_t dyn = 0;
    if (cap_waves != 0) {
        static const size_t st = static_lds_of(kern);
        dyn = residency_cap_lds(st, cap_waves / (kBlock<kV> / 64u));
    }
    hipLaunchKernelGGL(kern, grid_for(g, false, 0, kBlock<kV>), dim3(kBlock<kV>), dyn, s, img, out, shifted, g, t_dev,
                       q, shift);
    return hipGetLastError();
}

// uint8 -> fp32 tile kernels (the headline):
//  - frames of at most kBigWgSetsPerCU sets per CU, where the whole grid is
//    one or two rounds of resident waves: 1024-thread workgroups, no cap
//    (4096^2: 16.3 us against 18.2-20.0 capped at 7-12; 2048 x 16384 (32 sets
//    per CU, the C4 8-way slab): 32.6 against 33.3-34.5 capped at 7-12 --
//    round 4, profiles/r04/c/kb3_capsz_*.log; round 3 had capped 17-32 sets
//    per CU at 12 per CU);
//  - larger frames: one-wave workgroups, at most kF32CapWavesPerCU resident
//    per CU (16384^2: 214.8-215.6 us at 7, 219-220 at 8-10, 222 at 12,
//    250 uncapped 1024-thread).  Round 3, before the per-position
//    quantiser and the cap of 7: 8192^2: 58.6-58.7 us at 9-10 waves/CU
//    against 61.8-62.1 for the uncapped 512-thread kernel and 62.5 for the
//    uncapped one-wave kernel; 16384^2: 218-219 against 238; 2048 x 16384:
//    33.7 against 35.0 (profiles/r03/m/kb3_occsz_*.log).  With the cap the
//    packed-fp32 transform (kVarPacked) gains another 1-2 % (8192^2: 57.6 at
//    10 waves/CU against 58.7 for the scalar form).
constexpr uint32_t kBigWgSetsPerCU = 32;
// frame lists (fdct_frames_go) keep round 3's tiers: uncapped 512-thread
// workgroups up to 16 sets per CU, capped at 12 waves per CU up to 32
constexpr uint32_t kFramesUncappedSetsPerCU = 16;
constexpr uint32_t kMidCapSetsPerCU = 32;
constexpr uint32_t kF32CapWavesPerCUMid = 12;
constexpr unsigned kOneWaveWg = 1u << 12;
// uint8 -> int8 with the default JPEG table's forms: one-wave workgroups, at
// most kI8CapWavesPerCU resident per CU (round 4, two boxes: 8192^2
// 29.6-31.1 against 30.8-32.6 us for 256-thread workgroups, 4096^2 9.1-9.2
// against 9.5-9.6, 16384^2 equal; 24 per CU: 30.0-32.2.
// profiles/r04/f/kb3_i8cap_*.log, profiles/r04/g/kb3_i8cap_*.log)
constexpr uint32_t kI8CapWavesPerCU = 20;

template <unsigned kV, typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_tile_go(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                        const QParams& q, float shift, hipStream_t s) {
    if constexpr (std::is_same_v<TIn, uint8_t> && std::is_same_v<TOut, float>) {
        const uint32_t sets_per_cu = ((g.ntiles + 63u) / 64u + device_cus() - 1u) / device_cus();
        if (sets_per_cu <= kBigWgSetsPerCU)
            return fdct_go<(kV & ~(3u << 12)) | (3u << 12), TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                img, out, shifted, g, t_dev, q, shift, s);
        // kVarHoistRun (round 5): the whole-run test once per set and each
        // row's store one row later: 56.5 against 57.4-57.7 us at 8192^2,
        // bit-exact (tools/kbench3 group hoist, profiles/r05/o/)
        return fdct_go<(kV & ~(3u << 12)) | kOneWaveWg | kVarPacked | kVarHoistRun, TIn, TOut, kQuant, kBuiltinT,
                       kWriteback>(img, out, shifted, g, t_dev, q, shift, s, kF32CapWavesPerCU);
    }
    if constexpr (std::is_same_v<TIn, uint8_t> && std::is_same_v<TOut, int8_t> && (kV & kVarJpegQ) != 0u) {
        return fdct_go<(kV & ~(3u << 12)) | kOneWaveWg, TIn, TOut, kQuant, kBuiltinT, kWriteback>(
            img, out, shifted, g, t_dev, q, shift, s, kI8CapWavesPerCU);
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

// fp32 -> fp32 duo inverse and row-first kernels: the headline's residency cap
// once the grid holds at least kDuoCapWavesPerCU of their waves (32 tiles each)
// per CU: one-wave workgroups, at most kDuoCapWaves resident per CU.  8192^2
// inverse 86.0 against 89.0-89.4 us (profiles/r03/m/kb3_invb_8192.log); driver
// bench: idct_all_blocks_cuda 89.7 -> 86.8, cublasDCTv2 pair 139.3 / 139.5 ->
// 137.3 / 132.4.
constexpr uint32_t kDuoCapWavesPerCU = 64;
constexpr uint32_t kDuoCapWaves = 10;

// (kernel, block variant, dynamic LDS) for a duo launch of the grid g
template <unsigned kV>
struct DuoShape {
    static constexpr unsigned kCapped = (kV & ~(3u << 12)) | kOneWaveWg;
    static bool capped(const TileGrid& g) {
        const uint32_t waves = (g.ntiles + kDuoTiles - 1u) / kDuoTiles;
        return waves >= kDuoCapWavesPerCU * device_cus();
    }
};
template <typename K>
size_t duo_cap_lds(K kern) {
    static const size_t st = static_lds_of(kern);
    return residency_cap_lds(st, kDuoCapWaves);
}

template <unsigned kV, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t fdct_duo_go(const float* img, float* out, float* shifted, const TileGrid& g, const float* t_dev,
                       const QParams& q, float shift, hipStream_t s) {
    // The checked 3-op quotient (integer table: the JPEG default, the drop-in
    // surface) takes the inverse's residency cap since round 6: 8192^2
    // dct_all_blocks_cuda 125.7 against 131.5 us uncapped, without the
    // write-back 88.1 against 89.5 (tools/kbench3 groups dropcap / fwdcap,
    // profiles/r06/).  With IEEE division (any other table) it stays uncapped:
    // VALU-heavier, the cap made it slower (round 3: 91.6 -> 101.8 us).
    if constexpr ((kV & kVarFastDivChecked) != 0) {
        if (DuoShape<kV>::capped(g)) {
            constexpr unsigned kC = DuoShape<kV>::kCapped;
            auto* kern = fdct_duo_kernel<kQuant, kBuiltinT, kWriteback, kC>;
            hipLaunchKernelGGL(kern, duo_grid(g, kBlock<kC>), dim3(kBlock<kC>), duo_cap_lds(kern), s, img, out,
                               shifted, g, t_dev, q, shift);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((fdct_duo_kernel<kQuant, kBuiltinT, kWriteback, kV>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>),
                       0, s, img, out, shifted, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, bool kDequant, bool kBuiltinT, typename TOut>
hipError_t idct_duo_go(const float* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev,
                       const Mat64& q, float shift, hipStream_t s) {
    if constexpr (std::is_same_v<TOut, float>) {
        if (DuoShape<kV>::capped(g)) {
            constexpr unsigned kC = DuoShape<kV>::kCapped;
            auto* kern = idct_duo_kernel<kDequant, kBuiltinT, kC, TOut>;
            hipLaunchKernelGGL(kern, duo_grid(g, kBlock<kC>), dim3(kBlock<kC>), duo_cap_lds(kern), s, coef, out, dq_out,
                               g, t_dev, q, shift);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((idct_duo_kernel<kDequant, kBuiltinT, kV, TOut>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>), 0,
                       s, coef, out, dq_out, g, t_dev, q, shift);
    return hipGetLastError();
}

template <unsigned kV, bool kInv, bool kQ, bool kBuiltinT, bool kWb>
hipError_t rowfirst_duo_go(const float* src, float* out, float* wb, const TileGrid& g, const float* t_dev,
                           const Mat64& q, float shift, hipStream_t s) {
    if (DuoShape<kV>::capped(g)) {
        constexpr unsigned kC = DuoShape<kV>::kCapped;
        auto* kern = rowfirst_duo_kernel<kInv, kQ, kBuiltinT, kWb, kC>;
        hipLaunchKernelGGL(kern, duo_grid(g, kBlock<kC>), dim3(kBlock<kC>), duo_cap_lds(kern), s, src, out, wb, g,
                           t_dev, q, shift);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((rowfirst_duo_kernel<kInv, kQ, kBuiltinT, kWb, kV>), duo_grid(g, kBlock<kV>), dim3(kBlock<kV>),
                       0, s, src, out, wb, g, t_dev, q, shift);
    return hipGetLastError();
}

// uint8 -> quantised fp32 (verified quotient, built-in T, shift 128) on the
// duo mapping (launch_fdct_duo_u8): whole 32-tile runs, widths below 2^22 px,
// from kDuoFwdMinWavesPerCU of its waves per CU in AUTO (below that, 1024^2
// and smaller, the octet kernel is as fast); forced "duo" takes it at any
// size, forced "tile" or "octet" never.
// frames: how many frames of g one launch covers (a frame list).
inline bool duo_fwd_u8_fits(const TileGrid& g, uint32_t frames = 1) {
    const int m = mapping_mode();
    if (m == HPDCT_MAPPING_TILE || m == HPDCT_MAPPING_OCTET) return false;
    if (g.tiles_x % 32u != 0u || g.width >= (uint64_t(1) << 22)) return false;
    return m == HPDCT_MAPPING_DUO ||
           static_cast<uint64_t>(g.ntiles / 32u) * frames >= uint64_t(kDuoFwdMinWavesPerCU) * device_cus();
}

template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t launch_fdct_impl(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                            const QParams& q, float shift, int qmode, bool row_first, hipStream_t s) {
    const bool fastdiv = qmode != 0;
    // the default JPEG table's per-position forms: tile kernels (the octet
    // mapping of small frames keeps the verified quotient everywhere)
    const bool jpeg = qmode == 2;
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
    if constexpr (kFastDivOk && std::is_same_v<TOut, float>) {
        if (fastdiv && shift == 128.0f && duo_fwd_u8_fits(g)) return launch_fdct_duo_u8(img, out, g, q, qmode, s);
    }
    constexpr bool kF32 = std::is_same_v<TIn, float> && std::is_same_v<TOut, float>;
    const Mapping map = pick_mapping(g, kF32);
    if constexpr (kF32) {
        if (map == Mapping::kDuo) {
            if constexpr (kQuant) {  // integer table: the range-checked 3-op quotient
                if (fastdiv)
                    return fdct_duo_go<kDuoVar | kVarFastDivChecked, kQuant, kBuiltinT, kWriteback>(img, out, shifted,
                                                                                                    g, t_dev, q,
                                                                                                    shift, s);
            }
            return fdct_duo_go<kDuoVar, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev, q, shift, s);
        }
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
                if (jpeg)
                    return fdct_tile_go<kBase | kVarFastDiv | kVarJpegQ | kVarStraddle, TIn, TOut, kQuant, kBuiltinT,
                                        kWriteback>(img, out, shifted, g, t_dev, q, shift, s);
                if (fastdiv)
                    return fdct_tile_go<kBase | kVarFastDiv | kVarStraddle, TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                        img, out, shifted, g, t_dev, q, shift, s);
            }
            return fdct_tile_go<kBase | kVarStraddle, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g,
                                                                                           t_dev, q, shift, s);
        }
    }
    if constexpr (kFastDivOk) {
        if (jpeg)
            return fdct_tile_go<kBase | kVarFastDiv | kVarJpegQ, TIn, TOut, kQuant, kBuiltinT, kWriteback>(
                img, out, shifted, g, t_dev, q, shift, s);
        if (fastdiv)
            return fdct_tile_go<kBase | kVarFastDiv, TIn, TOut, kQuant, kBuiltinT, kWriteback>(img, out, shifted, g, t_dev,
                                                                                          q, shift, s);
    }
    (void)fastdiv;
    (void)jpeg;
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
    if constexpr (std::is_same_v<TOut, float>) {
        // the headline's residency cap when the whole list is a large grid
        const uint64_t sets = static_cast<uint64_t>((g.ntiles + 63u) / 64u) * static_cast<uint64_t>(n);
        const uint64_t per_cu = (sets + device_cus() - 1u) / device_cus();
        if (per_cu > kFramesUncappedSetsPerCU) {
            constexpr unsigned kC = (kV & ~(3u << 12)) | kOneWaveWg | kVarPacked;
            auto* kern = fdct_frames_kernel<TOut, kC>;
            static const size_t st = static_lds_of(kern);
            const size_t dyn =
                residency_cap_lds(st, per_cu <= kMidCapSetsPerCU ? kF32CapWavesPerCUMid : kF32CapWavesPerCU);
            const dim3 grid(grid_for(g, false, 0, kBlock<kC>).x, static_cast<uint32_t>(n));
            hipLaunchKernelGGL(kern, grid, dim3(kBlock<kC>), dyn, s, ft, g, q);
            return hipGetLastError();
        }
    }
    const dim3 grid(grid_for(g, false, 0, kBlock<kV>).x, static_cast<uint32_t>(n));
    hipLaunchKernelGGL((fdct_frames_kernel<TOut, kV>), grid, dim3(kBlock<kV>), 0, s, ft, g, q);
    return hipGetLastError();
}

template <typename TOut>
hipError_t launch_fdct_frames_impl(const FrameTable<TOut>& ft, int n, const TileGrid& g, const QParams& q, int qmode,
                                   hipStream_t s) {
    constexpr unsigned kBase = kProdVar<uint8_t, TOut>;
    constexpr unsigned kJ = kVarFastDiv | kVarJpegQ;
    if constexpr (std::is_same_v<TOut, float>) {
        // the duo forward (round 6), as for one frame
        if (qmode != 0 && duo_fwd_u8_fits(g, static_cast<uint32_t>(n)))
            return launch_fdct_duo_u8_frames(ft, n, g, q, qmode, s);
        if (g.tiles_x % 64u != 0u)
            return qmode == 2   ? fdct_frames_go<kBase | kJ | kVarStraddle>(ft, n, g, q, s)
                   : qmode == 1 ? fdct_frames_go<kBase | kVarFastDiv | kVarStraddle>(ft, n, g, q, s)
                                : fdct_frames_go<kBase | kVarStraddle>(ft, n, g, q, s);
    }
    return qmode == 2   ? fdct_frames_go<kBase | kJ>(ft, n, g, q, s)
           : qmode == 1 ? fdct_frames_go<kBase | kVarFastDiv>(ft, n, g, q, s)
                        : fdct_frames_go<kBase>(ft, n, g, q, s);
}

inline hipError_t launch_fill_hash_impl(uint8_t* out, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    const uint64_t lanes = (n + 15) / 16;
    const dim3 grid(static_cast<uint32_t>((lanes + kBlockThreads - 1) / kBlockThreads));
    hipLaunchKernelGGL(fill_hash_kernel, grid, dim3(kBlockThreads), 0, s, out, n, seed, first);
    return hipGetLastError();
}

}  // namespace hpdct
