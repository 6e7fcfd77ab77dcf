// hpdct_kernels.h -- host-visible declarations of the gfx950 kernels
// (launchers are explicit template instantiations in hpdct_fwd_*.hip /
// hpdct_inv.hip; the kernels themselves are in hpdct_kernels_impl.hpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hpdct {

constexpr uint32_t kBlockThreads = 256;  // 4 wave64 per workgroup

// 64 floats passed by value as a kernel argument (lands in SGPRs)
struct Mat64 {
    float v[64];
};

// Quantiser parameters passed by value: Q and RN(1/Q) (the latter is used
// only by the verified fast quotient).
struct QParams {
    Mat64 q;
    Mat64 r;
};

// Tile geometry of one launch: ntiles = (height/8) * (width/8) < 2^32.
struct TileGrid {
    uint32_t ntiles;
    uint32_t tiles_x;
    uint64_t width;  // elements per image row
};

// qmode (the quotient): 0 IEEE division; 1 the 3-operation quotient (only
// legal for a table whose entries are all integers in 1..255 with uint8 input
// and the built-in T, or fp32 input behind the duo kernels' range check; the
// caller checks); 2 as 1 plus the default JPEG table's per-position 3-op forms
// (hpdct_quant_forms.h: only the default table, uint8 input, built-in T,
// shift 128).  shift is 128 (reference level shift) or 0.
// row_first: cublasDCTv2 pass order (fp32 -> fp32 only).
template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback>
hipError_t launch_fdct(const TIn* img, TOut* out, float* shifted, const TileGrid& g, const float* t_dev,
                       const QParams& q, float shift, int qmode, bool row_first, hipStream_t s);

// dq_out (fp32 -> fp32 with dequantisation only, else nullptr): q*Q is also
// written there (the in-place multiply of the cublasDCTv2 inverse).
template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT>
hipError_t launch_idct(const TIn* coef, TOut* out, float* dq_out, const TileGrid& g, const float* t_dev,
                       const Mat64& q, float shift, bool row_first, hipStream_t s);

// Round trip (hpdct_roundtrip.hpp): uint8 frame -> fp32 quantised
// coefficients + optional reconstruction + optional quality sums, built-in T.
// Device accumulators, the layout of hpdct_roundtrip_sums (include/hpdct.h).
struct RtSums {
    unsigned long long sse_f32_fx;  // sum (x - (R+128))^2 * 2^16, per-tile fp32 sums rounded
    unsigned long long sse_u8;      // sum (x - u8(R+128))^2, exact
    unsigned long long sum_x2;      // sum x^2, exact
};
enum : int { kRtReconNone = 0, kRtReconU8 = 1, kRtReconF32 = 2 };
// fast: integer table in 1..255 with int8-range quotients (verified quotient);
// sums may be nullptr (no statistics), recon nullptr with kRtReconNone.
// zero_sums: the launch overwrites *sums, else adds to it.  The kernel adds
// into a library spread slot kept per sums pointer and a one-wave kernel folds
// it into *sums (a memset of *sums and the tile kernel when no slot can be had).
hipError_t launch_roundtrip(const uint8_t* img, float* coef, void* recon, int recon_kind, RtSums* sums,
                            const TileGrid& g, const QParams& qp, int fast, bool zero_sums, hipStream_t s);
// The pieces launch_roundtrip (hpdct_roundtrip.hip) chooses from:
//  - the tile-per-lane kernels, one unit per reconstruction kind
//    (hpdct_rt_tile_{u8,f32,none}.hip); sums: the struct (or spread
//    sub-slot 0) the workgroups add into, or nullptr;
//  - the two-lanes-per-tile kernel (hpdct_rt_duo.hip): fast 1 or 2, a uint8
//    reconstruction (recon) or none (nullptr); spread: a zeroed spread slot
//    (kRtSpread sub-slots, hpdct_roundtrip.hpp) the waves add into, or
//    nullptr for no sums;
//  - the finish kernel folding a spread slot into *dst (overwrite, or add
//    when accumulate) and zeroing it.
hipError_t launch_rt_tile_u8(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g,
                             const QParams& qp, int fast, hipStream_t s);
hipError_t launch_rt_tile_f32(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g,
                              const QParams& qp, int fast, hipStream_t s);
hipError_t launch_rt_tile_none(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g,
                               const QParams& qp, int fast, hipStream_t s);
hipError_t launch_rt_duo(const uint8_t* img, float* coef, void* recon, int recon_kind, unsigned long long* spread,
                         const TileGrid& g, const QParams& qp, int fast, hipStream_t s);
hipError_t launch_rt_duo_f32(const uint8_t* img, float* coef, void* recon, unsigned long long* spread,
                             const TileGrid& g, const QParams& qp, int fast, hipStream_t s);
hipError_t launch_rt_finish(RtSums* dst, unsigned long long* spread, bool accumulate, hipStream_t s);
// the spread slot of a sums pointer back to its device's free list
// (hpdct_roundtrip_release_sums); false when the pointer had none
bool release_sums_slot(const void* sums);

// uint8 -> quantised fp32 forward on the two-lanes-per-tile mapping (round 6;
// fdct_duo_u8_kernel, hpdct_rt_duo.hpp): qmode 1 or 2, built-in T, level
// shift 128, tiles_x a multiple of 32, width below 2^22 px.  kDuoFwdBlock-thread
// workgroups, at most kDuoFwdCapWgs resident per CU (16 waves); AUTO takes it
// from kDuoFwdMinWavesPerCU of its 32-tile waves per CU (launch_fdct_impl).
constexpr uint32_t kDuoFwdBlock = 256, kDuoFwdCapWgs = 4, kDuoFwdMinWavesPerCU = 4;
hipError_t launch_fdct_duo_u8(const uint8_t* img, float* coef, const TileGrid& g, const QParams& qp, int qmode,
                              hipStream_t s);

// A list of frames per launch (hpdct_forward_frames): up to kMaxFramesPerLaunch
// device pointer pairs travel in the kernel arguments (1 KiB).
constexpr int kMaxFramesPerLaunch = 64;
template <typename TOut>
struct FrameTable {
    const uint8_t* in[kMaxFramesPerLaunch];
    TOut* out[kMaxFramesPerLaunch];
};
// n <= kMaxFramesPerLaunch frames of grid g, uint8 -> TOut (float or int8_t),
// built-in T, quantised with q (qmode as launch_fdct).
template <typename TOut>
hipError_t launch_fdct_frames(const FrameTable<TOut>& ft, int n, const TileGrid& g, const QParams& q, int qmode,
                              hipStream_t s);
// the duo forward over such a list (fp32 out; the conditions of
// launch_fdct_duo_u8, the size rule on the whole list)
hipError_t launch_fdct_duo_u8_frames(const FrameTable<float>& ft, int n, const TileGrid& g, const QParams& qp,
                                     int qmode, hipStream_t s);

hipError_t launch_fill_hash(uint8_t* out, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s);

// int8 wire coefficients -> fp32 plane (hpdct_decode.hip)
hipError_t launch_decode_i8_f32(const int8_t* in, float* out, uint64_t n, hipStream_t s);

// hpdct_floor_probe (hpdct_probe.hip): kind 0 an empty kernel, 1 a u8 -> fp32
// copy, both on the grid the uint8 -> fp32 forward of g launches
hipError_t launch_floor_probe(int kind, const uint8_t* in, float* out, const TileGrid& g, hipStream_t s);
// hpdct_copy_ceiling (hpdct_probe.hip): element bytes 1 or 4 (o1_bytes 0: no
// second output), n a multiple of 2048, at most cap_waves resident per CU
hipError_t launch_copy_ceiling(const void* in, int in_bytes, void* o0, int o0_bytes, void* o1, int o1_bytes,
                               uint64_t n, uint32_t cap_waves, hipStream_t s);

// hpdct_mapping in force (0 auto, 1 tile, 2 octet); hpdct_api.cpp.
int mapping_mode();

// Records msg as hpdct_last_error_string() of this thread and returns st
// (hpdct_api.cpp; every C-ABI error return goes through it).
int set_last_error(int st, const char* msg);

}  // namespace hpdct
