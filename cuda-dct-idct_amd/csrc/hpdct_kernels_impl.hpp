// hpdct_kernels_impl.hpp -- fused 8x8 block DCT/IDCT + quantisation kernels for
// CDNA4 (gfx950).  Replaces the three-launch chains of dct_all_blocks_cuda /
// idct_all_blocks_cuda (main_newAppr.cu:252-332) with one HBM pass each.
//
// Mapping ("tile per lane"): lane L of a wave owns tile L of a 64-tile *set*
// (64 horizontally adjacent tiles in row-major tile order) and keeps the whole
// 8x8 tile in VGPRs, so both passes of T.X.T^T run in registers in the
// reference's exact FMA order with no LDS traffic, no barrier and no
// cross-lane shuffles.  Per set and wave:
//   - each u8 row load is one global_load_dwordx2 covering 512 contiguous
//     bytes (8 per set),
//   - each fp32 row store is two global_store_dwordx4 that together cover
//     2 KiB contiguous.
// Only the variants the library launches live here (hpdct_launch.hpp); the
// measured-and-rejected A/B variants and the phase-split diagnostics are in
// the tools-only tools/kbench_variants.hpp.
// Why not one wavefront per tile: a lane-per-pixel mapping needs 7 cross-lane
// operands per output per pass (14 DPP/ds_bpermute per pixel), which on its
// own costs as much LDS-crossbar time as the whole HBM stream; see DESIGN.md.
#pragma once

#include "hpdct_kernels.h"
#include "hpdct_quant_forms.h"
#include "hpdct_tile.hpp"

namespace hpdct {

// Compile-time kernel variants (bit flags) of the product kernels.  Bits not
// listed here are the tools' A/B variants (tools/kbench_variants.hpp).
enum : unsigned {
    kVarFastDiv = 1u,  // quotient by  q0=c*r; e=fma(-q0,Q,c); q=fma(e,r,q0)  (r = RN(1/Q)).  Gives the same
                       // roundf() as IEEE c/Q for every |c| <= 4096 and every integer Q in 1..255
                       // (exhaustive: tests/tools/verify_fastdiv.*); enabled unconditionally only for such
                       // tables with uint8 input and the built-in T (|C| <= 1024); fp32 input with such a
                       // table takes it per output row under kVarFastDivChecked.
    kVarLdsStore = 8u, // fp32 rows re-staged through LDS so every store instruction writes 1 KiB contiguous
    kVarNT = 16u,      // non-temporal (streaming) stores for the output planes
    // bits 12..13: workgroup size: 0 -> 256 threads, 1 -> 64, 2 -> 512, 3 -> 1024
    kVarRowFirst = 1u << 14,  // cublasDCTv2 pass order (row pass first), fp32 compat path
    kVarWbDequant = 1u << 15, // inverse: write q*Q back into the fp32 coefficient input
                              // (in-place multiply_matrices of main_cublass_2.cu:285)
    kVarFastDivChecked = 1u << 26,  // fp32 input (any T), integer table in 1..255: the 3-op quotient for an
                                    // output row when every lane's 8 values have |C| <= 4096 (wave-uniform
                                    // test, NaN/inf fail it), IEEE division otherwise: exact either way
                                    // (verify_fastdiv covers every |C| <= 4096)
    kVarPacked = 1u << 19,    // uint8 -> fp32 or int8 quantised, built-in T: packed-fp32 transform and
                              // quotient (fdct_tile_pk; fp32: 844 instead of 1,308 VALU instructions per set)
    kVarI8Pack = 1u << 17,    // int8 output: round-half-away folded into the truncating cvt, and each
                              // coefficient converted straight into its byte (SDWA dst_sel, one op)
    kVarJpegQ = 1u << 11,     // the DEFAULT JPEG table, uint8 input, built-in T, level shift 128 (with
                              // kVarFastDiv): per position the 3-op form F or H where it is proven exact
                              // below that position's |C| bound, the 6-op form elsewhere
                              // (hpdct_quant_forms.h, tests/tools/verify_quant_pos.c)
    kVarHoistRun = 1u << 20,  // packed u8 -> fp32 forward (the capped headline kernel): the whole-run test
                              // (split == 64) taken once per set, two straight-line copies of the body, and in
                              // the whole-run copy each row's re-staged stores issued one row later, after the
                              // next row's LDS writes (tools/kbench3 group hoist: 56.5 against 57.4-57.7 us)
    kVarStraddle = 1u << 30,  // fp32 LDS-staged rows: a 64-tile set that straddles two tile rows (width not a
                              // multiple of 512 px) stores two contiguous runs per instruction instead of
                              // 32 B per lane; launched only for such widths (the branch costs the
                              // power-of-two frames ~3 %, profiles/r01/ab_straddle.log)
};
// Bits only the product kernels give a meaning to: the tools' A/B variant
// bits must stay clear of them (static_assert in tools/kbench_variants.hpp).
constexpr unsigned kProductOnlyVarBits = kVarFastDivChecked | kVarJpegQ;
template <unsigned kVar>
constexpr uint32_t kBlock = ((kVar >> 12) & 3u) == 1u   ? 64u
                            : ((kVar >> 12) & 3u) == 2u ? 512u
                            : ((kVar >> 12) & 3u) == 3u ? 1024u
                                                        : kBlockThreads;

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

// convertToUnsignedChar (utils.cu:21): (unsigned char)fminf(fmaxf(x, 0), 255),
// two operations per pixel: v_cvt_u32_f32 truncates and saturates (NaN and
// negatives -> 0, +inf -> 0xffffffff), then min(., 255) is written straight
// into byte k of the packed word (SDWA dst_sel).  Same value for every fp32
// input, NaN and infinities included (tests/test_gpu_parity.py extremes).
__device__ __forceinline__ uint32_t cvt_u32_sat(float x) {
    uint32_t t;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(t) : "v"(x));
    return t;
}
__device__ __forceinline__ uint32_t pack_u8x4(float a, float b, float c, float d) {
    const uint32_t k255 = 255u;
    uint32_t w;
    asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD"
        : "=v"(w) : "v"(cvt_u32_sat(a)), "v"(k255));
    asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(w) : "v"(cvt_u32_sat(b)), "v"(k255));
    asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(w) : "v"(cvt_u32_sat(c)), "v"(k255));
    asm("v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(w) : "v"(cvt_u32_sat(d)), "v"(k255));
    return w;
}

// copysign(0.49999997f, x) as one v_bitop3_b32 (select: magnitude bits from
// the constant, sign bit from x).  The compiler's copysign is a v_bfi_b32,
// which issues at ~1.6x the cost of a v_bitop3_b32 / v_fma_f32 on gfx950
// (tools/valu_rate.hip, profiles/r02/s4/valu_rate.log).
__device__ __forceinline__ float signed_half(float x) {
    return __uint_as_float(
        __builtin_amdgcn_bitop3_b32(0x7fffffffu, __float_as_uint(0.49999997f), __float_as_uint(x), 0xca));
}

// copysign(kMag, x) for a compile-time magnitude, one v_bitop3_b32
template <int kPos>
__device__ __forceinline__ float signed_bias(float x) {
    constexpr float kMag = quantforms::jpeg_bias(kPos);
    return __uint_as_float(
        __builtin_amdgcn_bitop3_b32(0x7fffffffu, __float_as_uint(kMag), __float_as_uint(x), 0xca));
}

// roundf (round half away from zero) in three operations:
//   trunc(x + copysign(0.49999997f, x))
// bit-identical to roundf for all 2^32 fp32 inputs (NaN stays NaN); checked
// exhaustively by tests/tools/verify_round3.c (tests/test_tools.py).
__device__ __forceinline__ float round_half_away(float x) {
    return __builtin_truncf(x + signed_half(x));
}

// the quotient C / Q (IEEE, or the verified 3-op form)
template <unsigned kVar>
__device__ __forceinline__ float quotient(float c, float q, float r) {
    if constexpr (kVar & kVarFastDiv) {
        const float q0 = c * r;
        const float e = __builtin_fmaf(-q0, q, c);
        return __builtin_fmaf(e, r, q0);
    } else {
        (void)r;
        return c / q;
    }
}

// int8 coefficients: round-half-away(d) = trunc(d + copysign(0.49999997, d))
// and v_cvt_i32_f32 truncates, so the trunc is folded into the conversion;
// each conversion writes its byte of the packed dword directly (SDWA dst_sel).
__device__ __forceinline__ uint32_t pack_q_i8x4(float a, float b, float c, float d) {
    auto biased = [](float x) { return x + signed_half(x); };
    uint32_t w;
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD"
                 : "=v"(w) : "v"(biased(a)));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(biased(b)));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(biased(c)));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(biased(d)));
    return w;
}

// v_cvt_i32_f32 (truncating) of an already-biased value straight into byte
// kByte of w, the other bytes preserved (SDWA dst_sel).
template <int kByte>
__device__ __forceinline__ void cvt_into_byte(uint32_t& w, float biased) {
    static_assert(kByte >= 0 && kByte < 4, "byte");
    if constexpr (kByte == 0)
        asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                     : "+v"(w) : "v"(biased));
    else if constexpr (kByte == 1)
        asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                     : "+v"(w) : "v"(biased));
    else if constexpr (kByte == 2)
        asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                     : "+v"(w) : "v"(biased));
    else
        asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                     : "+v"(w) : "v"(biased));
}

// divide_matrices (utils_kernels.cu:42): round(C / Q)
template <unsigned kVar>
__device__ __forceinline__ float quantise(float c, float q, float r) {
    float d;
    if constexpr (kVar & kVarFastDiv) {
        const float q0 = c * r;
        const float e = __builtin_fmaf(-q0, q, c);
        d = __builtin_fmaf(e, r, q0);
    } else {
        (void)r;
        d = c / q;  // IEEE (hipcc default: correctly rounded fp32 division)
    }
    return round_half_away(d);
}

// divide_matrices at table position kPos (= v * 8 + u), returned BEFORE the
// final truncation (the caller truncates: v_trunc_f32 for fp32 output, the
// truncating int8 convert for the wire format).  With kVarJpegQ the
// position's proven 3-op form where there is one (F or H), else the quotient
// (verified 3-op or IEEE) plus the signed 0.49999997 of the 3-op roundf.
template <unsigned kVar, int kPos>
__device__ __forceinline__ float quantise_biased_at(float c, float q, float r) {
    if constexpr ((kVar & kVarJpegQ) != 0 && quantforms::jpeg_form(kPos) != quantforms::kFull) {
        (void)q;
        return __builtin_fmaf(c, r, signed_bias<kPos>(c));
    } else {
        const float d = quotient<kVar>(c, q, r);
        return d + signed_half(d);
    }
}
template <unsigned kVar, int kPos>
__device__ __forceinline__ float quantise_at(float c, float q, float r) {
    return __builtin_truncf(quantise_biased_at<kVar, kPos>(c, q, r));
}

// int8 bytes of four already-biased values (truncating convert straight into
// each byte, SDWA dst_sel)
__device__ __forceinline__ uint32_t pack_biased_i8x4(float a, float b, float c, float d) {
    uint32_t w;
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD" : "=v"(w) : "v"(a));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(b));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(c));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "+v"(w) : "v"(d));
    return w;
}

// divide_matrices for one output row of 8 values per lane, kVarFastDivChecked:
// the verified 3-op quotient when the whole wave's row is within |C| <= 4096,
// IEEE division otherwise (a wave-uniform branch).
__device__ __forceinline__ void quantise_row_checked(float (&d)[8], const float (&q)[8], const float (&r)[8]) {
    float m = 0.0f;
    unroll<8>([&](auto u) { m = __builtin_fmaxf(m, __builtin_fabsf(d[u])); });
    // !(m <= 4096) also catches NaN (fmax drops a NaN operand, so test every value)
    bool bad = !(m <= 4096.0f);
    unroll<8>([&](auto u) { bad = bad || (d[u] != d[u]); });
    if (__builtin_amdgcn_ballot_w64(bad) == 0) {
        unroll<8>([&](auto u) { d[u] = quantise<kVarFastDiv>(d[u], q[u], r[u]); });
    } else {
        unroll<8>([&](auto u) { d[u] = quantise<0u>(d[u], q[u], r[u]); });
    }
}

// Tile-set geometry: lane's tile and the element offset of its top-left pixel.
struct TilePos {
    uint64_t base;
    bool valid;
};
__device__ __forceinline__ TilePos tile_pos(const TileGrid& g, uint32_t tile) {
    TilePos p;
    p.valid = tile < g.ntiles;
    const uint32_t t = p.valid ? tile : 0u;
    const uint32_t ty = t / g.tiles_x;
    const uint32_t tx = t - ty * g.tiles_x;
    p.base = static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(tx) * 8u;
    return p;
}

// ---- raw tile registers per input type ------------------------------------
template <typename TIn>
struct RawTile;

template <>
struct RawTile<uint8_t> {  // 8 rows x 8 bytes = 16 VGPRs
    uint2 r[8];
    __device__ __forceinline__ void load(const uint8_t* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) { r[i] = *reinterpret_cast<const uint2*>(p + i * width); });
    }
    __device__ __forceinline__ void to_float(float (&x)[8][8], float shift) const {
        unroll<8>([&](auto i) {
            unroll<4>([&](auto j) {
                x[i][j] = byte_f32(r[i].x, j) - shift;
                x[i][j + 4] = byte_f32(r[i].y, j) - shift;
            });
        });
    }
    // X - 128 exactly: (int8_t)(b ^ 0x80) == b - 128 for b in 0..255 (the round
    // trip's load; hipcc emits one SDWA sign-extending convert per pixel here).
    // Not used by the forward kernels: as their level shift it measured slower
    // than v_cvt_f32_ubyteK + v_sub_f32 for the int8 output (35.7-36.3 against
    // 32.1-33.3 us) and equal for fp32, despite 48 fewer VALU instructions per
    // set (round 3, profiles/r03/kb3_cvt*.log)
    __device__ __forceinline__ void to_float_minus128(float (&x)[8][8]) const {
        unroll<8>([&](auto i) {
            const uint32_t lo = r[i].x ^ 0x80808080u, hi = r[i].y ^ 0x80808080u;
            unroll<4>([&](auto j) {
                x[i][j] = static_cast<float>(static_cast<int32_t>(static_cast<int8_t>(lo >> (8 * j))));
                x[i][j + 4] = static_cast<float>(static_cast<int32_t>(static_cast<int8_t>(hi >> (8 * j))));
            });
        });
    }
};

template <>
struct RawTile<int8_t> {  // int8 coefficients, 16 VGPRs
    uint2 r[8];
    __device__ __forceinline__ void load(const int8_t* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) { r[i] = *reinterpret_cast<const uint2*>(p + i * width); });
    }
    __device__ __forceinline__ void to_float(float (&x)[8][8], float) const {
        unroll<8>([&](auto i) {
            unroll<4>([&](auto j) {
                x[i][j] = static_cast<float>(static_cast<int8_t>((r[i].x >> (8 * j)) & 0xffu));
                x[i][j + 4] = static_cast<float>(static_cast<int8_t>((r[i].y >> (8 * j)) & 0xffu));
            });
        });
    }
};

template <>
struct RawTile<float> {  // 64 VGPRs
    float4 r[8][2];
    __device__ __forceinline__ void load(const float* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) {
            const float4* src = reinterpret_cast<const float4*>(p + i * width);
            r[i][0] = src[0];
            r[i][1] = src[1];
        });
    }
    __device__ __forceinline__ void to_float(float (&x)[8][8], float shift) const {
        unroll<8>([&](auto i) {
            x[i][0] = r[i][0].x - shift;
            x[i][1] = r[i][0].y - shift;
            x[i][2] = r[i][0].z - shift;
            x[i][3] = r[i][0].w - shift;
            x[i][4] = r[i][1].x - shift;
            x[i][5] = r[i][1].y - shift;
            x[i][6] = r[i][1].z - shift;
            x[i][7] = r[i][1].w - shift;
        });
    }
};

template <bool kNT>
__device__ __forceinline__ void st(float4* p, const float4& v) {
    if constexpr (kNT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}
template <bool kNT>
__device__ __forceinline__ void st(uint2* p, const uint2& v) {
    if constexpr (kNT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
    } else {
        *p = v;
    }
}

// One output row of the lane's tile, written straight from the lane
// (32 B per lane for fp32: two dwordx4 that cover 2 KiB per wave together).
template <bool kNT, typename TOut>
__device__ __forceinline__ void store_row(TOut* __restrict__ row, const float (&c)[8]) {
    if constexpr (std::is_same_v<TOut, float>) {
        float4* dst = reinterpret_cast<float4*>(row);
        st<kNT>(dst, make_float4(c[0], c[1], c[2], c[3]));
        st<kNT>(dst + 1, make_float4(c[4], c[5], c[6], c[7]));
    } else if constexpr (std::is_same_v<TOut, int8_t>) {
        st<kNT>(reinterpret_cast<uint2*>(row),
                make_uint2(pack_i8x4(c[0], c[1], c[2], c[3]), pack_i8x4(c[4], c[5], c[6], c[7])));
    } else {  // uint8 pixels: clamp + truncate
        st<kNT>(reinterpret_cast<uint2*>(row),
                make_uint2(pack_u8x4(c[0], c[1], c[2], c[3]), pack_u8x4(c[4], c[5], c[6], c[7])));
    }
}

// fp32 row through a wave-private 2 KiB LDS slot: lane l deposits its 32 B
// at [32l, 32l+32), then lane j stores [16j, 16j+16) and [1024+16j, ...) of
// the 64-tile row segment starting at seg (= the row pixel of the set's
// first tile), i.e. two stores of 1 KiB contiguous each.  LDS accesses of
// one wave execute in order, so no barrier is needed between deposit and
// pick-up; the slot alternates with the row parity to let them overlap.
// 16-byte store at a byte offset from a wave-uniform base
template <bool kNT>
__device__ __forceinline__ void st_at(float* base, uint32_t off, const float4& v) {
    st<kNT>(reinterpret_cast<float4*>(reinterpret_cast<char*>(base) + off), v);
}

template <bool kNT>
__device__ __forceinline__ void store_row_lds(float4* __restrict__ slot, float* __restrict__ seg, uint32_t lane,
                                              const float (&c)[8]) {
    // slot index map (identity).  Written as a call on purpose: with the plain
    // expressions hipcc (ROCm 7.2) schedules the 64-bit address arithmetic of
    // the stores differently and the headline kernel grows by 29 instructions.
    auto ix = [](uint32_t k) { return k; };
    slot[ix(2 * lane)] = make_float4(c[0], c[1], c[2], c[3]);
    slot[ix(2 * lane + 1)] = make_float4(c[4], c[5], c[6], c[7]);
    const float4 a = slot[lane];
    const float4 b = slot[64 + lane];
    st_at<kNT>(seg, 16u * ix(lane), a);
    st_at<kNT>(seg, 16u * (64u + ix(lane)), b);
}

// The same for a set that straddles a tile-row boundary (ragged widths): its
// first k tiles end tile row ty (row segment at seg), the other 64-k start
// tile row ty+1, 7 * width + 8k elements further on.  Each store instruction
// then writes two contiguous runs instead of falling back to one 32-B store
// per lane.  float4 q holds half q%2 of tile q/2's row: tiles >= k lie
// 7 * width + 8k - 4 * 2k = 7 * width elements past the run they would
// continue, so every address is seg + 16 q bytes, plus jump = 28 * width
// bytes from q = 2k on: one SGPR base and a 32-bit lane offset per store
// (the offsets do not depend on the row, so they are computed once per set).
template <bool kNT>
__device__ __forceinline__ void store_row_lds2(float4* __restrict__ slot, float* __restrict__ seg, uint32_t jump,
                                               uint32_t k, uint32_t lane, const float (&c)[8]) {
    slot[2 * lane] = make_float4(c[0], c[1], c[2], c[3]);
    slot[2 * lane + 1] = make_float4(c[4], c[5], c[6], c[7]);
    const float4 a = slot[lane];
    const float4 b = slot[64 + lane];
    const uint32_t q0 = lane, q1 = 64u + lane, h = 2u * k;
    st_at<kNT>(seg, 16u * q0 + (q0 < h ? 0u : jump), a);
    st_at<kNT>(seg, 16u * q1 + (q1 < h ? 0u : jump), b);
}

// Per-wave walk over 64-tile sets: one set per wave, wave w = set w.
// body(raw, p, split, seg): split (wave-uniform) = 64 when the whole set is 64
// valid tiles of one tile row, whose row segments start at element seg; k in
// 1..63 when the set is 64 valid tiles whose first k end one tile row (at seg)
// and whose other 64-k start the next (RowSink derives that segment); 0 for a
// ragged last set or a set over more than two tile rows (per-lane stores).
template <unsigned kVar, typename TIn, typename Body>
__device__ __forceinline__ void walk_sets(const TIn* __restrict__ src, const TileGrid& g, float4* slots, Body&& body) {
    (void)slots;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
    const uint32_t nsets = (g.ntiles + 63u) / 64u;
    auto seg_info = [&](uint32_t set, const TilePos& p, uint64_t& seg) -> uint32_t {
        const uint32_t t0 = set * 64u;
        if constexpr ((kVar & kVarStraddle) == 0) {
            const bool ok = t0 + 63u < g.ntiles && (t0 / g.tiles_x) == ((t0 + 63u) / g.tiles_x);
            seg = p.base - 8u * static_cast<uint64_t>(lane);
            return ok ? 64u : 0u;
        }
        if (t0 + 63u >= g.ntiles) {
            seg = 0;
            return 0u;
        }
        const uint32_t ty0 = t0 / g.tiles_x, tx0 = t0 - ty0 * g.tiles_x;
        const uint32_t k = g.tiles_x - tx0;  // tiles of the set left in tile row ty0
        if (k >= 64u) {
            seg = p.base - 8u * static_cast<uint64_t>(lane);
            return 64u;
        }
        seg = static_cast<uint64_t>(ty0) * 8u * g.width + static_cast<uint64_t>(tx0) * 8u;
        return 64u - k <= g.tiles_x ? k : 0u;
    };
    if (wave >= nsets) return;
    TilePos p;
    uint64_t seg;
    uint32_t ok;
    p = tile_pos(g, wave * 64u + lane);
    ok = seg_info(wave, p, seg);
    if (!p.valid) return;
    RawTile<TIn> raw;
    raw.load(src + p.base, g.width);
    body(raw, p, ok, seg);
}

// Emits one row of 8 values for the lane's tile: through the LDS re-staging
// (fp32 planes, whole 64-tile sets) or straight from the lane.
template <unsigned kVar, typename TOut>
struct RowSink {
    static constexpr bool kNT = (kVar & kVarNT) != 0;
    static constexpr bool kLds = (kVar & kVarLdsStore) != 0 && std::is_same_v<TOut, float>;
    TOut* __restrict__ plane;
    uint64_t width;
    float4* slots;  // this wave's 2 x 128 float4 LDS slots (kLds)

    template <typename V>
    __device__ __forceinline__ void operator()(V v, const TilePos& p, uint32_t split, uint64_t seg,
                                               const float (&c)[8]) const {
        if constexpr (kLds) {
            if (split == 64u) {
                store_row_lds<kNT>(slots + (v & 1) * 128, plane + seg + v * width, threadIdx.x & 63u, c);
                return;
            }
            if ((kVar & kVarStraddle) != 0 && split != 0u) {
                // the next tile row's first tile: 7 * width + 8 split elements past seg (dense pitch)
                store_row_lds2<kNT>(slots + (v & 1) * 128, plane + seg + v * width,
                                    28u * static_cast<uint32_t>(width), split, threadIdx.x & 63u, c);
                return;
            }
        }
        store_row<kNT>(plane + p.base + v * width, c);
    }
};

// The wave's two 2 KiB LDS slots (the store re-staging).
template <unsigned kVar>
__device__ __forceinline__ float4* wave_slots() {
    if constexpr ((kVar & kVarLdsStore) != 0) {
        __shared__ float4 stage[kBlock<kVar> / 64u][2 * 128];
        return stage[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
    } else {
        return nullptr;
    }
}

// true (wave-uniform) when every live lane's tile holds only
// values with |v| < 2^125.  Then no operand is inf/NaN and no partial sum of
// the first pass can overflow (|T row|_1 <= 8 * 0.7072 < 8), so the
// products by the zero entries of T contribute exactly +0 to chains that
// start from +0 and may be skipped; otherwise 0*inf / 0*NaN must produce NaN
// as in the reference, and the full chain runs.
__device__ __forceinline__ bool wave_tame(const float (&x)[8][8]) {
    uint32_t m = 0;
    unroll<8>([&](auto i) {
        unroll<8>([&](auto j) { m = max(m, __float_as_uint(x[i][j]) & 0x7fffffffu); });
    });
    return __builtin_amdgcn_ballot_w64(m >= 0x7e000000u) == 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// Forward: image -> (quantised) coefficients.
// ---------------------------------------------------------------------------
// fdct_body's per-set work: level shift, transform, quantiser, row stores
template <typename TIn, typename TOut, bool kQuant, bool kWriteback, unsigned kVar, typename TS, typename Sink,
          typename WbSink>
__device__ __forceinline__ void fdct_tile_body(const RawTile<TIn>& raw, const TilePos& p, uint32_t ok, uint64_t seg,
                                               const TS& T, const Sink& sink, const WbSink& wb_sink,
                                               TOut* __restrict__ out, const TileGrid& g, const QParams& qp,
                                               float shift) {
    float x[8][8];
    raw.to_float(x, shift);
    if constexpr (kWriteback) {
        // the reference leaves X-128 in its input (main_newAppr.cu:273)
        unroll<8>([&](auto i) { wb_sink(i, p, ok, seg, x[i]); });
    }
    auto emit = [&](auto v, float (&c)[8]) {
        if constexpr (kQuant && std::is_same_v<TOut, int8_t> && (kVar & kVarI8Pack) != 0) {
            unroll<8>([&](auto u) {
                c[u] = quantise_biased_at<kVar, v * 8 + u>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]);
            });
            const uint2 w =
                make_uint2(pack_biased_i8x4(c[0], c[1], c[2], c[3]), pack_biased_i8x4(c[4], c[5], c[6], c[7]));
            st<(kVar & kVarNT) != 0>(reinterpret_cast<uint2*>(out + p.base + v * g.width), w);
            return;
        }
        if constexpr (kQuant) {
            unroll<8>([&](auto u) { c[u] = quantise_at<kVar, v * 8 + u>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
        }
        sink(v, p, ok, seg, c);
    };
    if constexpr ((kVar & kVarRowFirst) != 0) {
        fdct_tile_rowfirst(T, x, emit);
    } else {
        fdct_tile(T, x, emit);
    }
}

// Packed-fp32 forward of uint8 pixels with the built-in T, quantised to fp32
// (kVarPacked).  bquot2(v, k, c2) returns the biased quotient pair (before the
// truncation) of output columns (pair_u(k, 0), pair_u(k, 1)) of row v.  The
// kernels define bquot2 themselves
// over their own QParams argument: handing the QParams to a device function
// by reference made hipcc keep the quotient operands in scratch memory
// (364 B per lane, 4x slower).
template <unsigned kVar, typename TOut, typename BQuot2>
__device__ __forceinline__ void fdct_packed_body(const uint8_t* __restrict__ img, TOut* __restrict__ out,
                                                 const TileGrid& g, float shift, BQuot2&& bquot2) {
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, float> sink{reinterpret_cast<float*>(out), g.width, slots};
    walk_sets<kVar>(img, g, slots, [&](const RawTile<uint8_t>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
      auto work = [&](auto whole_run) {
        // whole runs: each row's two re-staged float4 are stored one row later,
        // so the LDS read's latency hides under the next row's arithmetic
        float4 pend_a = make_float4(0.f, 0.f, 0.f, 0.f), pend_b = pend_a;
        constexpr bool kNTs = (kVar & kVarNT) != 0;
        const uint32_t lane = threadIdx.x & 63u;
        float* const run0 = reinterpret_cast<float*>(out) + seg;
        float xs[8][8];
        raw.to_float(xs, 0.0f);
        f32x2 x2[8][4];  // X - 128, exact (integers)
        unroll<8>([&](auto i) {
            unroll<4>([&](auto cp) { x2[i][cp] = f32x2{xs[i][2 * cp], xs[i][2 * cp + 1]} - f32x2{shift, shift}; });
        });
        fdct_tile_pk(x2, [&](auto v, f32x2(&c2)[4]) {
            float c[8];
            unroll<4>([&](auto k) {
                const f32x2 d2 = bquot2(v, k, c2[k]);
                c[pair_u(k, 0)] = d2.x;
                c[pair_u(k, 1)] = d2.y;
            });
            if constexpr (std::is_same_v<TOut, int8_t>) {
                // the truncating int8 convert straight into each byte (wire format)
                const uint2 w =
                    make_uint2(pack_biased_i8x4(c[0], c[1], c[2], c[3]), pack_biased_i8x4(c[4], c[5], c[6], c[7]));
                st<(kVar & kVarNT) != 0>(reinterpret_cast<uint2*>(out + p.base + v * g.width), w);
            } else {
                unroll<8>([&](auto u) { c[u] = __builtin_truncf(c[u]); });
                if constexpr (decltype(whole_run)::value) {
                    float4* const slot = slots + (v & 1) * 128;
                    slot[2 * lane] = make_float4(c[0], c[1], c[2], c[3]);
                    slot[2 * lane + 1] = make_float4(c[4], c[5], c[6], c[7]);
                    const float4 a = slot[lane], b = slot[64 + lane];
                    if constexpr (v > 0) {
                        st_at<kNTs>(run0 + (v - 1) * g.width, 16u * lane, pend_a);
                        st_at<kNTs>(run0 + (v - 1) * g.width, 16u * (64u + lane), pend_b);
                    }
                    pend_a = a, pend_b = b;
                } else {
                    sink(v, p, ok, seg, c);
                }
            }
        });
        if constexpr (decltype(whole_run)::value) {
            st_at<kNTs>(run0 + 7u * g.width, 16u * lane, pend_a);
            st_at<kNTs>(run0 + 7u * g.width, 16u * (64u + lane), pend_b);
        }
      };
      if constexpr ((kVar & kVarHoistRun) != 0 && (kVar & kVarLdsStore) != 0 && std::is_same_v<TOut, float>) {
          if (ok == 64u) {
              work(std::true_type{});
          } else {
              work(std::false_type{});
          }
      } else {
          work(std::false_type{});
      }
    });
}

// round(C / Q) for one pair of output columns, before the truncation: with
// kVarJpegQ and a proven 3-op form at BOTH positions one packed fma with a
// per-half signed bias; otherwise the verified 3-op quotient per half (or
// IEEE division) and the signed 0.49999997 of the 3-op roundf
// (verify_round3.c).  A generic lambda in each kernel, over its own QParams.
#define HPDCT_PK_BQUOT2(kVar, qp)                                                                  \
    [&](auto v, auto k, f32x2 c2) -> f32x2 {                                                       \
        constexpr int u0 = pair_u(k, 0), u1 = pair_u(k, 1);                                        \
        constexpr int p0 = v * 8 + u0, p1 = v * 8 + u1;                                            \
        const f32x2 q2 = {qp.q.v[p0], qp.q.v[p1]};                                                 \
        if constexpr (((kVar) & kVarJpegQ) != 0 && quantforms::jpeg_form(p0) != quantforms::kFull && \
                      quantforms::jpeg_form(p1) != quantforms::kFull) {                            \
            (void)q2;                                                                              \
            const f32x2 r2 = {qp.r.v[p0], qp.r.v[p1]};                                             \
            return fma2(c2, r2, f32x2{signed_bias<p0>(c2.x), signed_bias<p1>(c2.y)});              \
        } else {                                                                                   \
            f32x2 d2;                                                                              \
            if constexpr (((kVar) & kVarFastDiv) != 0) {                                           \
                const f32x2 r2 = {qp.r.v[p0], qp.r.v[p1]};                                         \
                const f32x2 q0 = c2 * r2;                                                          \
                const f32x2 e = fma2(-q0, q2, c2);                                                 \
                d2 = fma2(e, r2, q0);                                                              \
            } else {                                                                               \
                d2 = f32x2{c2.x / q2.x, c2.y / q2.y};                                              \
            }                                                                                      \
            return d2 + f32x2{__builtin_copysignf(0.49999997f, d2.x), __builtin_copysignf(0.49999997f, d2.y)}; \
        }                                                                                          \
    }

template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback, unsigned kVar>
__device__ __forceinline__ void fdct_body(const TIn* __restrict__ img, TOut* __restrict__ out,
                                          float* __restrict__ shifted, const TileGrid& g,
                                          const float* __restrict__ t_dev, const QParams& qp, float shift) {
    // finite inputs (u8) may skip the zero terms of the built-in T
    constexpr bool kSkipZero = std::is_same_v<TIn, uint8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, TOut> sink{out, g.width, slots};
    const RowSink<kVar, float> wb_sink{shifted, g.width, slots};

    walk_sets<kVar>(img, g, slots, [&](const RawTile<TIn>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
        fdct_tile_body<TIn, TOut, kQuant, kWriteback, kVar>(raw, p, ok, seg, T, sink, wb_sink, out, g, qp, shift);
    });
}

template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>, 1) void fdct_kernel(const TIn* __restrict__ img, TOut* __restrict__ out,
                                                            float* __restrict__ shifted, TileGrid g,
                                                            const float* __restrict__ t_dev, QParams qp, float shift) {
    if constexpr ((kVar & kVarPacked) != 0 && std::is_same_v<TIn, uint8_t> &&
                  (std::is_same_v<TOut, float> || std::is_same_v<TOut, int8_t>) && kBuiltinT && kQuant &&
                  !kWriteback && (kVar & kVarRowFirst) == 0) {
        fdct_packed_body<kVar, TOut>(img, out, g, shift, HPDCT_PK_BQUOT2(kVar, qp));
    } else {
        fdct_body<TIn, TOut, kQuant, kBuiltinT, kWriteback, kVar>(img, out, shifted, g, t_dev, qp, shift);
    }
}

// A list of independent, equally sized uint8 frames in one launch
// (hpdct_forward_frames): frame blockIdx.y, its pointers from the table in
// the kernel arguments; per frame exactly fdct_kernel's work (built-in T,
// quantised, level shift 128), so the output is bit-identical to one launch
// per frame.
template <typename TOut, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>, 1) void fdct_frames_kernel(FrameTable<TOut> ft, TileGrid g, QParams qp) {
    const uint32_t f = blockIdx.y;
    if constexpr ((kVar & kVarPacked) != 0 && std::is_same_v<TOut, float>) {
        fdct_packed_body<kVar, TOut>(ft.in[f], ft.out[f], g, 128.0f, HPDCT_PK_BQUOT2(kVar, qp));
    } else {
        fdct_body<uint8_t, TOut, true, true, false, kVar>(ft.in[f], ft.out[f], nullptr, g, nullptr, qp, 128.0f);
    }
}

// ---------------------------------------------------------------------------
// Inverse: (quantised) coefficients -> image.
// ---------------------------------------------------------------------------
template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>, 1) void idct_kernel(const TIn* __restrict__ coef, TOut* __restrict__ out,
                                                            float* __restrict__ dq_out, TileGrid g,
                                                            const float* __restrict__ t_dev, Mat64 q, float shift) {
    constexpr bool kSkipZero = std::is_same_v<TIn, int8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, TOut> sink{out, g.width, slots};
    const RowSink<kVar, float> dq_sink{dq_out, g.width, slots};

    walk_sets<kVar>(coef, g, slots, [&](const RawTile<TIn>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
        float d[8][8];
        raw.to_float(d, 0.0f);
        if constexpr (kDequant) {
            // multiply_matrices (utils_kernels.cu:55): D = q * Q[i][j]
            unroll<8>([&](auto i) { unroll<8>([&](auto j) { d[i][j] = d[i][j] * q.v[i * 8 + j]; }); });
            if constexpr ((kVar & kVarWbDequant) != 0) {
                unroll<8>([&](auto i) { dq_sink(i, p, ok, seg, d[i]); });
            }
        }
        auto emit = [&](auto v, float (&r)[8]) {
            // add_matrix_scalar (utils_kernels.cu:29): R + 128, no clamp
            unroll<8>([&](auto u) { r[u] = r[u] + shift; });
            sink(v, p, ok, seg, r);
        };
        if constexpr ((kVar & kVarRowFirst) != 0) {
            idct_tile_rowfirst(T, d, emit);
        } else {
            idct_tile(T, d, emit);
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

[[maybe_unused]] static __global__ __launch_bounds__(kBlockThreads) void fill_hash_kernel(uint8_t* __restrict__ out, uint64_t n,
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

}  // namespace hpdct
