// kbench_variants.hpp -- TOOLS ONLY (tools/kbench.hip, tools/kbench2.hip):
// the tile-per-lane kernels with every measured A/B variant and phase-split
// diagnostic, kept so the DESIGN.md measurements can be re-run.  The library
// never includes this file; its kernels are the product subset in
// cuda-dct-idct_amd/csrc/hpdct_kernels_impl.hpp (same arithmetic, same bit
// values for the product variant flags).  Rejected variants and their
// measurements (DESIGN.md sections 4.2, 4.4, 8):
//   kVarPersist / kVarPersist2  persistent waves + next-set prefetch
//   kVarTwoSets                 two sets per wave, 16 row loads up front
//   kVarXorCvt                  (int8)(b ^ 0x80) byte convert
//   kVarRowMajor                forward rows finished one at a time
//   kVarLdsSwz / kVarLdsLoad    swizzled store slots / LDS-staged fp32 loads
//   kVarNTLoad                  non-temporal 8-bit loads
//   kVarStSc1 / kVarStSc0Sc1    store cache policies
//   kVarPacked                  packed-fp32 (v_pk_fma_f32) transform
//   kVarFiniteSkip              zero-term skip for finite fp32 tiles
//   kVarXcdSwz / kVarPanel      XCD-contiguous / column-panel set orders
//   bits 8..10                  minimum waves per SIMD for the register allocator
//   kVarNoLoad / kVarNoStore    diagnostics: phase split of the kernel time
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {
namespace ab {

// Compile-time kernel variants (bit flags).
enum : unsigned {
    kVarFastDiv = 1u,  // quotient by  q0=c*r; e=fma(-q0,Q,c); q=fma(e,r,q0)  (r = RN(1/Q)).  Gives the same
                       // roundf() as IEEE c/Q for every |c| <= 4096 and every integer Q in 1..255
                       // (exhaustive: tests/tools/verify_fastdiv.*); only enabled for such tables and
                       // uint8 input with the built-in T (|C| <= 1024).
    kVarPersist = 2u,  // persistent waves + prefetch of the next tile set
    kVarXorCvt = 4u,   // uint8 -> (x - 128) as (float)(int8_t)(b ^ 0x80): one XOR per 4 pixels + one
                       // sign-extending byte convert per pixel instead of convert + subtract
    kVarLdsStore = 8u, // fp32 rows re-staged through LDS so every store instruction writes 1 KiB contiguous
    kVarNT = 16u,      // non-temporal (streaming) stores for the output planes
    kVarRowMajor = 32u,  // forward: finish each P row and its C row before the next (fewer live VGPRs?)
    kVarLdsSwz = 64u,    // LDS re-staging with the slot swizzle k ^ ((k >> 3) & 1): conflict-free deposits
    kVarLdsLoad = 128u,  // fp32 inputs: 1 KiB-contiguous row loads, re-staged through LDS into the tile layout
    // bits 8..10: minimum waves per SIMD requested from the register allocator (0 = compiler default)
    // bits 12..13: workgroup size: 0 -> 256 threads, 1 -> 64, 2 -> 512, 3 -> 1024
    kVarRowFirst = 1u << 14,  // cublasDCTv2 pass order (row pass first), fp32 compat path
    kVarWbDequant = 1u << 15, // inverse: write q*Q back into the fp32 coefficient input
                              // (in-place multiply_matrices of main_cublass_2.cu:285)
    kVarNTLoad = 1u << 16,    // non-temporal loads of the 8-bit input planes
    kVarI8Pack = 1u << 17,    // int8 output: round-half-away folded into the truncating cvt, and each
                              // coefficient converted straight into its byte (SDWA dst_sel, one op)
    kVarPersist2 = 1u << 22,    // persistent waves, next set prefetched under a wave-uniform branch only
                                // (per-lane addresses clamped instead of divergent loads), so the
                                // compute of set n overlaps the loads of set n+1
    kVarTwoSets = 1u << 23,     // each wave takes two consecutive sets, all 16 row loads issued up front:
                                // the first set's compute overlaps the second set's loads
    kVarStSc1 = 1u << 24,       // fp32 re-staged stores as global_store_dwordx4 ... sc1 (with kVarNT: sc1 nt)
    kVarStSc0Sc1 = 1u << 25,    // ... sc0 sc1 (with kVarNT: sc0 sc1 nt)
    kVarPacked = 1u << 19,      // uint8 input, built-in T, quantised: packed-fp32 transform and quotient
                                // (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32, fdct_tile_pk)
    kVarFiniteSkip = 1u << 18,  // fp32 input, built-in T: per-wave finiteness test of the loaded tiles;
                                // all finite -> the zero terms of T are skipped (exact: a chain from +0
                                // never holds -0), otherwise the full chain (0*inf, 0*NaN -> NaN)
    // (1u << 26: the product's kVarFastDivChecked)
    // diagnostics only (tools/kbench): split the kernel's time into its phases
    kVarNoLoad = 1u << 27,      // tile bytes synthesised from the lane id instead of loaded
    kVarXcdSwz = 1u << 29,      // XCD-contiguous workgroup order: the hardware deals workgroups round-robin
                                // over the 8 XCDs; remap so XCD x walks one contiguous 1/8 of the sets
    kVarNoStore = 1u << 28,
    kVarPanel = 1u << 31,       // wide frames (tiles_x a multiple of 512, > 512): sets walk 4096-px-wide
                                // column panels top to bottom, panel after panel, instead of whole rows
    kVarStraddle = 1u << 30,    // fp32 LDS-staged rows: a 64-tile set that straddles two tile rows (width not a
                                // multiple of 512 px) stores two contiguous runs per instruction instead of
                                // 32 B per lane; launched only for such widths (the branch costs the
                                // power-of-two frames ~3 %, profiles/r01/ab_straddle.log)     // int8 rows stored only when ntiles == 0xffffffff (never): loads + math
};
// the tools-only A/B bits never alias a product-only bit
static_assert(((kVarPersist | kVarXorCvt | kVarRowMajor | kVarLdsSwz | kVarLdsLoad | kVarNTLoad | kVarPersist2 |
                kVarTwoSets | kVarStSc1 | kVarStSc0Sc1 | kVarFiniteSkip | kVarNoLoad | kVarXcdSwz | kVarNoStore |
                kVarPanel | (7u << 8)) &
               hpdct::kProductOnlyVarBits) == 0,
              "a tools A/B variant bit aliases a product-only kernel variant bit");
template <unsigned kVar>
constexpr unsigned kMinWaves = ((kVar >> 8) & 7u) ? ((kVar >> 8) & 7u) : 1u;  // bit 11: the product's kVarJpegQ
template <unsigned kVar>
constexpr uint32_t kBlock = ((kVar >> 12) & 3u) == 1u   ? 64u
                            : ((kVar >> 12) & 3u) == 2u ? 512u
                            : ((kVar >> 12) & 3u) == 3u ? 1024u
                                                        : kBlockThreads;


// ---- tile-level A/B variants (formerly in hpdct_tile.hpp) ------------------
// forward with each P row and its C row finished before the next (kVarRowMajor)
template <bool kRowMajor, typename TS, typename Emit>
__device__ __forceinline__ void fdct_tile_ab(const TS& T, float (&x)[8][8], Emit&& emit) {
    if constexpr (kRowMajor) {
        unroll<8>([&](auto v) {
            float p[8], c[8];
            unroll<8>([&](auto col) {
                float s = 0.0f;
                unroll<8>([&](auto i) { s = T.template mac<v * 8 + i>(x[i][col], s); });
                p[col] = s;
            });
            unroll<8>([&](auto u) {
                float s = 0.0f;
                unroll<8>([&](auto i) { s = T.template mac<u * 8 + i>(p[i], s); });
                c[u] = s;
            });
            emit(v, c);
        });
    } else {
        hpdct::fdct_tile(T, x, emit);
    }
}

// Packed-fp32 forward (kVarPacked; v_pk_fma_f32: two IEEE fmas per
// instruction, each half rounded exactly like the scalar v_fma_f32), built-in
// T, finite inputs.  Pass 1 pairs columns; pass 2 pairs output columns whose
// zero patterns of T coincide ((0,2) (4,6) (1,5) (3,7)); a term zero in one
// half only adds fma(0, P, s) = s exactly.  emit2(v, c2): c2[k] =
// {C[v][kPairU[k][0]], C[v][kPairU[k][1]]}.
typedef float f32x2 __attribute__((ext_vector_type(2)));
inline constexpr int kPairU[4][2] = {{0, 2}, {4, 6}, {1, 5}, {3, 7}};

__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename Emit2>
__device__ __forceinline__ void fdct_tile_pk(const f32x2 (&x2)[8][4], Emit2&& emit2) {
    f32x2 p2[8][4];
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
    unroll<8>([&](auto v) {
        f32x2 c2[4];
        unroll<4>([&](auto k) {
            constexpr int u0 = kPairU[k][0], u1 = kPairU[k][1];
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

// roundf (round half away from zero) in three operations:
//   trunc(x + copysign(0.49999997f, x))
// bit-identical to roundf for all 2^32 fp32 inputs (NaN stays NaN); checked
// exhaustively by tests/tools/verify_round3.c (tests/test_tools.py).
__device__ __forceinline__ float round_half_away(float x) {
    return __builtin_truncf(x + __builtin_copysignf(0.49999997f, x));
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
    auto biased = [](float x) { return x + __builtin_copysignf(0.49999997f, x); };
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
    // an empty asm that consumes every register: the loads must have landed
    // here (persistent walk: keeps the wait out of the pipelined loop)
    __device__ __forceinline__ void settle() {
        unroll<8>([&](auto i) { asm volatile("" : "+v"(r[i].x), "+v"(r[i].y)); });
    }
    __device__ __forceinline__ void load(const uint8_t* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) { r[i] = *reinterpret_cast<const uint2*>(p + i * width); });
    }
    __device__ __forceinline__ void load_nt(const uint8_t* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) {
            const uint2* q = reinterpret_cast<const uint2*>(p + i * width);
            r[i].x = __builtin_nontemporal_load(&q->x);
            r[i].y = __builtin_nontemporal_load(&q->y);
        });
    }
    __device__ __forceinline__ void to_float(float (&x)[8][8], float shift) const {
        unroll<8>([&](auto i) {
            unroll<4>([&](auto j) {
                x[i][j] = byte_f32(r[i].x, j) - shift;
                x[i][j + 4] = byte_f32(r[i].y, j) - shift;
            });
        });
    }
    // X - 128 exactly: (int8_t)(b ^ 0x80) == b - 128 for b in 0..255
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
    __device__ __forceinline__ void settle() {
        unroll<8>([&](auto i) { asm volatile("" : "+v"(r[i].x), "+v"(r[i].y)); });
    }
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
struct RawTile<float> {
    __device__ __forceinline__ void settle() {
        unroll<16>([&](auto n) {
            float4& v = r[n / 2][n % 2];
            asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
        });
    }  // 64 VGPRs
    float4 r[8][2];
    __device__ __forceinline__ void load(const float* __restrict__ p, uint64_t width) {
        unroll<8>([&](auto i) {
            const float4* src = reinterpret_cast<const float4*>(p + i * width);
            r[i][0] = src[0];
            r[i][1] = src[1];
        });
    }
    // Whole 64-tile set in one tile row: lane j loads 16 B at [16j, 16j+16) and
    // [1024+16j, ...) of each 2 KiB row segment (two 1 KiB-contiguous loads per
    // row), the rows pass through the wave's LDS slots and every lane picks up
    // its own tile's 32 B.  In-order LDS within one wave: no barrier.
    __device__ __forceinline__ void load_staged(const float* __restrict__ seg, uint64_t width, uint32_t lane,
                                                float4* __restrict__ slots) {
        float4 a[8], b[8];
        unroll<8>([&](auto i) {
            const float4* src = reinterpret_cast<const float4*>(seg + i * width);
            a[i] = src[lane];
            b[i] = src[64 + lane];
        });
        unroll<8>([&](auto i) {
            float4* slot = slots + (i & 1) * 128;
            slot[lane] = a[i];
            slot[64 + lane] = b[i];
            r[i][0] = slot[2 * lane];
            r[i][1] = slot[2 * lane + 1];
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
// Optional slot swizzle sw(k) = k ^ ((k >> 3) & 1) (an involution that keeps
// [0,64) and [64,128)): the deposits of 8 consecutive lanes then hit 8
// distinct 16-B bank groups; the pick-up of slot j stores to position sw(j).
// 16-byte store with an explicit cache policy (kPol: 0 = st<kNT>, 1 = sc1,
// 2 = sc0 sc1; kNT adds nt) through a raw buffer store, whose aux operand
// carries the gfx940+ cache-policy bits (sc0 = 1, nt = 2, sc1 = 16); inline
// asm is not an option: the compiler would not track the store's read of its
// data registers.  `base` is wave-uniform, `off` the lane's byte offset.
template <bool kNT, int kPol>
__device__ __forceinline__ void st_pol(float* base, uint32_t off, const float4& v) {
    if constexpr (kPol == 0) {
        st<kNT>(reinterpret_cast<float4*>(reinterpret_cast<char*>(base) + off), v);
    } else {
        constexpr int kAux = (kPol == 1 ? 16 : 17) | (kNT ? 2 : 0);
        typedef int v4i __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
        const v4i w = {__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(w, rsrc, off, 0, kAux);
    }
}

template <bool kNT, bool kSwz, int kPol = 0>
__device__ __forceinline__ void store_row_lds(float4* __restrict__ slot, float* __restrict__ seg, uint32_t lane,
                                              const float (&c)[8]) {
    auto sw = [](uint32_t k) { return kSwz ? (k ^ ((k >> 3) & 1u)) : k; };
    slot[sw(2 * lane)] = make_float4(c[0], c[1], c[2], c[3]);
    slot[sw(2 * lane + 1)] = make_float4(c[4], c[5], c[6], c[7]);
    const float4 a = slot[lane];
    const float4 b = slot[64 + lane];
    st_pol<kNT, kPol>(seg, 16u * sw(lane), a);
    st_pol<kNT, kPol>(seg, 16u * (64u + sw(lane)), b);
}

// The same for a set that straddles a tile-row boundary (ragged widths): its
// first k tiles end tile row ty (row segment at seg), the other 64-k start
// tile row ty+1 (at seg2).  Each store instruction then writes two contiguous
// runs instead of falling back to one 32-B store per lane.
template <bool kNT>
__device__ __forceinline__ void store_row_lds2(float4* __restrict__ slot, float* __restrict__ seg,
                                               float* __restrict__ seg2, uint32_t k, uint32_t lane,
                                               const float (&c)[8]) {
    slot[2 * lane] = make_float4(c[0], c[1], c[2], c[3]);
    slot[2 * lane + 1] = make_float4(c[4], c[5], c[6], c[7]);
    const float4 a = slot[lane];
    const float4 b = slot[64 + lane];
    // float4 q holds half q%2 of tile q/2's row: tiles < k go to seg, the rest to seg2
    const uint32_t q0 = lane, q1 = 64u + lane, h = 2u * k;
    st<kNT>(reinterpret_cast<float4*>(q0 < h ? seg + 4u * q0 : seg2 + 4u * (q0 - h)), a);
    st<kNT>(reinterpret_cast<float4*>(q1 < h ? seg + 4u * q1 : seg2 + 4u * (q1 - h)), b);
}

// Per-wave walk over 64-tile sets: one set per wave (plain), or a grid-stride
// loop with the next set's loads issued before the current set's compute.
// body(raw, p, split, seg): split (wave-uniform) = 64 when the whole set is 64
// valid tiles of one tile row, whose row segments start at element seg; k in
// 1..63 when the set is 64 valid tiles whose first k end one tile row (at seg)
// and whose other 64-k start the next (RowSink derives that segment); 0 for a
// ragged last set or a set over more than two tile rows (per-lane stores).
template <unsigned kVar, typename TIn, typename Body>
__device__ __forceinline__ void walk_sets(const TIn* __restrict__ src, const TileGrid& g, float4* slots, Body&& body) {
    constexpr bool kPersist = (kVar & kVarPersist) != 0;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t block = blockIdx.x;
    if constexpr ((kVar & kVarXcdSwz) != 0) {
        // bijective: XCD x = block % 8 owns q (+1 for x < r) consecutive blocks
        const uint32_t nb = gridDim.x, q = nb / 8u, r = nb % 8u, x = block % 8u;
        block = x * q + (x < r ? x : r) + block / 8u;
    }
    const uint32_t wave = __builtin_amdgcn_readfirstlane(block * (kBlock<kVar> / 64u) + threadIdx.x / 64u);
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
    if constexpr ((kVar & kVarTwoSets) != 0) {
        const uint32_t s0 = wave * 2u;
        if (s0 >= nsets) return;
        auto clamp_tile = [&](uint32_t s_) {
            uint32_t t = s_ * 64u + lane;
            return t < g.ntiles ? t : g.ntiles - 1u;  // lanes past the end redo the last tile (same bytes)
        };
        RawTile<TIn> a, b;
        const TilePos pa = tile_pos(g, clamp_tile(s0)), pb = tile_pos(g, clamp_tile(s0 + 1u));
        a.load(src + pa.base, g.width);
        b.load(src + pb.base, g.width);
        uint64_t seg;
        uint32_t ok = seg_info(s0, pa, seg);
        body(a, pa, ok, seg);
        if (s0 + 1u < nsets) {  // wave-uniform
            ok = seg_info(s0 + 1u, pb, seg);
            body(b, pb, ok, seg);
        }
    } else if constexpr ((kVar & kVarPersist2) != 0) {
        const uint32_t nwaves = gridDim.x * (kBlock<kVar> / 64u);
        uint32_t set = wave;
        if (set >= nsets) return;
        auto load_set = [&](RawTile<TIn>& r, uint32_t s_) {
            uint32_t t = s_ * 64u + lane;
            if (t >= g.ntiles) t = g.ntiles - 1u;  // clamp: every lane loads, no divergent load
            r.load(src + tile_pos(g, t).base, g.width);
        };
        RawTile<TIn> cur;
        load_set(cur, set);
        cur.settle();  // first set waited here, once: no load of it is pending at the loop header
        while (true) {
            const uint32_t nset = set + nwaves;
            const bool more = nset < nsets;  // wave-uniform
            RawTile<TIn> nxt;
            if (more) load_set(nxt, nset);
            // lanes past the last tile run the body on their clamped tile (the
            // last valid one): they store byte-identical values to the same
            // addresses, so the loop body has no divergent branch and the
            // wait for the next set's loads does not have to drain the stores
            uint32_t t = set * 64u + lane;
            if (t >= g.ntiles) t = g.ntiles - 1u;
            const TilePos p = tile_pos(g, t);
            uint64_t seg;
            const uint32_t ok = seg_info(set, p, seg);
            body(cur, p, ok, seg);
            if (!more) break;
            cur = nxt;
            set = nset;
        }
    } else if constexpr (!kPersist) {
        if (wave >= nsets) return;
        TilePos p;
        uint64_t seg;
        uint32_t ok;
        constexpr uint32_t kPanelTiles = 512u;
        if ((kVar & kVarPanel) != 0 && g.tiles_x % kPanelTiles == 0u && g.tiles_x > kPanelTiles) {
            // set -> (panel, tile row, 64-tile chunk): every set is 64 tiles of one tile row
            constexpr uint32_t kSpr = kPanelTiles / 64u;
            const uint32_t per_panel = kSpr * (g.ntiles / g.tiles_x);
            const uint32_t pn = wave / per_panel, r = wave - pn * per_panel;
            const uint32_t ty = r / kSpr, cx = r - ty * kSpr;
            p.valid = true;
            seg = static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(pn * kPanelTiles + cx * 64u) * 8u;
            p.base = seg + 8u * static_cast<uint64_t>(lane);
            ok = 64u;
        } else {
            p = tile_pos(g, wave * 64u + lane);
            ok = seg_info(wave, p, seg);
        }
        if (!p.valid) return;
        RawTile<TIn> raw;
        if constexpr ((kVar & kVarNoLoad) != 0 && sizeof(TIn) == 1) {
            unroll<8>([&](auto i) {
                raw.r[i] = make_uint2((lane * 0x01010101u) ^ (i * 0x10325476u), (lane * 0x03050709u) + i);
            });
        } else if constexpr ((kVar & kVarLdsLoad) != 0 && std::is_same_v<TIn, float>) {
            if (ok == 64u) {
                raw.load_staged(src + seg, g.width, lane, slots);
            } else {
                raw.load(src + p.base, g.width);
            }
        } else if constexpr ((kVar & kVarNTLoad) != 0 && std::is_same_v<TIn, uint8_t>) {
            raw.load_nt(src + p.base, g.width);
        } else {
            raw.load(src + p.base, g.width);
        }
        body(raw, p, ok, seg);
    } else {
        const uint32_t nwaves = gridDim.x * (kBlock<kVar> / 64u);
        uint32_t set = wave;
        if (set >= nsets) return;
        TilePos p = tile_pos(g, set * 64u + lane);
        RawTile<TIn> cur;
        if (p.valid) cur.load(src + p.base, g.width);
        while (true) {
            const uint32_t nset = set + nwaves;
            const bool more = nset < nsets;  // wave-uniform
            TilePos np = p;
            RawTile<TIn> nxt;
            if (more) {
                np = tile_pos(g, nset * 64u + lane);
                if (np.valid) nxt.load(src + np.base, g.width);
            }
            uint64_t seg;
            const uint32_t ok = seg_info(set, p, seg);
            if (p.valid) body(cur, p, ok, seg);
            if (!more) break;
            cur = nxt;
            p = np;
            set = nset;
        }
    }
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
                constexpr int kPol = (kVar & kVarStSc1) ? 1 : (kVar & kVarStSc0Sc1) ? 2 : 0;
                store_row_lds<kNT, (kVar & kVarLdsSwz) != 0, kPol>(slots + (v & 1) * 128,
                                                                   plane + seg + v * width, threadIdx.x & 63u, c);
                return;
            }
            if ((kVar & kVarStraddle) != 0 && split != 0u) {
                // next tile row's first tile: seg - (width - 8k) + 8 width (dense pitch: tiles_x = width / 8)
                const uint64_t seg2 = seg + 7u * width + 8u * split;
                store_row_lds2<kNT>(slots + (v & 1) * 128, plane + seg + v * width, plane + seg2 + v * width, split,
                                    threadIdx.x & 63u, c);
                return;
            }
        }
        store_row<kNT>(plane + p.base + v * width, c);
    }
};

// The wave's two 2 KiB LDS slots (used by the store and load re-staging).
template <unsigned kVar>
__device__ __forceinline__ float4* wave_slots() {
    if constexpr ((kVar & (kVarLdsStore | kVarLdsLoad)) != 0) {
        __shared__ float4 stage[kBlock<kVar> / 64u][2 * 128];
        return stage[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
    } else {
        return nullptr;
    }
}

// kVarFiniteSkip: true (wave-uniform) when every live lane's tile holds only
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
template <typename TIn, typename TOut, bool kQuant, bool kBuiltinT, bool kWriteback, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>, kMinWaves<kVar>) void fdct_kernel(const TIn* __restrict__ img, TOut* __restrict__ out,
                                                             float* __restrict__ shifted, TileGrid g,
                                                             const float* __restrict__ t_dev, QParams qp,
                                                             float shift) {
    // finite inputs (u8) may skip the zero terms of the built-in T
    constexpr bool kSkipZero = std::is_same_v<TIn, uint8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, TOut> sink{out, g.width, slots};
    const RowSink<kVar, float> wb_sink{shifted, g.width, slots};

    walk_sets<kVar>(img, g, slots, [&](const RawTile<TIn>& raw, const TilePos& p, uint32_t ok,
                                                      uint64_t seg) {
        if constexpr ((kVar & kVarPacked) != 0 && std::is_same_v<TIn, uint8_t> && kBuiltinT && kQuant &&
                      !kWriteback && (kVar & kVarRowFirst) == 0) {
            float xs[8][8];
            raw.to_float(xs, 0.0f);
            f32x2 x2[8][4];
            unroll<8>([&](auto i) {
                unroll<4>([&](auto cp) { x2[i][cp] = f32x2{xs[i][2 * cp], xs[i][2 * cp + 1]} - f32x2{shift, shift}; });
            });
            fdct_tile_pk(x2, [&](auto v, f32x2(&c2)[4]) {
                // quotient per pair: the verified 3-op form (packed) or IEEE division
                f32x2 d2[4];
                unroll<4>([&](auto k) {
                    constexpr int u0 = kPairU[k][0], u1 = kPairU[k][1];
                    const f32x2 q2 = {qp.q.v[v * 8 + u0], qp.q.v[v * 8 + u1]};
                    if constexpr ((kVar & kVarFastDiv) != 0) {
                        const f32x2 r2 = {qp.r.v[v * 8 + u0], qp.r.v[v * 8 + u1]};
                        const f32x2 q0 = c2[k] * r2;
                        const f32x2 e = fma2(-q0, q2, c2[k]);
                        d2[k] = fma2(e, r2, q0);
                    } else {
                        d2[k] = f32x2{c2[k].x / q2.x, c2[k].y / q2.y};
                    }
                    // round half away: trunc(d + copysign(0.49999997, d)) (verify_round3.c)
                    d2[k] = d2[k] + f32x2{__builtin_copysignf(0.49999997f, d2[k].x),
                                          __builtin_copysignf(0.49999997f, d2[k].y)};
                });
                if constexpr (std::is_same_v<TOut, int8_t>) {
                    uint32_t w[2] = {0u, 0u};
                    unroll<4>([&](auto k) {
                        constexpr int u0 = kPairU[k][0], u1 = kPairU[k][1];
                        cvt_into_byte<u0 % 4>(w[u0 / 4], d2[k].x);
                        cvt_into_byte<u1 % 4>(w[u1 / 4], d2[k].y);
                    });
                    st<(kVar & kVarNT) != 0>(reinterpret_cast<uint2*>(out + p.base + v * g.width),
                                             make_uint2(w[0], w[1]));
                } else {
                    float c[8];
                    unroll<4>([&](auto k) {
                        c[kPairU[k][0]] = __builtin_truncf(d2[k].x);
                        c[kPairU[k][1]] = __builtin_truncf(d2[k].y);
                    });
                    sink(v, p, ok, seg, c);
                }
            });
            return;
        }
        float x[8][8];
        if constexpr ((kVar & kVarXorCvt) != 0 && std::is_same_v<TIn, uint8_t>) {
            raw.to_float_minus128(x);  // launcher guarantees shift == 128
        } else {
            raw.to_float(x, shift);
        }
        if constexpr (kWriteback) {
            // the reference leaves X-128 in its input (main_newAppr.cu:273)
            unroll<8>([&](auto i) { wb_sink(i, p, ok, seg, x[i]); });
        }
        auto emit = [&](auto v, float (&c)[8]) {
            if constexpr (kQuant && std::is_same_v<TOut, int8_t> && (kVar & kVarI8Pack) != 0) {
                unroll<8>([&](auto u) { c[u] = quotient<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
                const uint2 w = make_uint2(pack_q_i8x4(c[0], c[1], c[2], c[3]), pack_q_i8x4(c[4], c[5], c[6], c[7]));
                if constexpr ((kVar & kVarNoStore) != 0) {
                    if (g.ntiles != 0xffffffffu) return;
                }
                st<(kVar & kVarNT) != 0>(reinterpret_cast<uint2*>(out + p.base + v * g.width), w);
                return;
            }
            if constexpr (kQuant) {
                unroll<8>([&](auto u) { c[u] = quantise<kVar>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
            }
            sink(v, p, ok, seg, c);
        };
        if constexpr ((kVar & kVarRowFirst) != 0) {
            fdct_tile_rowfirst(T, x, emit);
        } else if constexpr ((kVar & kVarFiniteSkip) != 0 && kBuiltinT && !kSkipZero) {
            if (wave_tame(x)) {
                fdct_tile_ab<(kVar & kVarRowMajor) != 0>(TSource<true, true>(t_dev), x, emit);
            } else {
                fdct_tile_ab<(kVar & kVarRowMajor) != 0>(T, x, emit);
            }
        } else {
            fdct_tile_ab<(kVar & kVarRowMajor) != 0>(T, x, emit);
        }
    });
}

// ---------------------------------------------------------------------------
// Inverse: (quantised) coefficients -> image.
// ---------------------------------------------------------------------------
template <typename TIn, typename TOut, bool kDequant, bool kBuiltinT, unsigned kVar>
__global__ __launch_bounds__(kBlock<kVar>, kMinWaves<kVar>) void idct_kernel(const TIn* __restrict__ coef, TOut* __restrict__ out,
                                                             float* __restrict__ dq_out, TileGrid g,
                                                             const float* __restrict__ t_dev, Mat64 q, float shift) {
    constexpr bool kSkipZero = std::is_same_v<TIn, int8_t>;
    const TSource<kBuiltinT, kSkipZero> T(t_dev);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, TOut> sink{out, g.width, slots};
    const RowSink<kVar, float> dq_sink{dq_out, g.width, slots};

    walk_sets<kVar>(coef, g, slots, [&](const RawTile<TIn>& raw, const TilePos& p, uint32_t ok,
                                                       uint64_t seg) {
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
        } else if constexpr ((kVar & kVarFiniteSkip) != 0 && kBuiltinT && !kSkipZero) {
            if (wave_tame(d)) {
                idct_tile(TSource<true, true>(t_dev), d, emit);
            } else {
                idct_tile(T, d, emit);
            }
        } else {
            idct_tile(T, d, emit);
        }
    });
}

}  // namespace ab
}  // namespace hpdct
