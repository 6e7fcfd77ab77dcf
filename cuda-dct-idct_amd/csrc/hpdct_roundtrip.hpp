// hpdct_roundtrip.hpp -- the C3 round trip in one HBM pass: uint8 frame ->
// fp32 quantised coefficients + reconstruction (+ the PEEN/MSE sums), for
// CDNA4 / gfx950.
//
// The reference runs a round trip as dct_all_blocks_cuda then
// idct_all_blocks_cuda (main_newAppr.cu:99,120; benchmark_newAppr.cu:93,105),
// six launches and three fp32 planes through HBM each way; the quality check
// (README.md:62-69) happens on the host.  Here one lane keeps its 8x8 tile in
// VGPRs from the pixel load to the reconstructed pixel: the forward emits each
// quantised row (stored as the fp32 coefficient row) and keeps it as 8 packed
// int8 values; the inverse starts from those registers.  Arithmetic is the
// forward kernel's followed by the inverse kernel's, so coefficients and
// reconstruction are bit-identical to hpdct_forward + hpdct_inverse.
//
// HBM per pixel: 1 B read + 4 B coefficients (+ 1 B uint8 or 4 B fp32
// reconstruction) written, against 1 + 4 + 4 + 1 for the two kernels.
//
// Quality sums (kStats), per frame, as hpdct_quality.py defines them:
//   sum_x2  = sum x^2                       exact: v_dot4_u32_u8 on the packed
//   sse_u8  = sum (x - u8(R+128))^2        pixel bytes (x.x, x.r8, r8.r8), uint64
//   sse_f32 = sum (x - (R+128))^2          per tile FOUR fp32 fma chains, one per
//             (row parity, column parity) class of its pixels, each in row-major
//             order from +0, each rounded to a multiple of 2^-16 (rt_sse_fix)
//             and added as uint64: the result does not depend on the order tiles
//             finish in, but it is not the exact sum (relative error ~1e-10 at
//             8192^2, tests/test_gpu_roundtrip.py).  Four classes since round 5:
//             the two-lanes-per-tile kernel (hpdct_rt_duo.hpp) holds the rows of
//             one parity per lane and the columns of one parity per half of a
//             packed register, so its chains need no cross-lane hand-off; this
//             kernel keeps the same four chains, so both give the same sums.
// Workgroup partials are added with one 64-bit atomic per field per workgroup,
// into the caller's struct or sub-slot 0 of a library spread slot that
// rt_spread_finish_kernel then folds into the caller's struct.
#pragma once

#include "hpdct_kernels_impl.hpp"

namespace hpdct {

constexpr float kRtFixScale = 65536.0f;  // sse_f32 fixed point: 2^-16
// bit 63 of sse_f32_fx: some tile's sse_f32 was non-finite or >= 2^24 (the
// field then holds no sum; include/hpdct.h HPDCT_SSE_F32_INVALID)
constexpr unsigned long long kRtSseF32Invalid = 1ull << 63;

// sse_f32 of one fp32 chain in fixed point (units 2^-16): ok stays true when
// the chain is finite and below 2^24 (fixed point below 2^40), otherwise the
// chain adds nothing and ok turns false (the caller then sets
// kRtSseF32Invalid, so the field can neither wrap nor read as a small value).
__device__ __forceinline__ unsigned long long rt_sse_fix(float chain, bool& ok) {
    const float fx = __builtin_rintf(chain * kRtFixScale);
    const bool good = fx < 0x1p40f;  // false for NaN
    ok = ok && good;
    return good ? static_cast<unsigned long long>(fx) : 0ull;
}

// The spread slot of the sums (round 5): kRtSpread sub-slots of 3 x uint64,
// kRtSpreadStride words (256 B) apart, so that the atomics of many waves land
// on kRtSpread different lines; rt_spread_finish_kernel folds them.
constexpr int kRtSpread = 64;
constexpr uint32_t kRtSpreadStride = 32;
constexpr size_t kRtSpreadBytes = kRtSpread * kRtSpreadStride * sizeof(unsigned long long);

namespace {

// unpack int8 byte k of w into an exact float (sign-extending byte convert)
__device__ __forceinline__ float i8_byte_f32(uint32_t w, int k) {
    return static_cast<float>(static_cast<int8_t>((w >> (8 * k)) & 0xffu));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    unroll<6>([&](auto s) { v += __shfl_xor(v, 1 << s, 64); });
    return v;
}

// Sum over the wave in DPP steps (row_shr 1, 2, 4, 8 inside each 16-lane row,
// then row_bcast 15 and 31 across rows): lane 63 ends with the total, read
// back with one readlane.  No LDS traffic, unlike __shfl_xor.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), kCtrl, kRowMask, 0xf, false));
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void dpp_add(uint32_t& v) {
    v += dpp_u32<kCtrl, kRowMask>(v);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void dpp_add(unsigned long long& v) {
    const uint32_t lo = dpp_u32<kCtrl, kRowMask>(static_cast<uint32_t>(v));
    const uint32_t hi = dpp_u32<kCtrl, kRowMask>(static_cast<uint32_t>(v >> 32));
    v += (static_cast<unsigned long long>(hi) << 32) | lo;
}
template <typename U>
__device__ __forceinline__ U wave_sum_dpp(U v) {
    dpp_add<0x111, 0xf>(v);  // row_shr:1
    dpp_add<0x112, 0xf>(v);  // row_shr:2
    dpp_add<0x114, 0xf>(v);  // row_shr:4
    dpp_add<0x118, 0xf>(v);  // row_shr:8
    dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    if constexpr (sizeof(U) == 8) {
        const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v)), 63));
        const uint32_t hi =
            static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v >> 32)), 63));
        return (static_cast<unsigned long long>(hi) << 32) | lo;
    } else {
        return static_cast<U>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
    }
}

}  // namespace

// kFast: integer table in 1..255 whose quotients fit int8 (library QState
// fastdiv_ok && int8_ok): the verified 3-op quotient and the quantised rows
// kept as packed int8 (16 VGPRs).  Otherwise IEEE division and the rows kept
// as fp32 (64 VGPRs).
// 512-thread workgroups, at least 4 waves per SIMD (<= 128 VGPRs: two
// workgroups per CU); 2 with an fp32 reconstruction (its row re-staging needs
// more registers than 128 without spilling).
// kRaw: where the sums find the pixels again at the inverse's output rows:
//   0  the loaded tile kept in VGPRs through both transforms (16 VGPRs)
//   1  re-read from global memory when the inverse starts (the wave read those
//      4 KiB microseconds earlier: served by L2 / Infinity Cache)
//   2  stashed in LDS after the load (4 KiB per wave): the product
// (8192^2, u8 reconstruction + sums: 89.1 / 82.7 / 72.5 us; no sums 65 us;
// profiles/r01/mappings/kbench2_rt.log)
template <int kRecon>
constexpr int kRtWaves = kRecon == kRtReconF32 ? 2 : 4;
// Epilogue: one 64-bit atomic add per field per workgroup into the caller's
// struct.  Measured alternatives (round 3, profiles/r03/kb_rt16.log, 8192^2):
// one struct per workgroup (no two workgroups on one line) 78.4-78.8 us
// against 79.7 us; per-wave atomics 607 us.
// kQMode: 0 IEEE division (kFast false), 1 the verified 3-op quotient (kFast),
// 2 as 1 with the default JPEG table's per-position 3-op forms (kVarJpegQ).
// kBlock: threads per workgroup.  256 since round 4 (8192^2, u8 recon: 77.9-78.3
// against 78.6-80.7 us with sums, 68.8 against 70.8 without, 1024: 87.0;
// profiles/r04/b/kb3_jqrtb_8192.log)
constexpr int kRtBlock = 256;
template <int kRecon, bool kStats, int kQMode, int kRaw = 2, bool kStraddle = false, int kBlock = kRtBlock>
__global__ __launch_bounds__(kBlock, kRtWaves<kRecon>) void roundtrip_kernel(const uint8_t* __restrict__ img,
                                                                          float* __restrict__ coef,
                                                                          void* __restrict__ recon,
                                                                          RtSums* __restrict__ sums, TileGrid g,
                                                                          QParams qp) {
    constexpr bool kFast = kQMode != 0;
    static_assert(kBlock == 256 || kBlock == 512 || kBlock == 1024, "workgroup size");
    constexpr unsigned kBlockBits = kBlock == 256 ? 0u : kBlock == 512 ? 2u : 3u;
    constexpr unsigned kVar = (kBlockBits << 12) | kVarNT | kVarLdsStore | (kFast ? kVarFastDiv : 0u) |
                              (kQMode == 2 ? kVarJpegQ : 0u) | (kStraddle ? kVarStraddle : 0u);
    // built-in T.  The forward's u8 pixels are finite, so the zero terms of T
    // are skipped exactly; so are the inverse's for kFast (int8-range q times
    // Q in 1..255).  With IEEE division and a caller's table, q = round(C/Q)
    // may be +-inf (|Q| tiny): then the inverse runs the full chain, where
    // 0 * inf = NaN as in the reference and the standalone fp32 inverse.
    const TSource<true, true> T(nullptr);
    const TSource<true, false> T_full(nullptr);
    float4* const slots = wave_slots<kVar>();
    const RowSink<kVar, float> coef_sink{coef, g.width, slots};
    const RowSink<kVar, float> rf32_sink{static_cast<float*>(recon), g.width, slots};
    float acc_f[2][2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};  // this lane's tile: the four sse_f32 chains
    uint32_t acc_xx = 0u, acc_xr = 0u, acc_rr = 0u;  // sum x^2, x.r8, r8^2 (<= 64 * 255^2)

    uint2* stash = nullptr;  // kRaw == 2: this wave's [row][lane] pixel words
    if constexpr (kStats && kRaw == 2) {
        __shared__ uint2 raw_lds[kBlock / 64][8 * 64];
        stash = raw_lds[__builtin_amdgcn_readfirstlane(threadIdx.x / 64u)];
    }
    const uint32_t lane = threadIdx.x & 63u;

    walk_sets<kVar>(img, g, slots, [&](const RawTile<uint8_t>& raw, const TilePos& p, uint32_t ok, uint64_t seg) {
        if constexpr (kStats && kRaw == 2) unroll<8>([&](auto i) { stash[i * 64u + lane] = raw.r[i]; });
        float x[8][8];
        raw.to_float_minus128(x);  // sub_matrix_scalar (utils_kernels.cu:16), exact: (int8)(b ^ 0x80)
        // ---- forward: T.(X-128).T^T, round(C/Q), fp32 coefficient rows out
        uint2 q8[8];
        float qf[kFast ? 1 : 8][8];
        fdct_tile(T, x, [&](auto v, float (&c)[8]) {
            unroll<8>([&](auto u) { c[u] = quantise_at<kVar, v * 8 + u>(c[u], qp.q.v[v * 8 + u], qp.r.v[v * 8 + u]); });
            coef_sink(v, p, ok, seg, c);
            if constexpr (kFast) {
                // c holds integers in [-127, 127]: the truncating convert is exact
                uint32_t w0 = 0u, w1 = 0u;
                cvt_into_byte<0>(w0, c[0]), cvt_into_byte<1>(w0, c[1]), cvt_into_byte<2>(w0, c[2]),
                    cvt_into_byte<3>(w0, c[3]);
                cvt_into_byte<0>(w1, c[4]), cvt_into_byte<1>(w1, c[5]), cvt_into_byte<2>(w1, c[6]),
                    cvt_into_byte<3>(w1, c[7]);
                q8[v] = make_uint2(w0, w1);
            } else {
                unroll<8>([&](auto u) { qf[v][u] = c[u]; });
            }
        });
        // ---- inverse: D = q*Q (multiply_matrices, utils_kernels.cu:55),
        // T^T.D.T + 128 (main_newAppr.cu:220-250, utils_kernels.cu:29)
        uint2 again[kStats && kRaw == 1 ? 8 : 1];
        if constexpr (kStats && kRaw == 1) {
            unroll<8>([&](auto i) { again[i] = *reinterpret_cast<const uint2*>(img + p.base + i * g.width); });
        }
        float d[8][8];
        unroll<8>([&](auto i) {
            unroll<8>([&](auto j) {
                float qv;
                if constexpr (kFast) {
                    qv = i8_byte_f32(j < 4 ? q8[i].x : q8[i].y, j & 3);
                } else {
                    qv = qf[i][j];
                }
                d[i][j] = qv * qp.q.v[i * 8 + j];
            });
        });
        auto emit_inv = [&](auto v, float (&r)[8]) {
            unroll<8>([&](auto u) { r[u] = r[u] + 128.0f; });
            uint2 r8;  // convertToUnsignedChar (utils.cu:21): clamp, truncate, packed
            if constexpr (kStats || kRecon == kRtReconU8) {
                r8 = make_uint2(pack_u8x4(r[0], r[1], r[2], r[3]), pack_u8x4(r[4], r[5], r[6], r[7]));
            }
            if constexpr (kStats) {
                // integer sums on the packed bytes, 4 pixels per v_dot4_u32_u8:
                // sum (x - r8)^2 = sum x^2 - 2 sum x.r8 + sum r8^2 (exact in uint32)
                uint2 w;
                if constexpr (kRaw == 0) {
                    w = raw.r[v];
                } else if constexpr (kRaw == 1) {
                    w = again[v];
                } else {
                    w = stash[v * 64u + lane];
                }
                acc_xx = __builtin_amdgcn_udot4(w.x, w.x, acc_xx, false);
                acc_xx = __builtin_amdgcn_udot4(w.y, w.y, acc_xx, false);
                acc_xr = __builtin_amdgcn_udot4(w.x, r8.x, acc_xr, false);
                acc_xr = __builtin_amdgcn_udot4(w.y, r8.y, acc_xr, false);
                acc_rr = __builtin_amdgcn_udot4(r8.x, r8.x, acc_rr, false);
                acc_rr = __builtin_amdgcn_udot4(r8.y, r8.y, acc_rr, false);
                unroll<8>([&](auto u) {
                    const float e = byte_f32(u < 4 ? w.x : w.y, u & 3) - r[u];
                    acc_f[v & 1][u & 1] = __builtin_fmaf(e, e, acc_f[v & 1][u & 1]);
                });
            }
            if constexpr (kRecon == kRtReconU8) {
                st<true>(reinterpret_cast<uint2*>(static_cast<uint8_t*>(recon) + p.base + v * g.width), r8);
            } else if constexpr (kRecon == kRtReconF32) {
                rf32_sink(v, p, ok, seg, r);
            }
        };
        if constexpr (kFast) {
            idct_tile(T, d, emit_inv);
        } else if (wave_tame(d)) {
            idct_tile(T, d, emit_inv);
        } else {
            idct_tile(T_full, d, emit_inv);
        }
    });

    if constexpr (kStats) {
        // lanes without a tile (ragged last set, or waves past the end) hold zeros.
        // A chain's fixed point below 2^40 (sse < 2^24) is added exactly; a
        // larger or non-finite one (IEEE path with an extreme table) adds
        // nothing and sets the sticky bit 63 of the field (rt_sse_fix)
        bool f_ok = true;
        unsigned long long f = rt_sse_fix(acc_f[0][0], f_ok) + rt_sse_fix(acc_f[0][1], f_ok) +
                               rt_sse_fix(acc_f[1][0], f_ok) + rt_sse_fix(acc_f[1][1], f_ok);
        unsigned long long e8 = static_cast<unsigned long long>(acc_xx + acc_rr - 2u * acc_xr);
        unsigned long long xx = static_cast<unsigned long long>(acc_xx);
        f = wave_sum_u64(f), e8 = wave_sum_u64(e8), xx = wave_sum_u64(xx);
        // a wave's f is < 64 * 4 * 2^40: bit 63 of its slot carries the wave's flag
        if (__builtin_amdgcn_ballot_w64(!f_ok) != 0) f |= kRtSseF32Invalid;
        __shared__ unsigned long long part[kBlock / 64][3];
        const uint32_t w = threadIdx.x / 64u;
        if ((threadIdx.x & 63u) == 0u) part[w][0] = f, part[w][1] = e8, part[w][2] = xx;
        __syncthreads();
        if (threadIdx.x < 3u) {
            unsigned long long s = 0, bad = 0;
            for (uint32_t k = 0; k < kBlock / 64u; ++k) {
                s += part[k][threadIdx.x] & ~kRtSseF32Invalid;
                bad |= part[k][threadIdx.x] & kRtSseF32Invalid;
            }
            auto* const dst = reinterpret_cast<unsigned long long*>(sums) + threadIdx.x;
            if (s) atomicAdd(dst, s);
            if (bad) atomicOr(dst, kRtSseF32Invalid);
        }
    }
}

// Folds the kRtSpread sub-slots of a spread slot into *dst (overwriting it,
// or adding to it when accumulate) and zeroes them: one wave, lane i takes
// sub-slot i.  Next on the stream after a round trip that added into the slot
// (hpdct_roundtrip_u8 and _accumulate, round 5).  The one-wave kernel costs
// less than the memset it replaced (round 4: 77.6 us per 8192^2 launch against
// 79.3 with a memset of the caller's struct before the kernel,
// profiles/r04/j/kb3_rtring_8192.log).
// Every step is atomic: each sub-slot word is taken and zeroed by
// one atomic exchange, and an accumulate adds into *dst with atomic adds.  So
// two accumulate launches with one sums pointer on different streams (one
// slot, two round trips and two folds in flight) lose nothing: whatever one
// fold takes of the other launch's partial sums the other fold no longer
// finds, and both folds' adds land.  An overwrite is a plain store: two
// overwrites of one struct in flight race by definition.
template <int kN = kRtSpread>
__global__ __launch_bounds__(64) void rt_spread_finish_kernel(RtSums* __restrict__ dst,
                                                              unsigned long long* __restrict__ slot, int accumulate) {
    const uint32_t l = threadIdx.x;
    unsigned long long v[3] = {0ull, 0ull, 0ull}, bad[3] = {0ull, 0ull, 0ull};
    for (uint32_t k = l; k < static_cast<uint32_t>(kN); k += 64u) {
        unroll<3>([&](auto f) {
            const unsigned long long x = atomicExch(&slot[k * kRtSpreadStride + f], 0ull);
            v[f] += x & ~kRtSseF32Invalid, bad[f] |= x & kRtSseF32Invalid;
        });
    }
    unroll<3>([&](auto f) {
        const unsigned long long sum = wave_sum_dpp(v[f]);
        const bool flagged = __builtin_amdgcn_ballot_w64(bad[f] != 0ull) != 0ull;
        if (l == 0u) {
            auto* const d = reinterpret_cast<unsigned long long*>(dst) + f;
            if (accumulate) {
                if (sum) atomicAdd(d, sum);
                if (flagged) atomicOr(d, kRtSseF32Invalid);
            } else {
                *d = flagged ? (sum | kRtSseF32Invalid) : sum;
            }
        }
    });
}

inline dim3 roundtrip_grid(const TileGrid& g, uint32_t block = kRtBlock) {
    const uint32_t sets = (g.ntiles + 63u) / 64u, waves = block / 64u;
    return dim3((sets + waves - 1u) / waves);
}

namespace rt_detail {
template <int kRecon, bool kStats, int kQMode>
hipError_t go(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g, const QParams& qp,
              hipStream_t s) {
    if constexpr (kQMode != 0) {
        if (g.tiles_x % 64u != 0u) {  // straddling sets: two-run staged stores (kVarStraddle)
            hipLaunchKernelGGL((roundtrip_kernel<kRecon, kStats, kQMode, 2, true>), roundtrip_grid(g), dim3(kRtBlock),
                               0, s, img, coef, recon, sums, g, qp);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((roundtrip_kernel<kRecon, kStats, kQMode>), roundtrip_grid(g), dim3(kRtBlock), 0, s, img,
                       coef, recon, sums, g, qp);
    return hipGetLastError();
}
template <int kRecon, bool kStats>
hipError_t go_q(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g, const QParams& qp,
                int qmode, hipStream_t s) {
    switch (qmode) {
        case 2: return go<kRecon, kStats, 2>(img, coef, recon, sums, g, qp, s);
        case 1: return go<kRecon, kStats, 1>(img, coef, recon, sums, g, qp, s);
        default: return go<kRecon, kStats, 0>(img, coef, recon, sums, g, qp, s);
    }
}
template <int kRecon>
hipError_t go_r(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g, const QParams& qp,
                int qmode, hipStream_t s) {
    if (sums) return go_q<kRecon, true>(img, coef, recon, sums, g, qp, qmode, s);
    return go_q<kRecon, false>(img, coef, recon, sums, g, qp, qmode, s);
}
}  // namespace rt_detail

}  // namespace hpdct
