// kbench3.hip -- lean A/B bench for the round-3 kernel work (fast to build:
// only the library headers and the variants under test, not the whole
// variant zoo of kbench2).  One HxW uint8 frame per buffer set, sets rotated
// (16 sets at 8192^2 = 1 GiB of inputs, 4x the Infinity Cache), interleaved
// rounds, median of per-batch averages, every variant checked bit-for-bit
// against its group's first entry before timing.
//
//   kbench3 [n=8192 | HxW] [iters=64] [rounds=3] [group=all|fwd] [sets=16]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "hpdct_launch.hpp"
#include "kbench_dma.hpp"
#include "kbench_band.hpp"
#include "kbench_spec.hpp"
#include "kbench_rtpk.hpp"

using namespace hpdct;

int hpdct::mapping_mode() { return 0; }

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

struct Ctx {
    TileGrid g;
    QParams qp;
    uint32_t cus;
};
typedef void (*LaunchFn)(const void* in, void* out, const Ctx& c, hipStream_t s);
struct Variant {
    std::string group, name;
    LaunchFn launch;
    double bpp;    // algorithmic bytes per pixel
    size_t obpp;   // output plane bytes per pixel (the check compares this plane)
    bool check;
};

template <unsigned kVar>
void prod_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::fdct_kernel<uint8_t, float, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}

template <uint32_t kWaves, uint32_t kWgsPerCu>
void dma_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (!dma::dma_ok<kWaves>(c.g)) {
        fprintf(stderr, "dma: width must be a multiple of %u px\n", kWaves * 512u);
        exit(2);
    }
    (void)dma::dma_go<kVarFastDiv, kWaves>(static_cast<const uint8_t*>(in), static_cast<float*>(out), c.g, c.qp, c.cus,
                                           kWgsPerCu, s);
}

// banded persistent schedule with register prefetch (kbench_band.hpp)
template <typename TOut, unsigned kVar, uint32_t kWavesPerCU, bool kPk = false>
void band_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    (void)band::band_go<TOut, kVar, kPk>(static_cast<const uint8_t*>(in), static_cast<TOut*>(out), c.g, c.qp, c.cus,
                                    kWavesPerCU, s);
}
template <unsigned kVar>
void prod_i8_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}

// C2's small frames: the octet kernel (8 tiles per wave) the library picks
// below 8 sets per CU, at a chosen workgroup size (kVar bits 12..13)
template <unsigned kVar>
void oct_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::fdct_octet_kernel<uint8_t, float, true, true, false, kVar>), octet_grid(c.g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr,
                       c.g, nullptr, c.qp, 128.0f);
}

// the tools-only tile kernel (kbench_variants.hpp), e.g. with ab::kVarPacked
template <typename TOut, unsigned kVar>
void ab_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::ab::fdct_kernel<uint8_t, TOut, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, ab::kBlock<kVar>), dim3(ab::kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<TOut*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}

// ---- C3 round trip, u8 reconstruction into `out`, coefficients into g_coef[set]
std::vector<uint8_t*> g_img;
std::vector<float*> g_coef;
std::vector<float*> g_shift;  // drop-in forward's X-128 write-back planes
RtSums* g_sums = nullptr;
RtSums* g_sums_ring = nullptr;  // kRing slots: each launch adds into the next one
constexpr int kRing = 1024;
int g_ring_next = 0;
int set_of(const void* in) {
    for (size_t i = 0; i < g_img.size(); ++i)
        if (g_img[i] == in) return (int)i;
    return 0;
}
template <bool kStats>
void rt_prod(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, kStats, true, 2, false, 512>), roundtrip_grid(c.g, 512), dim3(512), 0, s,
                       static_cast<const uint8_t*>(in), g_coef[set_of(in)], out, kStats ? g_sums : nullptr, c.g, c.qp);
}
template <bool kStats>
void rt_pk(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((rtpk::roundtrip_pk_kernel<kStats>), roundtrip_grid(c.g, 512), dim3(512), 0, s,
                       static_cast<const uint8_t*>(in), g_coef[set_of(in)], static_cast<uint8_t*>(out),
                       kStats ? g_sums : nullptr, c.g, c.qp);
}

// wave-specialised: 4 store waves + kCompute compute waves per CU (kbench_spec.hpp)
template <uint32_t kCompute, bool kMath, uint32_t kSleep>
void spec_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (!spec::spec_ok(c.g)) {
        fprintf(stderr, "spec: width must be a multiple of 512 px\n");
        exit(2);
    }
    (void)spec::spec_go<kCompute, kMath, kSleep, kVarFastDiv>(static_cast<const uint8_t*>(in),
                                                              static_cast<float*>(out), c.g, c.qp, c.cus, s);
}

// ---- VALU issue probe: kWaves waves per CU, each kChains independent fma
// chains of kIters steps (scalar v_fma_f32, or packed v_pk_fma_f32 doing two
// fmas per instruction); inline asm so the compiler neither packs the scalar
// form nor unpacks the packed one.  Same fma count in both forms.
template <bool kPk, uint32_t kChains>
__global__ __launch_bounds__(256) void issue_probe(float* out, uint32_t iters, float a) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    float acc = 0.0f;
    if constexpr (kPk) {
        f2 s[kChains];
        const f2 m = {a, a};
        unroll<kChains>([&](auto k) { s[k] = f2{(float)threadIdx.x + k, (float)k}; });
        for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
            for (uint32_t k = 0; k < kChains; ++k) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(s[k]) : "v"(m));
        }
        unroll<kChains>([&](auto k) { acc += s[k].x + s[k].y; });
    } else {
        float s[2 * kChains];
        unroll<2 * kChains>([&](auto k) { s[k] = (float)threadIdx.x + k; });
        for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
            for (uint32_t k = 0; k < 2 * kChains; ++k) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[k]) : "v"(a));
        }
        unroll<2 * kChains>([&](auto k) { acc += s[k]; });
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
// bpp is unused for these (no pixels); the printed "frac" column is meaningless
template <bool kPk, uint32_t kWavesPerCU>
void issue_go(const void*, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((issue_probe<kPk, 8>), dim3(c.cus * kWavesPerCU / 4u), dim3(256), 0, s, static_cast<float*>(out),
                       4096u, 0.999f);
}

// ---- access-pattern probes (no arithmetic; values are not a transform) ----
// The headline kernel's traffic per 64-tile set (8 row loads of 512 B, 16 NT
// stores of 1 KiB) issued by W persistent waves that walk the sets in bands
// (set = j * W + wave: at step j all waves work on consecutive sets, so the
// chip-wide write front is W x 16 KiB) with the next set's rows prefetched
// into registers; W = kWavesPerCU x CUs.
template <bool kPrefetch, uint32_t kWpb = 4>
__global__ __launch_bounds__(64 * kWpb) void pat_band(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                      TileGrid g, uint32_t nsets) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * kWpb;
    uint32_t s = __builtin_amdgcn_readfirstlane(blockIdx.x * kWpb + (threadIdx.x >> 6));
    auto base_of = [&](uint32_t set) {
        const uint32_t t0 = set * 64u, ty = t0 / g.tiles_x, tx = t0 - ty * g.tiles_x;
        return static_cast<uint64_t>(ty) * 8u * g.width + static_cast<uint64_t>(tx) * 8u;
    };
    uint2 r[8];
    if (s >= nsets) return;
    unroll<8>([&](auto i) { r[i] = *reinterpret_cast<const uint2*>(in + base_of(s) + i * g.width + 8u * lane); });
    for (; s < nsets; s += nw) {
        uint2 nx[8];
        const bool more = kPrefetch && s + nw < nsets;
        if (more) {
            unroll<8>([&](auto i) { nx[i] = *reinterpret_cast<const uint2*>(in + base_of(s + nw) + i * g.width + 8u * lane); });
        }
        float* o = out + base_of(s);
        unroll<8>([&](auto i) {
            const float4 a = make_float4((float)(r[i].x & 255u), (float)(r[i].x >> 24), (float)(r[i].y & 255u),
                                         (float)(r[i].y >> 24));
            st_at<true>(o + i * g.width, 16u * lane, a);
            st_at<true>(o + i * g.width, 1024u + 16u * lane, a);
        });
        if constexpr (kPrefetch) {
            if (more) unroll<8>([&](auto i) { r[i] = nx[i]; });
        } else if (s + nw < nsets) {
            unroll<8>([&](auto i) { r[i] = *reinterpret_cast<const uint2*>(in + base_of(s + nw) + i * g.width + 8u * lane); });
        }
    }
}
template <uint32_t kWavesPerCU, bool kPrefetch>
void pat_band_go(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t nsets = c.g.ntiles / 64u;
    hipLaunchKernelGGL((pat_band<kPrefetch>), dim3(std::min(nsets / 4u, c.cus * kWavesPerCU / 4u)), dim3(256), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), c.g, nsets);
}
// the same traffic, one set per wave, non-persistent (the product's dispatch)
void pat_grid_go(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t nsets = c.g.ntiles / 64u;
    hipLaunchKernelGGL((pat_band<false>), dim3(nsets / 4u), dim3(256), 0, s, static_cast<const uint8_t*>(in),
                       static_cast<float*>(out), c.g, nsets);
}

// the headline's access pattern in one-wave workgroups (the product's dispatch
// shape since round 3), at most kWaves resident per CU (0: uncapped)
template <uint32_t kWaves>
void pat_grid_cap1_go(const void* in, void* out, const Ctx& c, hipStream_t s);

// ---- occupancy caps through dynamic LDS (round 3, session 3): kWg workgroups
// per CU at most, so a 256-thread workgroup gives 4 x kWg waves per CU.  The
// kernels do not use the dynamic part; it only reserves LDS.
inline size_t cap_dyn_lds(uint32_t wg_per_cu, size_t static_bytes) {
    size_t per = (160u * 1024u) / wg_per_cu;
    per &= ~static_cast<size_t>(511);
    return per > static_bytes ? per - static_bytes : 0;
}
// dynamic LDS bytes that leave room for at most kWg workgroups of `kern` per CU
template <typename K>
size_t cap_for(K kern, uint32_t wg_per_cu) {
    hipFuncAttributes a{};
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kern));
    const size_t dyn = cap_dyn_lds(wg_per_cu, a.sharedSizeBytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(dyn));
    return dyn;
}
// the headline's access pattern (no arithmetic), one set per wave, capped
template <uint32_t kWg>
void pat_grid_cap_go(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t nsets = c.g.ntiles / 64u;
    static const size_t dyn = cap_for(pat_band<false>, kWg);
    hipLaunchKernelGGL((pat_band<false>), dim3(nsets / 4u), dim3(256), dyn, s, static_cast<const uint8_t*>(in),
                       static_cast<float*>(out), c.g, nsets);
}
template <uint32_t kWaves>
void pat_grid_cap1_go(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t nsets = c.g.ntiles / 64u;
    static const size_t dyn = kWaves ? cap_for(pat_band<false, 1>, kWaves) : 0;
    hipLaunchKernelGGL((pat_band<false, 1>), dim3(nsets), dim3(64), dyn, s, static_cast<const uint8_t*>(in),
                       static_cast<float*>(out), c.g, nsets);
}
// the tools-only tile kernel (scalar or packed) with kWg workgroups per CU at most
template <typename TOut, unsigned kVar, uint32_t kWg>
void ab_fwd_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    constexpr uint32_t kB = ab::kBlock<kVar>;
    auto* k = hpdct::ab::fdct_kernel<uint8_t, TOut, true, true, false, kVar>;
    static const size_t dyn = cap_for(k, kWg);
    hipLaunchKernelGGL(k, grid_for(c.g, false, c.cus, kB), dim3(kB), dyn, s, static_cast<const uint8_t*>(in),
                       static_cast<TOut*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}
// the library's headline kernel itself, capped
template <unsigned kVar, uint32_t kWg>
void prod_f32_fwd_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = hpdct::fdct_kernel<uint8_t, float, true, true, false, kVar>;
    static const size_t dyn = cap_for(k, kWg);
    hipLaunchKernelGGL(k, grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), dyn, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}
// the library's int8 forward kernel, capped at kWg workgroups per CU (0: uncapped)
template <unsigned kVar, uint32_t kWg>
void prod_i8_fwd_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = hpdct::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    hipLaunchKernelGGL(k, grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), dyn, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}
// C3 round trip with a quotient mode (1: verified 3-op, 2: + JPEG per-position forms)
template <bool kStats, int kQMode>
void rt_q(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, kStats, kQMode, 2, false, 512>), roundtrip_grid(c.g, 512), dim3(512), 0, s,
                       static_cast<const uint8_t*>(in), g_coef[set_of(in)], out, kStats ? g_sums : nullptr, c.g, c.qp);
}
// the sums zeroed by three stream write-value commands instead of a memset
template <int kQMode>
void rt_wv(const void* in, void* out, const Ctx& c, hipStream_t s) {
    for (int k = 0; k < 3; ++k) (void)hipStreamWriteValue64(s, reinterpret_cast<uint64_t*>(g_sums) + k, 0ull, 0);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, true, kQMode, 2, false, 512>), roundtrip_grid(c.g, 512), dim3(512), 0, s,
                       static_cast<const uint8_t*>(in), g_coef[set_of(in)], out, g_sums, c.g, c.qp);
}
template <bool kStats, int kQMode, int kB>
void rt_qb(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, kStats, kQMode, 2, false, kB>), roundtrip_grid(c.g, kB), dim3(kB),
                       0, s, static_cast<const uint8_t*>(in), g_coef[set_of(in)], out, kStats ? g_sums : nullptr, c.g,
                       c.qp);
}
// one wave: the caller's sums = the slot's, and the slot back to zero
__global__ __launch_bounds__(64) void rt_finish_probe(RtSums* __restrict__ dst, RtSums* __restrict__ slot) {
    if (threadIdx.x < 3u) {
        auto* const src = reinterpret_cast<unsigned long long*>(slot) + threadIdx.x;
        reinterpret_cast<unsigned long long*>(dst)[threadIdx.x] = *src;
        *src = 0ull;
    }
}
// C3 round trip, 256-thread workgroups, where the sums go: kMode 0 the same
// struct every launch (hpdct_roundtrip_u8_accumulate into one struct), 1 the
// next slot of a ring (the driver bench's sums ring), 2 ring slot + a 24-byte
// device copy into the one struct after the kernel, 3 memset of the one struct
// + kernel (hpdct_roundtrip_u8), 4 memset of the ring slot + kernel, 5 one
// library slot + a one-wave kernel that copies it out and zeroes it
template <int kMode>
void rt_where(const void* in, void* out, const Ctx& c, hipStream_t s) {
    RtSums* const slot = g_sums_ring + (g_ring_next++ % (kRing - 1));  // kRing - 1: mode 5's slot
    RtSums* const dst = kMode == 0 || kMode == 3 ? g_sums : kMode == 5 ? g_sums_ring + kRing - 1 : slot;
    if (kMode == 3 || kMode == 4) (void)hipMemsetAsync(dst, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, true, 2, 2, false, 256>), roundtrip_grid(c.g, 256), dim3(256), 0,
                       s, static_cast<const uint8_t*>(in), g_coef[set_of(in)], out, dst, c.g, c.qp);
    if (kMode == 2) (void)hipMemcpyAsync(g_sums, slot, sizeof(RtSums), hipMemcpyDeviceToDevice, s);
    if (kMode == 5) hipLaunchKernelGGL(rt_finish_probe, dim3(1), dim3(64), 0, s, g_sums, dst);
}
// C3 round trip (512-thread workgroups), capped at kWg workgroups per CU (0: uncapped)
template <bool kStats, uint32_t kWg>
void rt_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = roundtrip_kernel<kRtReconU8, kStats, true, 2, false, 512>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL(k, roundtrip_grid(c.g, 512), dim3(512), dyn, s, static_cast<const uint8_t*>(in), g_coef[set_of(in)],
                       out, kStats ? g_sums : nullptr, c.g, c.qp);
}
// fp32 inverse (duo mapping, built-in T, dequantise), coefficients from g_coef, capped (0: uncapped)
template <uint32_t kWg>
void inv_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = idct_duo_kernel<true, true, kDuoVar, float>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    hipLaunchKernelGGL(k, duo_grid(c.g, kBlock<kDuoVar>), dim3(kBlock<kDuoVar>), dyn, s, g_coef[set_of(in)],
                       static_cast<float*>(out), nullptr, c.g, nullptr, c.qp.q, 128.0f);
}

// fp32 inverse, duo mapping with a chosen block size (kVar bits 12..13), capped (0: uncapped)
template <unsigned kVar, uint32_t kWg>
void inv_cap_v(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = idct_duo_kernel<true, true, kVar, float>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    hipLaunchKernelGGL(k, duo_grid(c.g, kBlock<kVar>), dim3(kBlock<kVar>), dyn, s, g_coef[set_of(in)],
                       static_cast<float*>(out), nullptr, c.g, nullptr, c.qp.q, 128.0f);
}
// the drop-in forward (fp32 in, built-in T here, X-128 written back into g_coef[set]), duo, capped
template <unsigned kVar, uint32_t kWg>
void dropin_fwd_cap(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = fdct_duo_kernel<true, true, true, kVar>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    float* src = g_coef[set_of(in)];
    hipLaunchKernelGGL(k, duo_grid(c.g, kBlock<kVar>), dim3(kBlock<kVar>), dyn, s, src, static_cast<float*>(out),
                       g_shift[set_of(in)], c.g, nullptr, c.qp, 128.0f);
}

// the drop-in forward as the compat entry points launch it (round 6 A/B): the
// caller's T in a device buffer (bitwise the built-in one), the JPEG table's
// checked quotient, uncapped (through round 5) or one-wave workgroups capped
// per CU (round 6)
float* g_T = nullptr;
template <unsigned kVar, uint32_t kWg, bool kWb = true>
void dropin_fwd_rt(const void* in, void* out, const Ctx& c, hipStream_t s) {
    auto* k = fdct_duo_kernel<true, false, kWb, kVar>;
    static const size_t dyn = kWg ? cap_for(k, kWg) : 0;
    float* src = g_coef[set_of(in)];
    hipLaunchKernelGGL(k, duo_grid(c.g, kBlock<kVar>), dim3(kBlock<kVar>), dyn, s, src, static_cast<float*>(out),
                       kWb ? g_shift[set_of(in)] : nullptr, c.g, g_T, c.qp, 128.0f);
}

int main(int argc, char** argv) {
    int n = 8192, hgt = 8192;
    if (argc > 1) {
        n = hgt = atoi(argv[1]);
        if (const char* x = strchr(argv[1], 'x')) n = atoi(x + 1);
    }
    const int iters = argc > 2 ? atoi(argv[2]) : 64;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const std::string only = argc > 4 ? argv[4] : "all";
    const int nsets = argc > 5 ? atoi(argv[5]) : 16;
    const size_t px = (size_t)hgt * n;
    Ctx c;
    c.g = TileGrid{(uint32_t)(px / 64), (uint32_t)(n / 8), (uint64_t)n};
    for (int i = 0; i < 64; ++i) {
        c.qp.q.v[i] = kDefaultQ.v[i];
        c.qp.r.v[i] = 1.0f / kDefaultQ.v[i];
    }
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    c.cus = (uint32_t)cus;

    constexpr unsigned F = kVarFastDiv;
    constexpr unsigned P = kProdVar<uint8_t, float> | F;
    constexpr unsigned I8 = kProdVar<uint8_t, int8_t> | F;
    // the headline's capped variant (one-wave workgroups, packed transform)
    constexpr unsigned PK1 = (P & ~(3u << 12)) | kOneWaveWg | kVarPacked;
    std::vector<Variant> vars = {
        {"fwd", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 8w x 2/cu", dma_f32_fwd<8, 2>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 8w x 1/cu", dma_f32_fwd<8, 1>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 4w x 4/cu", dma_f32_fwd<4, 4>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 4w x 2/cu", dma_f32_fwd<4, 2>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 8w not persistent", dma_f32_fwd<8, 64>, 5, 4, true},
        {"fwd", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"fwd", "fwd u8->f32 dma 8w x 2/cu again", dma_f32_fwd<8, 2>, 5, 4, true},
        {"band", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"band", "fwd u8->f32 band 4 w/cu", band_fwd<float, (P & ~(3u << 12)), 4>, 5, 4, true},
        {"band", "fwd u8->f32 band 8 w/cu b256", band_fwd<float, (P & ~(3u << 12)), 8>, 5, 4, true},
        {"band", "fwd u8->f32 band 8 w/cu b512", band_fwd<float, P, 8>, 5, 4, true},
        {"band", "fwd u8->f32 band 16 w/cu b512", band_fwd<float, P, 16>, 5, 4, true},
        {"band", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"band", "fwd u8->f32 band 4 w/cu again", band_fwd<float, (P & ~(3u << 12)), 4>, 5, 4, true},
        {"bandi8", "fwd u8->i8 library (b512)", prod_i8_fwd<I8>, 2, 1, true},
        {"bandi8", "fwd u8->i8 band 4 w/cu", band_fwd<int8_t, (I8 & ~(3u << 12)), 4>, 2, 1, true},
        {"bandi8", "fwd u8->i8 band 8 w/cu b256", band_fwd<int8_t, (I8 & ~(3u << 12)), 8>, 2, 1, true},
        {"bandi8", "fwd u8->i8 band 16 w/cu b512", band_fwd<int8_t, I8, 16>, 2, 1, true},
        {"bandi8", "fwd u8->i8 library (b512) again", prod_i8_fwd<I8>, 2, 1, true},
        {"bandpk", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"bandpk", "fwd u8->f32 band 4 w/cu", band_fwd<float, (P & ~(3u << 12)), 4>, 5, 4, true},
        {"bandpk", "fwd u8->f32 band 4 w/cu packed", band_fwd<float, (P & ~(3u << 12)), 4, true>, 5, 4, true},
        {"bandpk", "fwd u8->f32 band 8 w/cu b256 packed", band_fwd<float, (P & ~(3u << 12)), 8, true>, 5, 4, true},
        {"bandpk", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"bandpk", "fwd u8->f32 band 4 w/cu packed again", band_fwd<float, (P & ~(3u << 12)), 4, true>, 5, 4, true},
        {"pk", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"pk", "fwd u8->f32 packed (b512)", ab_fwd<float, P | ab::kVarPacked>, 5, 4, true},
        {"pk", "fwd u8->f32 packed (b256)", ab_fwd<float, (P & ~(3u << 12)) | ab::kVarPacked>, 5, 4, true},
        {"pk", "fwd u8->f32 packed (b1024)", ab_fwd<float, P | (3u << 12) | ab::kVarPacked>, 5, 4, true},
        {"pk", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"pk", "fwd u8->f32 packed (b512) again", ab_fwd<float, P | ab::kVarPacked>, 5, 4, true},
        {"rtpk", "rt + sums, library", rt_prod<true>, 6, 1, true},
        {"rtpk", "rt + sums, packed", rt_pk<true>, 6, 1, true},
        {"rtpk", "rt no sums, library", rt_prod<false>, 6, 1, true},
        {"rtpk", "rt no sums, packed", rt_pk<false>, 6, 1, true},
        {"rtpk", "rt + sums, library again", rt_prod<true>, 6, 1, true},
        {"rtpk", "rt + sums, packed again", rt_pk<true>, 6, 1, true},
        {"pki8", "fwd u8->i8 library (b512)", prod_i8_fwd<I8>, 2, 1, true},
        {"pki8", "fwd u8->i8 packed (b512)", ab_fwd<int8_t, I8 | ab::kVarPacked>, 2, 1, true},
        {"pki8", "fwd u8->i8 packed (b256)", ab_fwd<int8_t, (I8 & ~(3u << 12)) | ab::kVarPacked>, 2, 1, true},
        {"pki8", "fwd u8->i8 library (b512) again", prod_i8_fwd<I8>, 2, 1, true},
        {"pki8", "fwd u8->i8 packed (b512) again", ab_fwd<int8_t, I8 | ab::kVarPacked>, 2, 1, true},
        // 8 chains x 4096 steps x 2 fmas per lane pair: 65,536 fma per lane in both forms
        {"issue", "valu scalar fma, 4 waves/cu", issue_go<false, 4>, 0, 4, false},
        {"issue", "valu packed fma, 4 waves/cu", issue_go<true, 4>, 0, 4, false},
        {"issue", "valu scalar fma, 8 waves/cu", issue_go<false, 8>, 0, 4, false},
        {"issue", "valu packed fma, 8 waves/cu", issue_go<true, 8>, 0, 4, false},
        {"issue", "valu scalar fma, 16 waves/cu", issue_go<false, 16>, 0, 4, false},
        {"issue", "valu packed fma, 16 waves/cu", issue_go<true, 16>, 0, 4, false},
        // the two library forward kernels alone (frame-size sweeps: kbench3 HxW 64 3 libf32 / libi8)
        {"libf32", "fwd u8->f32 library", prod_f32_fwd<P>, 5, 4, true},
        {"libi8", "fwd u8->i8 library", prod_i8_fwd<I8>, 2, 1, true},
        {"spec", "fwd u8->f32 library", prod_f32_fwd<P>, 5, 4, true},
        {"spec", "fwd u8->f32 spec 4 store + 12 compute", spec_fwd<12, true, 0>, 5, 4, true},
        {"spec", "fwd u8->f32 spec 4 store + 8 compute", spec_fwd<8, true, 0>, 5, 4, true},
        {"spec", "fwd u8->f32 library again", prod_f32_fwd<P>, 5, 4, true},
        {"spec", "fwd u8->f32 spec 4 store + 12 compute again", spec_fwd<12, true, 0>, 5, 4, true},
        {"specpat", "pat one set per wave (grid)", pat_grid_go, 5, 4, false},
        {"specpat", "spec pattern 4+12, no compute", spec_fwd<12, false, 0>, 5, 4, false},
        {"specpat", "spec pattern 4+12, sleep 40x64 cyc per set", spec_fwd<12, false, 40>, 5, 4, false},
        {"specpat", "spec pattern 4+8, sleep 40x64 cyc per set", spec_fwd<8, false, 40>, 5, 4, false},
        {"specpat", "pat one set per wave (grid) again", pat_grid_go, 5, 4, false},
        // occupancy caps (dynamic LDS): does the one-set-per-wave dispatch gain DRAM efficiency with fewer
        // waves per CU, as the banded schedule did (0.77 at 4 w/cu), and can the packed math keep up there?
        // round 5: the headline's limiter at cap 7, counters in their own passes
        {"lim", "fwd u8->f32 product kernel, cap 7 w/cu", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        {"lim", "pat 1-wave WGs, cap 4 w/cu", pat_grid_cap1_go<4>, 5, 4, false},
        {"lim", "pat 1-wave WGs, cap 7 w/cu", pat_grid_cap1_go<7>, 5, 4, false},
        {"lim", "pat 1-wave WGs, uncapped", pat_grid_cap1_go<0>, 5, 4, false},
        {"lim1", "fwd u8->f32 product kernel, cap 7 w/cu", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        // the whole-run test hoisted out of the per-row stores (two straight-line body copies)
        {"hoist", "fwd u8->f32 product kernel, cap 7 w/cu", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        {"hoist", "fwd u8->f32 hoisted run test, cap 7 w/cu", prod_f32_fwd_cap<(530457u | kVarHoistRun), 7>, 5, 4, true},
        {"hoist", "fwd u8->f32 hoisted run test, cap 6 w/cu", prod_f32_fwd_cap<(530457u | kVarHoistRun), 6>, 5, 4, true},
        {"hoist", "fwd u8->f32 hoisted run test, cap 8 w/cu", prod_f32_fwd_cap<(530457u | kVarHoistRun), 8>, 5, 4, true},
        {"hoist", "fwd u8->f32 product kernel, cap 7 w/cu again", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        {"hoist", "fwd u8->f32 hoisted run test, cap 7 w/cu again", prod_f32_fwd_cap<(530457u | kVarHoistRun), 7>, 5, 4, true},
        // the headline without the LDS re-staging of its rows (each lane stores its tile's 32-B rows directly):
        // at <= 7 waves per CU a wave's 8 LDS round trips are poorly hidden
        {"nolds", "fwd u8->f32 product kernel, cap 7 w/cu", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        {"nolds", "fwd u8->f32 no LDS staging, cap 7 w/cu", prod_f32_fwd_cap<(530457u & ~8u), 7>, 5, 4, true},
        {"nolds", "fwd u8->f32 no LDS staging, cap 8 w/cu", prod_f32_fwd_cap<(530457u & ~8u), 8>, 5, 4, true},
        {"nolds", "fwd u8->f32 no LDS staging, cap 10 w/cu", prod_f32_fwd_cap<(530457u & ~8u), 10>, 5, 4, true},
        {"nolds", "fwd u8->f32 no LDS staging, cap 12 w/cu", prod_f32_fwd_cap<(530457u & ~8u), 12>, 5, 4, true},
        {"nolds", "fwd u8->f32 product kernel, cap 7 w/cu again", prod_f32_fwd_cap<530457u, 7>, 5, 4, true},
        {"nolds", "fwd u8->f32 no LDS staging, cap 7 w/cu again", prod_f32_fwd_cap<(530457u & ~8u), 7>, 5, 4, true},
        {"lim4", "pat 1-wave WGs, cap 4 w/cu", pat_grid_cap1_go<4>, 5, 4, false},
        {"lim7", "pat 1-wave WGs, cap 7 w/cu", pat_grid_cap1_go<7>, 5, 4, false},
        {"occpat", "pat one set per wave (grid)", pat_grid_go, 5, 4, false},
        {"occpat", "pat grid cap 4 w/cu", pat_grid_cap_go<1>, 5, 4, false},
        {"occpat", "pat grid cap 8 w/cu", pat_grid_cap_go<2>, 5, 4, false},
        {"occpat", "pat grid cap 12 w/cu", pat_grid_cap_go<3>, 5, 4, false},
        {"occpat", "pat grid cap 16 w/cu", pat_grid_cap_go<4>, 5, 4, false},
        {"occpat", "pat grid cap 24 w/cu", pat_grid_cap_go<6>, 5, 4, false},
        {"occpat", "pat one set per wave (grid) again", pat_grid_go, 5, 4, false},
        {"occ", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"occ", "fwd u8->f32 scalar b256 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)), 2>, 5, 4, true},
        {"occ", "fwd u8->f32 scalar b256 cap 12 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)), 3>, 5, 4, true},
        {"occ", "fwd u8->f32 packed (b512)", ab_fwd<float, P | ab::kVarPacked>, 5, 4, true},
        {"occ", "fwd u8->f32 packed b256 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | ab::kVarPacked, 2>, 5, 4, true},
        {"occ", "fwd u8->f32 packed b256 cap 12 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | ab::kVarPacked, 3>, 5, 4, true},
        {"occ", "fwd u8->f32 packed b512 cap 8 w/cu", ab_fwd_cap<float, P | ab::kVarPacked, 1>, 5, 4, true},
        {"occ", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"occ", "fwd u8->f32 packed b256 cap 12 w/cu again", ab_fwd_cap<float, (P & ~(3u << 12)) | ab::kVarPacked, 3>, 5, 4, true},
        // round 3, session 3: finer occupancy caps (64-thread workgroups = one wave each)
        {"occ2", "fwd u8->f32 library (b512)", prod_f32_fwd<P>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b256 cap 12 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)), 3>, 5, 4, true},
        {"occ2", "fwd u8->f32 library kernel b512 cap 8 w/cu", prod_f32_fwd_cap<P, 1>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b64 cap 6 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 6>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b64 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 8>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b64 cap 10 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 10>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b64 cap 12 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 12>, 5, 4, true},
        {"occ2", "fwd u8->f32 packed b64 cap 6 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 6>, 5, 4, true},
        {"occ2", "fwd u8->f32 packed b64 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 8>, 5, 4, true},
        {"occ2", "fwd u8->f32 packed b256 cap 4 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | ab::kVarPacked, 1>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b256 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)), 2>, 5, 4, true},
        {"occ2", "fwd u8->f32 library (b512) again", prod_f32_fwd<P>, 5, 4, true},
        {"occ2", "fwd u8->f32 scalar b256 cap 12 w/cu again", ab_fwd_cap<float, (P & ~(3u << 12)), 3>, 5, 4, true},
        {"occi8", "fwd u8->i8 library (b512)", prod_i8_fwd<I8>, 2, 1, true},
        {"occi8", "fwd u8->i8 scalar b256 cap 12 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)), 3>, 2, 1, true},
        {"occi8", "fwd u8->i8 scalar b256 cap 16 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)), 4>, 2, 1, true},
        {"occi8", "fwd u8->i8 packed b256 cap 12 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)) | ab::kVarPacked, 3>, 2, 1, true},
        {"occi8", "fwd u8->i8 packed b256 cap 8 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)) | ab::kVarPacked, 2>, 2, 1, true},
        {"occi8", "fwd u8->i8 library (b512) again", prod_i8_fwd<I8>, 2, 1, true},
        {"rtocc", "rt + sums, library", rt_cap<true, 0>, 6, 1, true},
        {"rtocc", "rt + sums, cap 8 w/cu", rt_cap<true, 1>, 6, 1, true},
        {"rtocc", "rt no sums, library", rt_cap<false, 0>, 6, 1, true},
        {"rtocc", "rt no sums, cap 8 w/cu", rt_cap<false, 1>, 6, 1, true},
        {"rtocc", "rt + sums, library again", rt_cap<true, 0>, 6, 1, true},
        {"invocc", "inv f32->f32 duo library", inv_cap<0>, 8, 4, true},
        {"invocc", "inv f32->f32 duo cap 8 w/cu", inv_cap<2>, 8, 4, true},
        {"invocc", "inv f32->f32 duo cap 12 w/cu", inv_cap<3>, 8, 4, true},
        {"invocc", "inv f32->f32 duo cap 16 w/cu", inv_cap<4>, 8, 4, true},
        {"invocc", "inv f32->f32 duo cap 24 w/cu", inv_cap<6>, 8, 4, true},
        {"invocc", "inv f32->f32 duo library again", inv_cap<0>, 8, 4, true},
        // round 3, session 3: 1-wave workgroups, occupancy caps (sweep; also run at other frame sizes)
        {"occsz", "fwd u8->f32 library", prod_f32_fwd<P>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 uncapped", ab_fwd<float, (P & ~(3u << 12)) | (1u << 12)>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 8>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 9 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 9>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 10 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 10>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 11 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 11>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 12 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 12>, 5, 4, true},
        {"occsz", "fwd u8->f32 packed b64 cap 8 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 8>, 5, 4, true},
        {"occsz", "fwd u8->f32 packed b64 cap 10 w/cu", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 10>, 5, 4, true},
        {"occsz", "fwd u8->f32 library again", prod_f32_fwd<P>, 5, 4, true},
        {"occsz", "fwd u8->f32 scalar b64 cap 10 w/cu again", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12), 10>, 5, 4, true},
        {"occsz", "fwd u8->f32 packed b64 cap 8 w/cu again", ab_fwd_cap<float, (P & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 8>, 5, 4, true},
        {"occi8b", "fwd u8->i8 library (b512)", prod_i8_fwd<I8>, 2, 1, true},
        {"occi8b", "fwd u8->i8 scalar b64 uncapped", ab_fwd<int8_t, (I8 & ~(3u << 12)) | (1u << 12)>, 2, 1, true},
        {"occi8b", "fwd u8->i8 scalar b64 cap 12 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)) | (1u << 12), 12>, 2, 1, true},
        {"occi8b", "fwd u8->i8 scalar b64 cap 16 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)) | (1u << 12), 16>, 2, 1, true},
        {"occi8b", "fwd u8->i8 packed b64 cap 16 w/cu", ab_fwd_cap<int8_t, (I8 & ~(3u << 12)) | (1u << 12) | ab::kVarPacked, 16>, 2, 1, true},
        {"occi8b", "fwd u8->i8 library (b512) again", prod_i8_fwd<I8>, 2, 1, true},
        {"invb", "inv f32->f32 duo library", inv_cap<0>, 8, 4, true},
        {"invb", "inv f32->f32 duo b256 cap 8 w/cu", inv_cap<2>, 8, 4, true},
        {"invb", "inv f32->f32 duo b256 cap 12 w/cu", inv_cap<3>, 8, 4, true},
        {"invb", "inv f32->f32 duo b64 uncapped", inv_cap_v<kDuoVar | (1u << 12), 0>, 8, 4, true},
        {"invb", "inv f32->f32 duo b64 cap 8 w/cu", inv_cap_v<kDuoVar | (1u << 12), 8>, 8, 4, true},
        {"invb", "inv f32->f32 duo b64 cap 10 w/cu", inv_cap_v<kDuoVar | (1u << 12), 10>, 8, 4, true},
        {"invb", "inv f32->f32 duo b64 cap 12 w/cu", inv_cap_v<kDuoVar | (1u << 12), 12>, 8, 4, true},
        {"invb", "inv f32->f32 duo library again", inv_cap<0>, 8, 4, true},
        {"dropin", "dropin fwd f32 duo library", dropin_fwd_cap<kDuoVar, 0>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo b256 cap 8 w/cu", dropin_fwd_cap<kDuoVar, 2>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo b256 cap 12 w/cu", dropin_fwd_cap<kDuoVar, 3>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo b64 cap 8 w/cu", dropin_fwd_cap<kDuoVar | (1u << 12), 8>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo b64 cap 10 w/cu", dropin_fwd_cap<kDuoVar | (1u << 12), 10>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo b64 cap 12 w/cu", dropin_fwd_cap<kDuoVar | (1u << 12), 12>, 12, 4, true},
        {"dropin", "dropin fwd f32 duo library again", dropin_fwd_cap<kDuoVar, 0>, 12, 4, true},
        {"c2oct", "octet 256-thread WGs (library)", oct_f32_fwd<kOctVar<float> | kVarFastDiv>, 5, 4, true},
        {"c2oct", "octet 512-thread WGs", oct_f32_fwd<(kOctVar<float> | kVarFastDiv) | (2u << 12)>, 5, 4, true},
        {"c2oct", "octet 1024-thread WGs", oct_f32_fwd<(kOctVar<float> | kVarFastDiv) | (3u << 12)>, 5, 4, true},
        {"c2oct", "octet 256-thread WGs again", oct_f32_fwd<kOctVar<float> | kVarFastDiv>, 5, 4, true},
        {"c2oct", "tile 1024-thread WGs (the library's above 8 sets/CU)", prod_f32_fwd<((kProdVar<uint8_t, float> | kVarFastDiv | kVarJpegQ) & ~(3u << 12)) | (3u << 12)>, 5, 4, true},
        {"dropcap", "dropin uncapped (round 5)", dropin_fwd_rt<kDuoVar | kVarFastDivChecked, 0>, 12, 4, true},
        {"dropcap", "dropin b64 cap 10", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10>, 12, 4, true},
        {"dropcap", "dropin b64 cap 8", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 8>, 12, 4, true},
        {"dropcap", "dropin b64 cap 10 again", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10>, 12, 4, true},
        {"dropcap", "dropin uncapped again", dropin_fwd_rt<kDuoVar | kVarFastDivChecked, 0>, 12, 4, true},
        {"fwdcap", "fwd no wb uncapped (round 5)", dropin_fwd_rt<kDuoVar | kVarFastDivChecked, 0, false>, 8, 4, true},
        {"fwdcap", "fwd no wb b64 cap 10", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10, false>, 8, 4, true},
        {"fwdcap", "fwd no wb uncapped again", dropin_fwd_rt<kDuoVar | kVarFastDivChecked, 0, false>, 8, 4, true},
        // round 6, after the duo forward's 16-wave cap: the fp32 duo forward in 256-thread workgroups
        {"duocap16", "dropin b64 cap 10 (product)", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10>, 12, 4, true},
        {"duocap16", "dropin b64 cap 16", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 16>, 12, 4, true},
        {"duocap16", "dropin b64 cap 6", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 6>, 12, 4, true},
        {"duocap16", "dropin b256 cap 4 WGs", dropin_fwd_rt<(kDuoVar | kVarFastDivChecked) & ~(3u << 12), 4>, 12, 4, true},
        {"duocap16", "dropin b256 cap 3 WGs", dropin_fwd_rt<(kDuoVar | kVarFastDivChecked) & ~(3u << 12), 3>, 12, 4, true},
        {"duocap16", "fwd no wb b64 cap 10 (product)", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10, false>, 8, 4, true},
        {"duocap16", "fwd no wb b256 cap 4 WGs", dropin_fwd_rt<(kDuoVar | kVarFastDivChecked) & ~(3u << 12), 4, false>, 8, 4, true},
        {"duocap16", "dropin b64 cap 10 (product) again", dropin_fwd_rt<kDuoVar | kVarFastDivChecked | (1u << 12), 10>, 12, 4, true},
        {"duocap16", "dropin b256 cap 4 WGs again", dropin_fwd_rt<(kDuoVar | kVarFastDivChecked) & ~(3u << 12), 4>, 12, 4, true},
        // round 4: the default JPEG table's per-position 3-op quantiser forms (kVarJpegQ) against the
        // verified 6-op form, in the product's dispatch, and the headline cap re-swept with them
        {"jq", "fwd u8->f32 library cap 10 (6-op)", prod_f32_fwd_cap<PK1, 10>, 5, 4, true},
        {"jq", "fwd u8->f32 jpegq cap 8 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 8>, 5, 4, true},
        {"jq", "fwd u8->f32 jpegq cap 9 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 9>, 5, 4, true},
        {"jq", "fwd u8->f32 jpegq cap 10 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jq", "fwd u8->f32 jpegq cap 12 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 12>, 5, 4, true},
        {"jq", "fwd u8->f32 library cap 10 (6-op) again", prod_f32_fwd_cap<PK1, 10>, 5, 4, true},
        {"jq", "fwd u8->f32 jpegq cap 10 w/cu again", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqi8", "fwd u8->i8 library b512 (6-op)", prod_i8_fwd<I8>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq b512", prod_i8_fwd<I8 | kVarJpegQ>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq b256", prod_i8_fwd<(I8 & ~(3u << 12)) | kVarJpegQ>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq b1024", prod_i8_fwd<(I8 & ~(3u << 12)) | (3u << 12) | kVarJpegQ>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq b64 cap 16 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 16>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq packed b512", prod_i8_fwd<I8 | kVarJpegQ | kVarPacked>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq packed b256", prod_i8_fwd<(I8 & ~(3u << 12)) | kVarJpegQ | kVarPacked>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq packed b64 cap 16 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ | kVarPacked, 16>, 2, 1, true},
        {"jqi8", "fwd u8->i8 library b512 (6-op) again", prod_i8_fwd<I8>, 2, 1, true},
        {"jqi8", "fwd u8->i8 jpegq b512 again", prod_i8_fwd<I8 | kVarJpegQ>, 2, 1, true},
        // round 4, session 2: the packed int8 forward (JPEG forms and the 6-op quotient) across block sizes / caps
        {"jqi8b", "fwd u8->i8 library b512 (6-op)", prod_i8_fwd<I8>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 packed 6-op b512", prod_i8_fwd<I8 | kVarPacked>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b512", prod_i8_fwd<I8 | kVarJpegQ | kVarPacked>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b1024", prod_i8_fwd<(I8 & ~(3u << 12)) | (3u << 12) | kVarJpegQ | kVarPacked>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b64 cap 8 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ | kVarPacked, 8>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b64 cap 12 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ | kVarPacked, 12>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b64 cap 20 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ | kVarPacked, 20>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b64 uncapped", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ | kVarPacked, 0>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 library b512 (6-op) again", prod_i8_fwd<I8>, 2, 1, true},
        {"jqi8b", "fwd u8->i8 jpegq packed b512 again", prod_i8_fwd<I8 | kVarJpegQ | kVarPacked>, 2, 1, true},
        // round 4, session 3: int8 block sizes with and without the JPEG forms; headline cap 7 vs 10 repeated
        {"jqi8c", "fwd u8->i8 6-op b512", prod_i8_fwd<(I8 & ~(3u << 12)) | (2u << 12)>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 6-op b256", prod_i8_fwd<(I8 & ~(3u << 12))>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 jpegq b512", prod_i8_fwd<(I8 & ~(3u << 12)) | (2u << 12) | kVarJpegQ>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 jpegq b256", prod_i8_fwd<(I8 & ~(3u << 12)) | kVarJpegQ>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 jpegq b64 uncapped", prod_i8_fwd<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 6-op b256 again", prod_i8_fwd<(I8 & ~(3u << 12))>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 jpegq b256 again", prod_i8_fwd<(I8 & ~(3u << 12)) | kVarJpegQ>, 2, 1, true},
        {"jqi8c", "fwd u8->i8 jpegq b512 again", prod_i8_fwd<(I8 & ~(3u << 12)) | (2u << 12) | kVarJpegQ>, 2, 1, true},
        {"jqcap", "fwd u8->f32 jpegq cap 10 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 7 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 9 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 9>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 10 w/cu b", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 7 w/cu b", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 10 w/cu c", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqcap", "fwd u8->f32 jpegq cap 7 w/cu c", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        // round 4, session 4: the cap per frame size with the JPEG forms (run at 16384^2, 2048x16384, 4096^2)
        {"capsz", "fwd u8->f32 jpegq cap 7 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq cap 8 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 8>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq cap 10 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq cap 12 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 12>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq scalar b1024 uncapped", prod_f32_fwd<(P & ~(3u << 12)) | (3u << 12) | kVarJpegQ>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq cap 7 w/cu again", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        {"capsz", "fwd u8->f32 jpegq cap 12 w/cu again", prod_f32_fwd_cap<PK1 | kVarJpegQ, 12>, 5, 4, true},
        // round 4, session 5: the fp32 duo inverse's cap below 10 (the headline moved from 10 to 7)
        {"invc", "inv f32->f32 duo b64 cap 10 w/cu (product)", inv_cap_v<kDuoVar | (1u << 12), 10>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 6 w/cu", inv_cap_v<kDuoVar | (1u << 12), 6>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 7 w/cu", inv_cap_v<kDuoVar | (1u << 12), 7>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 8 w/cu", inv_cap_v<kDuoVar | (1u << 12), 8>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 10 w/cu again", inv_cap_v<kDuoVar | (1u << 12), 10>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 7 w/cu again", inv_cap_v<kDuoVar | (1u << 12), 7>, 8, 4, true},
        {"invc", "inv f32->f32 duo b64 cap 8 w/cu again", inv_cap_v<kDuoVar | (1u << 12), 8>, 8, 4, true},
        // int8 forward, one-wave workgroups at higher caps (VALU-bound: needs waves)
        {"i8cap", "fwd u8->i8 jpegq b256 (product)", prod_i8_fwd<I8 | kVarJpegQ>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b64 cap 16 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 16>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b64 cap 20 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 20>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b64 cap 24 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 24>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b256 cap 24 w/cu", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | kVarJpegQ, 6>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b256 (product) again", prod_i8_fwd<I8 | kVarJpegQ>, 2, 1, true},
        {"i8cap", "fwd u8->i8 jpegq b64 cap 20 w/cu again", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 20>, 2, 1, true},
        // the u8 -> int8 product alone, for counter passes (tools/gpu_session.sh pmcsq:...:i8lim)
        {"i8lim", "fwd u8->i8 jpegq b64 cap 20 w/cu (product)", prod_i8_fwd_cap<(I8 & ~(3u << 12)) | (1u << 12) | kVarJpegQ, 20>, 2, 1, true},
        // round trip workgroup size
        {"jqrtb", "rt + sums, jpegq b512", rt_q<true, 2>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq b256", rt_qb<true, 2, 256>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq b1024", rt_qb<true, 2, 1024>, 6, 1, true},
        {"jqrtb", "rt no sums, jpegq b512", rt_q<false, 2>, 6, 1, true},
        {"jqrtb", "rt no sums, jpegq b256", rt_qb<false, 2, 256>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq b512 again", rt_q<true, 2>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq b256 again", rt_qb<true, 2, 256>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq, zeroed by write-value", rt_wv<2>, 6, 1, true},
        {"jqrtb", "rt + sums, jpegq b512 again 2", rt_q<true, 2>, 6, 1, true},
        // round trip: which cache line the sums go to, memset or not
        {"rtring", "rt sums: one struct, accumulate", rt_where<0>, 6, 1, true},
        {"rtring", "rt sums: ring slot, accumulate", rt_where<1>, 6, 1, true},
        {"rtring", "rt sums: ring slot + 24 B copy", rt_where<2>, 6, 1, true},
        {"rtring", "rt sums: memset one struct (product)", rt_where<3>, 6, 1, true},
        {"rtring", "rt sums: memset ring slot", rt_where<4>, 6, 1, true},
        {"rtring", "rt no sums", rt_qb<false, 2, 256>, 6, 1, true},
        {"rtring", "rt sums: slot + finish kernel", rt_where<5>, 6, 1, true},
        {"rtring", "rt sums: one struct, accumulate again", rt_where<0>, 6, 1, true},
        {"rtring", "rt sums: ring slot, accumulate again", rt_where<1>, 6, 1, true},
        {"rtring", "rt sums: memset one struct again", rt_where<3>, 6, 1, true},
        {"rtring", "rt sums: ring slot + 24 B copy again", rt_where<2>, 6, 1, true},
        {"rtring", "rt sums: slot + finish kernel again", rt_where<5>, 6, 1, true},
        // the headline cap below 8 with the JPEG forms (fewer VALU per set)
        {"jqf", "fwd u8->f32 jpegq cap 10 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqf", "fwd u8->f32 jpegq cap 6 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 6>, 5, 4, true},
        {"jqf", "fwd u8->f32 jpegq cap 7 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 7>, 5, 4, true},
        {"jqf", "fwd u8->f32 jpegq cap 8 w/cu", prod_f32_fwd_cap<PK1 | kVarJpegQ, 8>, 5, 4, true},
        {"jqf", "fwd u8->f32 jpegq cap 10 w/cu again", prod_f32_fwd_cap<PK1 | kVarJpegQ, 10>, 5, 4, true},
        {"jqrt", "rt + sums, library (6-op)", rt_q<true, 1>, 6, 1, true},
        {"jqrt", "rt + sums, jpegq", rt_q<true, 2>, 6, 1, true},
        {"jqrt", "rt no sums, library (6-op)", rt_q<false, 1>, 6, 1, true},
        {"jqrt", "rt no sums, jpegq", rt_q<false, 2>, 6, 1, true},
        {"jqrt", "rt + sums, library (6-op) again", rt_q<true, 1>, 6, 1, true},
        {"jqrt", "rt + sums, jpegq again", rt_q<true, 2>, 6, 1, true},
        {"pat", "pat one set per wave (grid)", pat_grid_go, 5, 4, false},
        {"pat", "pat band 4 w/cu", pat_band_go<4, false>, 5, 4, false},
        {"pat", "pat band 4 w/cu prefetch", pat_band_go<4, true>, 5, 4, false},
        {"pat", "pat band 8 w/cu", pat_band_go<8, false>, 5, 4, false},
        {"pat", "pat band 8 w/cu prefetch", pat_band_go<8, true>, 5, 4, false},
        {"pat", "pat band 16 w/cu", pat_band_go<16, false>, 5, 4, false},
        {"pat", "pat band 16 w/cu prefetch", pat_band_go<16, true>, 5, 4, false},
        {"pat", "pat band 32 w/cu", pat_band_go<32, false>, 5, 4, false},
        {"pat", "pat one set per wave (grid) again", pat_grid_go, 5, 4, false},
        {"pat", "pat band 2 w/cu prefetch", pat_band_go<2, true>, 5, 4, false},
    };
    vars.erase(std::remove_if(vars.begin(), vars.end(),
                              [&](const Variant& v) { return only != "all" && v.group != only; }),
               vars.end());

    std::vector<uint8_t*> img(nsets);
    std::vector<void*> out(nsets);
    std::vector<uint8_t> h(px);
    srand(42);
    for (size_t i = 0; i < px; ++i) h[i] = (uint8_t)(rand() % 256);
    for (int s = 0; s < nsets; ++s) {
        CK(hipMalloc(&img[s], px));
        CK(hipMalloc(&out[s], px * 4));
        if (s == 0) {
            CK(hipMemcpy(img[s], h.data(), px, hipMemcpyHostToDevice));
        } else {
            CK(launch_fill_hash_impl(img[s], px, 1000u + s, 0, 0));
        }
    }
    const bool want_rt = std::any_of(vars.begin(), vars.end(), [](const Variant& v) { return v.group == "rtpk"; });
    const bool want_coef = std::any_of(vars.begin(), vars.end(), [](const Variant& v) {
        return v.group == "rtpk" || v.group == "rtocc" || v.group == "invocc" || v.group == "invb" ||
               v.group == "dropin" || v.group == "dropcap" || v.group == "fwdcap" || v.group == "duocap16" || v.group == "jqrt" || v.group == "jqrtb" || v.group == "invc" ||
               v.group == "rtring";
    });
    if (want_coef) {
        g_img = img;
        g_coef.resize(nsets);
        for (auto& p : g_coef) CK(hipMalloc(&p, px * 4));
        if (std::any_of(vars.begin(), vars.end(),
                        [](const Variant& v) {
                            return v.group == "dropin" || v.group == "dropcap" || v.group == "fwdcap" || v.group == "duocap16";
                        })) {
            g_shift.resize(nsets);
            for (auto& p : g_shift) CK(hipMalloc(&p, px * 4));
            CK(hipMalloc(&g_T, 64 * sizeof(float)));
            CK(hipMemcpy(g_T, kBuiltinT.v, 64 * sizeof(float), hipMemcpyHostToDevice));
        }
        CK(hipMalloc(&g_sums, sizeof(RtSums)));
        CK(hipMalloc(&g_sums_ring, kRing * sizeof(RtSums)));
        CK(hipMemset(g_sums_ring, 0, kRing * sizeof(RtSums)));
        // the inverse's input: each set's quantised coefficients (the forward of its frame)
        for (int k = 0; k < nsets; ++k) hipLaunchKernelGGL((hpdct::fdct_kernel<uint8_t, float, true, true, false, kProdVar<uint8_t, float> | kVarFastDiv>),
                                                           grid_for(c.g, false, c.cus, 512), dim3(512), 0, 0, img[k], g_coef[k], nullptr, c.g, nullptr, c.qp, 128.0f);
    }
    CK(hipDeviceSynchronize());
    if (want_rt) {  // coefficients and sums of the packed round trip == the library's, set 1
        std::vector<float> c0(px), c1(px);
        RtSums s0, s1;
        rt_prod<true>(img[1], out[2], c, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(c0.data(), g_coef[1], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&s0, g_sums, sizeof(s0), hipMemcpyDeviceToHost));
        CK(hipMemset(g_coef[1], 0xa5, px * 4));
        rt_pk<true>(img[1], out[2], c, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(c1.data(), g_coef[1], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&s1, g_sums, sizeof(s1), hipMemcpyDeviceToHost));
        const bool cok = memcmp(c0.data(), c1.data(), px * 4) == 0;
        const bool sok = memcmp(&s0, &s1, sizeof(s0)) == 0;
        printf("check rt packed coefficients %s, sums %s (sse_u8 %llu sum_x2 %llu sse_f32_fx %llu)\n",
               cok ? "bit-exact" : "MISMATCH", sok ? "identical" : "DIFFER", (unsigned long long)s1.sse_u8,
               (unsigned long long)s1.sum_x2, (unsigned long long)s1.sse_f32_fx);
        if (!cok || !sok) return 1;
    }
    if (std::any_of(vars.begin(), vars.end(), [](const Variant& v) { return v.group == "rtring"; })) {
        // the finish kernel's sums == memset + atomics, launch after launch, and its slot zero after each
        for (int rep = 0; rep < 4; ++rep) {
            RtSums s0, s1, z;
            rt_where<3>(img[rep & 1], out[2], c, 0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(&s0, g_sums, sizeof(s0), hipMemcpyDeviceToHost));
            CK(hipMemset(g_sums, 0xa5, sizeof(RtSums)));
            rt_where<5>(img[rep & 1], out[2], c, 0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(&s1, g_sums, sizeof(s1), hipMemcpyDeviceToHost));
            CK(hipMemcpy(&z, g_sums_ring + kRing - 1, sizeof(z), hipMemcpyDeviceToHost));
            const bool sok = memcmp(&s0, &s1, sizeof(s0)) == 0;
            const bool zok = (z.sse_f32_fx | z.sse_u8 | z.sum_x2) == 0;
            printf("check rt finish sums set %d: %s (sse_u8 %llu), slot %s\n", rep & 1, sok ? "identical" : "DIFFER",
                   (unsigned long long)s1.sse_u8, zok ? "zero" : "NOT ZERO");
            if (!sok || !zok) return 1;
        }
    }
    // correctness: each variant against its group's first entry, on sets 0 and 1
    {
        std::vector<uint8_t> ref(px * 4), got(px * 4);
        for (int s = 0; s < 2; ++s) {
            std::string cur;
            for (auto& v : vars) {
                const size_t nb = px * v.obpp;
                CK(hipMemset(out[2], 0xa5, nb));
                v.launch(img[s], out[2], c, 0);
                const hipError_t le = hipGetLastError();
                if (le != hipSuccess) {
                    printf("check %-40s LAUNCH FAILED: %s\n", v.name.c_str(), hipGetErrorString(le));
                    return 1;
                }
                CK(hipDeviceSynchronize());
                if (v.group != cur) {
                    cur = v.group;
                    CK(hipMemcpy(ref.data(), out[2], nb, hipMemcpyDeviceToHost));
                    continue;
                }
                if (!v.check) continue;
                CK(hipMemcpy(got.data(), out[2], nb, hipMemcpyDeviceToHost));
                size_t bad = 0;
                for (size_t i = 0; i < nb; ++i) bad += ref[i] != got[i];
                printf("check set %d %-40s %s", s, v.name.c_str(), bad ? "MISMATCH" : "bit-exact\n");
                if (bad) {
                    printf(" (%zu bytes)\n", bad);
                    return 1;
                }
            }
        }
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(vars.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int w = 0; w < 2 * nsets; ++w) vars[v].launch(img[w % nsets], out[w % nsets], c, 0);
            for (int i = 0; i < iters; i += nsets) {
                CK(hipEventRecord(a, 0));
                for (int k = 0; k < nsets; ++k) vars[v].launch(img[k], out[k], c, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                us[v].push_back(ms * 1e3f / nsets);
            }
        }
    }
    printf("%-42s %10s %10s %6s %8s\n", "variant", "median_us", "min_us", "B/px", "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = us[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        printf("%-42s %10.2f %10.2f %6.0f %8.3f\n", vars[v].name.c_str(), med, t[0], vars[v].bpp,
               vars[v].bpp * px / (med * 1e-6) / 8e12);
    }
    return 0;
}
