// kb_rt.hip -- A/B of the C3 round trip: the tile-per-lane product kernel
// (hpdct_roundtrip.hpp) against the two-lanes-per-tile kernel
// (hpdct_rt_duo.hpp) at several register budgets.  One HxW uint8 frame per
// buffer set, sets rotated (16 sets at 8192^2 = 1 GiB of inputs, 4x the
// Infinity Cache), interleaved rounds, median of per-batch averages.  Before
// timing, every variant's coefficients, uint8 reconstruction and sums are
// compared byte for byte with the product's on two sets.
//
//   kb_rt [n=8192 | HxW] [iters=64] [rounds=3] [group=all (= rtduo) | ragged] [sets=16]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hpdct_launch.hpp"
#include "kbench_rtduo_pk.hpp"
#include "kbench_rtfold.hpp"

using namespace hpdct;
// the product's mapping switch lives in hpdct_api.cpp; the harness is AUTO
int hpdct::mapping_mode() { return 0; }
// the library's duo-forward launcher (hpdct_rt_duo.hip), which launch_fdct_impl calls
template <int kQ>
static hipError_t duo_fwd_lib(const uint8_t* img, float* coef, const TileGrid& g, const QParams& qp, hipStream_t s) {
    auto* const kern = fdct_duo_u8_kernel<kQ>;
    static const size_t st = static_lds_of(kern);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(g, kDuoFwdBlock), dim3(kDuoFwdBlock),
                       residency_cap_lds(st, kDuoFwdCapWgs), s, img, coef, g, qp);
    return hipGetLastError();
}
hipError_t hpdct::launch_fdct_duo_u8(const uint8_t* img, float* coef, const TileGrid& g, const QParams& qp,
                                     int qmode, hipStream_t s) {
    return qmode == 2 ? duo_fwd_lib<2>(img, coef, g, qp, s) : duo_fwd_lib<1>(img, coef, g, qp, s);
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

struct Ctx {
    TileGrid g;
    QParams qp;
    RtSums* sums;  // zeroed by the launcher (memset), as hpdct_roundtrip_u8 did through round 3
};
typedef void (*Fn)(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s);

template <bool kStats>
void tile_rt(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(c.sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, kStats, 2, 2, false, 256>), roundtrip_grid(c.g, 256), dim3(256),
                       0, s, img, coef, static_cast<void*>(recon), kStats ? c.sums : nullptr, c.g, c.qp);
}
// the product: the kernel adds into a zeroed spread slot, the finish kernel
// folds it over the caller's struct (no memset)
unsigned long long* g_spread = nullptr;
template <bool kStats, int kB, int kW, bool kPk = false, bool kRun = true>
void duo_sp(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    RtSums* const sp = reinterpret_cast<RtSums*>(kStats ? g_spread : nullptr);
    if constexpr (kPk) {
        hipLaunchKernelGGL((roundtrip_duo_pk_kernel<kStats, 2, kRtReconU8, kB, kW>), roundtrip_duo_grid(c.g, kB),
                           dim3(kB), 0, s, img, coef, recon, sp, c.g, c.qp);
    } else {
        hipLaunchKernelGGL((roundtrip_duo_kernel<kStats, 2, kRtReconU8, kRun, kB, kW>), roundtrip_duo_grid(c.g, kB),
                           dim3(kB), 0, s, img, coef, recon, sp, c.g, c.qp);
    }
    if (kStats) hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}
// finish-kernel A/B: kMode 0 the product's (shfl sums), 1 no finish at all
// (timing only: the slot keeps growing), 2 DPP sums instead of shfl
__global__ __launch_bounds__(64) void finish_dpp(RtSums* __restrict__ dst, unsigned long long* __restrict__ slot,
                                                 int accumulate) {
    const uint32_t l = threadIdx.x;
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    if (l < static_cast<uint32_t>(kRtSpread)) {
        unroll<3>([&](auto f) {
            v[f] = slot[l * kRtSpreadStride + f];
            slot[l * kRtSpreadStride + f] = 0ull;
        });
    }
    unroll<3>([&](auto f) {
        const unsigned long long sum = wave_sum_dpp(v[f] & ~kRtSseF32Invalid);
        const bool bad = __builtin_amdgcn_ballot_w64((v[f] & kRtSseF32Invalid) != 0ull) != 0ull;
        if (l == 0u) {
            auto* const d = reinterpret_cast<unsigned long long*>(dst) + f;
            unsigned long long out = accumulate ? *d + sum : sum;
            if (bad) out |= kRtSseF32Invalid;
            *d = out;
        }
    });
}
template <int kMode>
void duo_fin(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6>), roundtrip_duo_grid(c.g, 256),
                       dim3(256), 0, s, img, coef, recon,
                       reinterpret_cast<RtSums*>(kMode == 1 ? g_spread + (1u << 18) : g_spread), c.g, c.qp);
    if (kMode == 0) hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
    if (kMode == 2) hipLaunchKernelGGL(finish_dpp, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}

// runs per wave and sub-slots A/B
template <int kSets, int kN>
void duo_sn(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6, kSets, kN>),
                       roundtrip_duo_grid(c.g, 256, kSets), dim3(256), 0, s, img, coef, recon,
                       reinterpret_cast<RtSums*>(g_spread), c.g, c.qp);
    hipLaunchKernelGGL(rt_spread_finish_kernel<kN>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}

// sums decomposition: kMode 0 sums computed, no atomics (null sums); 1 one
// plain 32-B record per wave (no contention); timing only
template <int kMode>
void duo_dec(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    if (kMode == 0) {
        hipLaunchKernelGGL((roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6, 1, -64>), roundtrip_duo_grid(c.g, 256),
                           dim3(256), 0, s, img, coef, recon, nullptr, c.g, c.qp);
    } else {
        hipLaunchKernelGGL((roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6, 1, 0>), roundtrip_duo_grid(c.g, 256),
                           dim3(256), 0, s, img, coef, recon, reinterpret_cast<RtSums*>(g_spread + (1u << 18)), c.g,
                           c.qp);
    }
}

// round 6: the fold inside the round-trip kernel (tickets, the last wave
// folds; roundtrip_duo_fold_kernel): one dispatch per launch
template <int kMode>
void duo_kfold(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((roundtrip_duo_fold_kernel<true, 2, kRtReconU8, 256, 6>), roundtrip_duo_grid(c.g, 256),
                       dim3(256), 0, s, img, coef, recon, g_spread, c.sums, c.g, c.qp, kMode);
}

// the bench's sums-ring leg: one spread slot per ring entry (a library slot per
// caller sums pointer), kRing entries used in turn; kAcc: the fold adds
int g_ring_k = 0;
template <int kRing, int kAcc>
void duo_ring(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    unsigned long long* const slot = g_spread + (size_t)(g_ring_k++ % kRing) * (kRtSpreadBytes / 8);
    hipLaunchKernelGGL((roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6>), roundtrip_duo_grid(c.g, 256),
                       dim3(256), 0, s, img, coef, recon, reinterpret_cast<RtSums*>(slot), c.g, c.qp);
    hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, slot, kAcc);
}

// round 6: the duo round trip under a residency cap (dynamic-LDS reservation,
// residency_cap_lds): at most kWgs 256-thread workgroups (4 waves) per CU; the
// kernel's registers allow 6 (24 waves per CU)
template <bool kStats, int kWgs>
void duo_cap(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    auto kern = roundtrip_duo_kernel<kStats, 2, kRtReconU8, true, 256, 6>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kWgs);
    RtSums* const sp = reinterpret_cast<RtSums*>(kStats ? g_spread : nullptr);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(c.g, 256), dim3(256), dyn, s, img, coef, recon, sp, c.g, c.qp);
    if (kStats) hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}

// round 6: is a two-lanes-per-tile forward worth building for the headline?
// The duo round trip with no reconstruction and no sums moves the headline's
// bytes (1 B in, 4 B out) while still computing the inverse it then drops: an
// upper bound on a duo forward's time.  Against the headline product (the
// tile kernel, 7 waves per CU), optionally under a residency cap.
void headline_product(const uint8_t* img, float* coef, uint8_t*, const Ctx& c, hipStream_t s) {
    (void)launch_fdct_impl<uint8_t, float, true, true, false>(img, coef, nullptr, c.g, nullptr, c.qp, 128.0f, 2,
                                                              false, s);
}
// (without a reconstruction and sums the compiler drops the inverse: 583 VALU
// and 20 lane swaps per wave, 58 VGPRs -- a forward-only duo kernel).  kB:
// workgroup size; kWgs: resident workgroups per CU (0: no cap)
template <int kB, int kWgs>
void duo_fwd(const uint8_t* img, float* coef, uint8_t*, const Ctx& c, hipStream_t s) {
    auto kern = roundtrip_duo_kernel<false, 2, kRtReconNone, true, kB, 6>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kWgs);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(c.g, kB), dim3(kB), dyn, s, img, coef, nullptr, nullptr, c.g, c.qp);
}
// round 6: the int8 wire format on the duo forward (the plane passed as
// float* is written as px int8 bytes)
void headline_i8_product(const uint8_t* img, float* coef, uint8_t*, const Ctx& c, hipStream_t s) {
    (void)launch_fdct_impl<uint8_t, int8_t, true, true, false>(img, reinterpret_cast<int8_t*>(coef), nullptr, c.g,
                                                               nullptr, c.qp, 128.0f, 2, false, s);
}
template <int kWgs>
void duo_i8(const uint8_t* img, float* coef, uint8_t*, const Ctx& c, hipStream_t s) {
    auto kern = fdct_duo_u8_kernel<2, int8_t>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kWgs);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(c.g, 256), dim3(256), dyn, s, img, reinterpret_cast<int8_t*>(coef),
                       c.g, c.qp);
}
// kSets runs of 32 tiles per wave (a grid apart), forward only
template <int kSets, int kWgs>
void duo_fwd_s(const uint8_t* img, float* coef, uint8_t*, const Ctx& c, hipStream_t s) {
    auto kern = roundtrip_duo_kernel<false, 2, kRtReconNone, true, 256, 6, kSets>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kWgs);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(c.g, 256, kSets), dim3(256), dyn, s, img, coef, nullptr, nullptr,
                       c.g, c.qp);
}
// the fp32-reconstruction round trip (+ sums + fold), capped; the recon plane
// passed as uint8_t* holds px floats (group f32cap allocates them so; its
// reconstruction check against the uint8 product is moot: run with KB_CONTINUE)
template <bool kStats, int kWgs>
void duo_f32rt(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    auto kern = roundtrip_duo_kernel<kStats, 2, kRtReconF32, true, 256, 6>;
    static const size_t dyn = residency_cap_lds(static_lds_of(kern), kWgs);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(c.g, 256), dim3(256), dyn, s, img, coef, static_cast<void*>(recon),
                       reinterpret_cast<RtSums*>(kStats ? g_spread : nullptr), c.g, c.qp);
    if (kStats) hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}
template <int kWgs>
void duo_norecon(const uint8_t* img, float* coef, uint8_t* r, const Ctx& c, hipStream_t s) {
    duo_fwd<256, kWgs>(img, coef, r, c, s);
}

// the tile kernel with the product's sums path (spread sub-slot 0 + finish)
template <bool kStats>
void tile_sp(const uint8_t* img, float* coef, uint8_t* recon, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, kStats, 2, 2, false, 256>), roundtrip_grid(c.g, 256), dim3(256), 0,
                       s, img, coef, static_cast<void*>(recon), reinterpret_cast<RtSums*>(kStats ? g_spread : nullptr),
                       c.g, c.qp);
    if (kStats) hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, c.sums, g_spread, 0);
}

struct V {
    std::string group, name;
    Fn fn;
    bool stats;
    bool recon = true;  // writes the uint8 reconstruction (checked)
};

template <typename K>
int vgprs_of(K k) {
    hipFuncAttributes a{};
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k));
    return a.numRegs;
}

int main(int argc, char** argv) {
    uint64_t H = 8192, W = 8192;
    if (argc > 1) {
        const char* x = strchr(argv[1], 'x');
        if (x) {
            H = strtoull(argv[1], nullptr, 10), W = strtoull(x + 1, nullptr, 10);
        } else {
            H = W = strtoull(argv[1], nullptr, 10);
        }
    }
    const int iters = argc > 2 ? atoi(argv[2]) : 64;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const std::string only = argc > 4 ? argv[4] : "all";
    const uint64_t px = H * W;
    int nsets = argc > 5 ? atoi(argv[5]) : (int)std::max<uint64_t>(2, (4ull << 28) / px + 1);
    nsets = std::max(nsets, 2);
    Ctx c;
    c.g.tiles_x = (uint32_t)(W / 8), c.g.ntiles = (uint32_t)((H / 8) * (W / 8)), c.g.width = W;
    for (int i = 0; i < 64; ++i) c.qp.q.v[i] = kDefaultQ.v[i], c.qp.r.v[i] = 1.0f / kDefaultQ.v[i];
    CK(hipMalloc(&c.sums, sizeof(RtSums)));
    CK(hipMalloc(&g_spread, 1u << 22));  // spread sub-slots, or one 32-B record per workgroup (-1)
    CK(hipMemset(g_spread, 0, 1u << 22));

    std::vector<V> vars = {
        {"rtduo", "tile rt + sums, spread + finish", tile_sp<true>, true},
        {"rtduo", "duo + sums (product: 1 run/wave, 64 sub-slots)", duo_sp<true, 256, 6>, true},
        {"rtduo", "duo + sums, 256 sub-slots", duo_sn<1, 256>, true},
        {"rtduo", "duo + sums, 2 runs/wave", duo_sn<2, 64>, true},
        {"rtduo", "duo + sums, 2 runs/wave, 256 sub-slots", duo_sn<2, 256>, true},
        {"rtduo", "duo + sums, 4 runs/wave, 256 sub-slots", duo_sn<4, 256>, true},
        {"rtduo", "duo + sums, no finish kernel (timing)", duo_fin<1>, false},
        {"rtduo", "duo no sums", duo_sp<false, 256, 6>, false},
        {"rtduo", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"rtduo", "duo + sums, 2 runs/wave, 256 sub-slots again", duo_sn<2, 256>, true},
        {"rtduo", "duo + sums, 256 sub-slots again", duo_sn<1, 256>, true},
        {"rtduo", "tile rt + sums, spread + finish again", tile_sp<true>, true},
        // counter passes (rocprofv3 --pmc): one variant each
        {"pmc_tile", "tile rt + sums, spread + finish", tile_sp<true>, true},
        {"pmc_duo", "duo + sums (product)", duo_sp<true, 256, 6>, true},
        {"pmc_duo_nosums", "duo no sums", duo_sp<false, 256, 6>, false},
        {"pmc_tile_nosums", "tile rt no sums", tile_rt<false>, false},
        {"pmc_pk", "duo pk + sums", duo_sp<true, 256, 6, true>, true},
        {"pmc_pk_nosums", "duo pk no sums", duo_sp<false, 256, 6, true>, false},
        {"pk", "duo + sums (product)", duo_sp<true, 256, 6>, true},
        {"pk", "duo pk + sums", duo_sp<true, 256, 6, true>, true},
        {"pk", "duo no sums", duo_sp<false, 256, 6>, false},
        {"pk", "duo pk no sums", duo_sp<false, 256, 6, true>, false},
        {"pk", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"pk", "duo pk + sums again", duo_sp<true, 256, 6, true>, true},
        // any width (tiles_x not a multiple of 32): the ragged kernel only
        {"ab", "duo + sums (product)", duo_sp<true, 256, 6>, true},
        {"ab", "duo no sums", duo_sp<false, 256, 6>, false},
        {"ab", "tile rt + sums, spread + finish", tile_sp<true>, true},
        {"ab", "duo + sums, no atomics (timing)", duo_dec<0>, false},
        {"ab", "duo + sums, plain record per wave (timing)", duo_dec<1>, false},
        {"ab", "duo + sums, no finish kernel (timing)", duo_fin<1>, false},
        {"ab", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"ab", "duo no sums again", duo_sp<false, 256, 6>, false},
        {"lx", "duo + sums (product)", duo_sp<true, 256, 6>, true},
        {"lx", "duo no sums", duo_sp<false, 256, 6>, false},
        {"lx", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"occ", "duo + sums (product)", duo_sp<true, 256, 6>, true},
        {"occ", "duo + sums, w7", duo_sp<true, 256, 7>, true},
        {"occ", "duo no sums", duo_sp<false, 256, 6>, false},
        {"occ", "duo no sums, w7", duo_sp<false, 256, 7>, false},
        {"occ", "duo no sums, w8", duo_sp<false, 256, 8>, false},
        {"occ", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"fold", "duo + sums (product: kernel + fold kernel)", duo_sp<true, 256, 6>, true},
        {"fold", "duo + sums, fold in the kernel (tickets)", duo_kfold<0>, true},
        {"fold", "duo + sums, no finish kernel (timing)", duo_fin<1>, false},
        {"fold", "duo no sums", duo_sp<false, 256, 6>, false},
        {"fold", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"fold", "duo + sums, fold in the kernel again", duo_kfold<0>, true},
        {"finish", "duo + sums, atomic fold kernel (product)", duo_sp<true, 256, 6>, true},
        {"finish", "duo + sums, plain-load fold kernel (round 5)", duo_fin<2>, true},
        {"finish", "duo + sums, no fold kernel (timing)", duo_fin<1>, false},
        {"finish", "duo + sums, atomic fold kernel again", duo_sp<true, 256, 6>, true},
        {"finish", "duo + sums, plain-load fold kernel again", duo_fin<2>, true},
        {"ring", "duo + sums, one slot (product)", duo_sp<true, 256, 6>, true},
        {"ring", "duo + sums, ring of 100 slots", duo_ring<100, 0>, true},
        {"ring", "duo + sums, one slot, accumulate", duo_ring<1, 1>, false},
        {"ring", "duo + sums, ring of 100 slots, accumulate", duo_ring<100, 1>, false},
        {"ring", "duo + sums, ring of 16 slots", duo_ring<16, 0>, true},
        {"ring", "duo + sums, one slot (product) again", duo_sp<true, 256, 6>, true},
        {"ring", "duo + sums, ring of 100 slots again", duo_ring<100, 0>, true},
        {"rtcap", "duo + sums (product, uncapped: 6 WGs/CU)", duo_sp<true, 256, 6>, true},
        {"rtcap", "duo + sums, cap 5 WGs (20 waves) per CU", duo_cap<true, 5>, true},
        {"rtcap", "duo + sums, cap 4 WGs (16 waves) per CU", duo_cap<true, 4>, true},
        {"rtcap", "duo + sums, cap 3 WGs (12 waves) per CU", duo_cap<true, 3>, true},
        {"rtcap", "duo no sums (uncapped)", duo_sp<false, 256, 6>, false},
        {"rtcap", "duo no sums, cap 5 WGs per CU", duo_cap<false, 5>, false},
        {"rtcap", "duo no sums, cap 4 WGs per CU", duo_cap<false, 4>, false},
        {"rtcap", "duo no sums, cap 3 WGs per CU", duo_cap<false, 3>, false},
        {"rtcap", "duo + sums (product) again", duo_sp<true, 256, 6>, true},
        {"rtcap", "duo + sums, cap 5 WGs again", duo_cap<true, 5>, true},
        {"rtcap", "duo + sums, cap 4 WGs again", duo_cap<true, 4>, true},
        {"fwdduo", "headline product (tile, 7 waves/CU)", headline_product, false, false},
        {"fwdduo", "duo rt, no recon/sums (6 WGs/CU)", duo_norecon<0>, false, false},
        {"fwdduo", "duo rt, no recon/sums, cap 5 WGs", duo_norecon<5>, false, false},
        {"fwdduo", "duo rt, no recon/sums, cap 4 WGs", duo_norecon<4>, false, false},
        {"fwdduo", "duo rt, no recon/sums, cap 3 WGs", duo_norecon<3>, false, false},
        {"fwdduo", "duo rt, no recon/sums, cap 2 WGs", duo_norecon<2>, false, false},
        {"fwdduo", "headline product again", headline_product, false, false},
        {"fwdduo", "duo rt, no recon/sums again", duo_norecon<0>, false, false},
        {"fwdcap", "headline product (tile, 7 waves/CU)", headline_product, false, false},
        {"fwdcap", "duo fwd 256-thr, cap 5 WGs (20 waves)", duo_fwd<256, 5>, false, false},
        {"fwdcap", "duo fwd 256-thr, cap 4 WGs (16 waves)", duo_fwd<256, 4>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 12 waves", duo_fwd<64, 12>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 14 waves", duo_fwd<64, 14>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 16 waves", duo_fwd<64, 16>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 18 waves", duo_fwd<64, 18>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 20 waves", duo_fwd<64, 20>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 24 waves", duo_fwd<64, 24>, false, false},
        {"fwdcap", "duo fwd 128-thr, cap 8 WGs (16 waves)", duo_fwd<128, 8>, false, false},
        {"fwdcap", "headline product again", headline_product, false, false},
        {"fwdcap", "duo fwd 256-thr, cap 4 WGs again", duo_fwd<256, 4>, false, false},
        {"fwdcap", "duo fwd 64-thr, cap 16 waves again", duo_fwd<64, 16>, false, false},
        {"i8duo", "int8 product (tile, 20 waves/CU)", headline_i8_product, false, false},
        {"i8duo", "int8 duo fwd, uncapped (6 WGs/CU)", duo_i8<0>, false, false},
        {"i8duo", "int8 duo fwd, cap 5 WGs", duo_i8<5>, false, false},
        {"i8duo", "int8 duo fwd, cap 4 WGs", duo_i8<4>, false, false},
        {"i8duo", "int8 duo fwd, cap 3 WGs", duo_i8<3>, false, false},
        {"i8duo", "int8 product again", headline_i8_product, false, false},
        {"i8duo", "int8 duo fwd, uncapped again", duo_i8<0>, false, false},
        {"i8duo", "int8 duo fwd, cap 5 WGs again", duo_i8<5>, false, false},
        {"fwdsets", "product (duo fwd, 1 run/wave, cap 4 WGs)", headline_product, false, false},
        {"fwdsets", "duo fwd, 2 runs/wave, cap 4 WGs", duo_fwd_s<2, 4>, false, false},
        {"fwdsets", "duo fwd, 2 runs/wave, cap 3 WGs", duo_fwd_s<2, 3>, false, false},
        {"fwdsets", "duo fwd, 2 runs/wave, cap 5 WGs", duo_fwd_s<2, 5>, false, false},
        {"fwdsets", "duo fwd, 4 runs/wave, cap 4 WGs", duo_fwd_s<4, 4>, false, false},
        {"fwdsets", "duo fwd, 1 run/wave, cap 4 WGs (kernel)", duo_fwd_s<1, 4>, false, false},
        {"fwdsets", "product again", headline_product, false, false},
        {"fwdsets", "duo fwd, 2 runs/wave, cap 4 WGs again", duo_fwd_s<2, 4>, false, false},
        {"f32cap", "f32 recon + sums (product, uncapped)", duo_f32rt<true, 0>, true},
        {"f32cap", "f32 recon + sums, cap 5 WGs", duo_f32rt<true, 5>, true},
        {"f32cap", "f32 recon + sums, cap 4 WGs", duo_f32rt<true, 4>, true},
        {"f32cap", "f32 recon + sums, cap 3 WGs", duo_f32rt<true, 3>, true},
        {"f32cap", "f32 recon, no sums (uncapped)", duo_f32rt<false, 0>, false},
        {"f32cap", "f32 recon, no sums, cap 4 WGs", duo_f32rt<false, 4>, false},
        {"f32cap", "u8 recon, no sums (uncapped)", duo_sp<false, 256, 6>, false},
        {"f32cap", "u8 recon, no sums, cap 4 WGs", duo_cap<false, 4>, false},
        {"f32cap", "f32 recon + sums (product) again", duo_f32rt<true, 0>, true},
        {"f32cap", "f32 recon + sums, cap 4 WGs again", duo_f32rt<true, 4>, true},
        {"ragged", "tile rt + sums, spread + finish", tile_sp<true>, true},
        {"ragged", "duo + sums, ragged kernel", duo_sp<true, 256, 5, false, false>, true},
        {"ragged", "duo no sums, ragged kernel", duo_sp<false, 256, 5, false, false>, false},
        {"ragged", "duo + sums, ragged kernel, w6", duo_sp<true, 256, 6, false, false>, true},
    };
    vars.erase(std::remove_if(vars.begin(), vars.end(),
                              [&](const V& v) { return only == "all" ? v.group == "ragged" : v.group != only; }),
               vars.end());
    printf("frame %llux%llu, %d sets, VGPRs: tile %d, duo %d, duo pk %d, ragged %d\n", (unsigned long long)H,
           (unsigned long long)W, nsets, vgprs_of(roundtrip_kernel<kRtReconU8, true, 2, 2, false, 256>),
           vgprs_of(roundtrip_duo_kernel<true, 2, kRtReconU8, true, 256, 6>),
           vgprs_of(roundtrip_duo_pk_kernel<true, 2, kRtReconU8, 256, 6>),
           vgprs_of(roundtrip_duo_kernel<true, 2, kRtReconU8, false, 256, 5>));

    std::vector<uint8_t*> img(nsets), rec(nsets);
    std::vector<float*> coef(nsets);
    std::vector<uint8_t> h(px);
    srand(42);
    for (size_t i = 0; i < px; ++i) h[i] = (uint8_t)(rand() % 256);
    for (int s = 0; s < nsets; ++s) {
        CK(hipMalloc(&img[s], px));
        CK(hipMalloc(&rec[s], px * (only == "f32cap" ? 4 : 1)));  // f32cap: fp32 reconstructions
        CK(hipMalloc(&coef[s], px * 4));
        if (s == 0) {
            CK(hipMemcpy(img[s], h.data(), px, hipMemcpyHostToDevice));
        } else {
            const uint64_t lanes = (px + 15) / 16;
            hipLaunchKernelGGL(fill_hash_kernel, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, 0, img[s], px,
                               1000ull + s, 0ull);
        }
    }
    CK(hipDeviceSynchronize());

    // correctness: coefficients, reconstruction and sums == the product's, sets 0 and 1
    {
        std::vector<float> c0(px), c1(px);
        std::vector<uint8_t> r0(px), r1(px);
        for (int s = 0; s < 2; ++s) {
            RtSums s0{}, s1{};
            if (only == "i8duo") {  // int8 variants: the reference is the int8 product, the rest of the plane 0xa5
                CK(hipMemset(coef[2], 0xa5, px * 4));
                headline_i8_product(img[s], coef[2], rec[2], c, 0);
            } else {
                tile_rt<true>(img[s], coef[2], rec[2], c, 0);
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(c0.data(), coef[2], px * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(r0.data(), rec[2], px, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&s0, c.sums, sizeof(s0), hipMemcpyDeviceToHost));
            for (auto& v : vars) {
                CK(hipMemset(coef[2], 0xa5, px * 4));
                CK(hipMemset(rec[2], 0x5a, px));
                CK(hipMemset(c.sums, 0xee, sizeof(RtSums)));
                v.fn(img[s], coef[2], rec[2], c, 0);
                const hipError_t le = hipGetLastError();
                if (le != hipSuccess) {
                    printf("check %-40s LAUNCH FAILED: %s\n", v.name.c_str(), hipGetErrorString(le));
                    return 1;
                }
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(c1.data(), coef[2], px * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(r1.data(), rec[2], px, hipMemcpyDeviceToHost));
                CK(hipMemcpy(&s1, c.sums, sizeof(s1), hipMemcpyDeviceToHost));
                size_t bc = 0, br = 0;
                for (size_t i = 0; i < px; ++i) bc += memcmp(&c0[i], &c1[i], 4) != 0, br += r0[i] != r1[i];
                if (!v.recon) br = 0;
                const bool sok = !v.stats || memcmp(&s0, &s1, sizeof(s0)) == 0;
                printf("check set %d %-40s coef %s recon %s sums %s\n", s, v.name.c_str(),
                       bc ? "MISMATCH" : "bit-exact", !v.recon ? "-" : br ? "MISMATCH" : "bit-exact",
                       v.stats ? (sok ? "identical" : "DIFFER") : "-");
                if (bc || br || !sok) {
                    printf("  %zu coefficients, %zu pixels differ; sums %llu %llu %llu vs %llu %llu %llu\n", bc, br,
                           s0.sse_f32_fx, s0.sse_u8, s0.sum_x2, s1.sse_f32_fx, s1.sse_u8, s1.sum_x2);
                    for (size_t i = 0, n = 0; i < px && n < 8; ++i)
                        if (memcmp(&c0[i], &c1[i], 4) != 0 || r0[i] != r1[i]) {
                            printf("  px %zu (row %zu col %zu): coef %g vs %g, recon %u vs %u\n", i, i / W, i % W,
                                   c0[i], c1[i], r0[i], r1[i]);
                            ++n;
                        }
                    if (!getenv("KB_CONTINUE")) return 1;
                }
            }
        }
    }

    // KB_REC_BUFS=n: the reconstructions rotate over n planes instead of one per
    // set (the bench's C3 legs rotate two)
    const int nrec = getenv("KB_REC_BUFS") ? std::max(1, std::min(nsets, atoi(getenv("KB_REC_BUFS")))) : nsets;
    printf("reconstruction planes: %d\n", nrec);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(vars.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int w = 0; w < 2 * nsets; ++w) vars[v].fn(img[w % nsets], coef[w % nsets], rec[w % nrec], c, 0);
            for (int i = 0; i < iters; i += nsets) {
                CK(hipEventRecord(a, 0));
                for (int k = 0; k < nsets; ++k) vars[v].fn(img[k], coef[k], rec[k % nrec], c, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                us[v].push_back(ms * 1e3f / nsets);
            }
        }
    }
    printf("%-42s %10s %10s %8s\n", "variant", "median_us", "min_us", "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = us[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        printf("%-42s %10.2f %10.2f %8.3f\n", vars[v].name.c_str(), med, t[0], 6.0 * px / (med * 1e-6) / 8e12);
    }
    return 0;
}


