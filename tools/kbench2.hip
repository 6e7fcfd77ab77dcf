// kbench2.hip -- focused A/B of two kernels of the path on one 8192x8192
// frame, with 4 rotating buffer sets (> 1 GB, so the Infinity Cache cannot
// serve the stream):
//   inv   fp32 quantised coefficients -> uint8 pixels (the C3 round trip's
//         decode): tile (product), tile with LDS-staged 1 KiB loads, octet, duo
//   i8    uint8 pixels -> int8 coefficients (the wire format): the product,
//         s_setprio around the load phase, occupancy capped by dynamic LDS,
//         workgroup sizes, and phase splits (no load / no store / neither)
// Every variant of a group is compared bit-for-bit with the group's first
// entry (the phase-split diagnostics excepted).  Interleaved rounds.
//
//   rt    uint8 frame -> fp32 coefficients + reconstruction (+ PEEN/MSE sums):
//         the two product kernels against the one-pass round trip
//
//   wide  uint8 -> fp32 (the headline kernel) on wide / large / short frames:
//         workgroup sizes, NT loads, column panels, two sets per wave,
//         persistent waves with prefetch
//
//   kbench2 [n=8192 | HxW] [iters=64] [rounds=3] [group=all|inv|i8|rt|wide|tlb|tlb8|mfma] [sets=4] [alloc=0|1]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <string>
#include <vector>

#include "hpdct_launch.hpp"
#include "kbench_variants.hpp"
#include "kbench_mfma.hpp"
#include "hpdct_roundtrip.hpp"
#include "kbench_linread.hpp"
#include "kbench_dma.hpp"

using namespace hpdct;

// the library's process-wide mapping switch (hpdct_api.cpp): AUTO here
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
    bool check;  // compared with the group's first variant
};

// ---- inverse fp32 -> u8 ----------------------------------------------------
template <unsigned kVar>
void inv_tile(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((ab::idct_kernel<float, uint8_t, true, true, kVar>), grid_for(c.g, false, c.cus, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, static_cast<const float*>(in), static_cast<uint8_t*>(out), nullptr,
                       c.g, nullptr, c.qp.q, 128.0f);
}
template <unsigned kVar>
void inv_octet(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((idct_octet_kernel<float, uint8_t, true, true, kVar>), octet_grid(c.g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, static_cast<const float*>(in), static_cast<uint8_t*>(out), nullptr,
                       c.g, nullptr, c.qp.q, 128.0f);
}
template <unsigned kVar>
void inv_duo(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((idct_duo_kernel<true, true, kVar, uint8_t>), duo_grid(c.g, kBlock<kVar>), dim3(kBlock<kVar>),
                       0, s, static_cast<const float*>(in), static_cast<uint8_t*>(out), nullptr, c.g, nullptr,
                       c.qp.q, 128.0f);
}

// ---- forward u8 -> int8 ----------------------------------------------------
template <unsigned kVar, uint32_t kLdsBytes = 0>
void i8_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), kLdsBytes, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp,
                       128.0f);
}

// int8: two sets per wave (16 row loads up front) and persistent waves with a
// prefetch of the next set, for the VALU/memory overlap the phase split shows
template <unsigned kVar>
void i8_fwd_two(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t sets = (c.g.ntiles + 63u) / 64u, per = kBlock<kVar> / 64u;
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, int8_t, true, true, false, kVar | ab::kVarTwoSets>),
                       dim3(((sets + 1) / 2 + per - 1) / per), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp,
                       128.0f);
}
template <unsigned kVar>
void i8_fwd_persist(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, int8_t, true, true, false, kVar | ab::kVarPersist2>),
                       grid_for(c.g, true, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp,
                       128.0f);
}

// ---- forward u8 -> fp32 (the headline kernel), set order A/B on wide frames
template <unsigned kVar, uint32_t kLdsBytes = 0>
void f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), kLdsBytes, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp,
                       128.0f);
}

// two sets per wave (all 16 row loads up front) and persistent waves with a
// prefetch of the next set: half the grid / a resident grid
template <unsigned kVar>
void f32_fwd_two(const void* in, void* out, const Ctx& c, hipStream_t s) {
    const uint32_t sets = (c.g.ntiles + 63u) / 64u, per = kBlock<kVar> / 64u;
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar | ab::kVarTwoSets>),
                       dim3(((sets + 1) / 2 + per - 1) / per), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}
template <unsigned kVar>
void f32_fwd_persist(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar | ab::kVarPersist2>),
                       grid_for(c.g, true, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}

// the LIBRARY's tile kernels (hpdct_kernels_impl.hpp), for A/B of product-side variants
template <unsigned kVar>
void prod_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::fdct_kernel<uint8_t, float, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<float*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}
template <unsigned kVar>
void prod_i8_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    hipLaunchKernelGGL((hpdct::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>),
                       grid_for(c.g, false, c.cus, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), nullptr, c.g, nullptr, c.qp, 128.0f);
}

void lin_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (!lin::linread_ok(c.g)) {
        fprintf(stderr, "linread: width must be a multiple of 8192 px\n");
        exit(2);
    }
    lin::linread_go<kVarFastDiv>(static_cast<const uint8_t*>(in), static_cast<float*>(out), c.g, c.qp, s);
}

// linear input reads through an LDS-DMA double buffer, persistent workgroups (kbench_dma.hpp)
template <uint32_t kWaves, uint32_t kWgsPerCu>
void dma_f32_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (!dma::dma_ok<kWaves>(c.g)) {
        fprintf(stderr, "dma: width must be a multiple of %u px\n", kWaves * 512u);
        exit(2);
    }
    (void)dma::dma_go<kVarFastDiv, kWaves>(static_cast<const uint8_t*>(in), static_cast<float*>(out), c.g, c.qp, c.cus,
                                           kWgsPerCu, s);
}

template <bool kFast>
void mfma_i8_fwd(const void* in, void* out, const Ctx& c, hipStream_t s) {
    (void)hpdct::fdct_mfma_i8_go<kFast>(static_cast<const uint8_t*>(in), static_cast<int8_t*>(out), c.g, c.qp, s);
}

// ---- round trip u8 -> fp32 coefficients + reconstruction (+ sums) ---------
// the coefficient plane of set s is g_coef2[s] (found from the input pointer)
std::vector<uint8_t*> g_img;
std::vector<float*> g_coef2;
RtSums* g_sums = nullptr;
int set_of(const void* in) {
    for (size_t i = 0; i < g_img.size(); ++i)
        if (g_img[i] == in) return (int)i;
    return 0;
}
void rt_two_kernels(const void* in, void* out, const Ctx& c, hipStream_t s) {
    float* cf = g_coef2[set_of(in)];
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kProdVar<uint8_t, float> | kVarFastDiv>),
                       grid_for(c.g, false, c.cus, kBlock<kProdVar<uint8_t, float>>),
                       dim3(kBlock<kProdVar<uint8_t, float>>), 0, s, static_cast<const uint8_t*>(in), cf, nullptr, c.g,
                       nullptr, c.qp, 128.0f);
    (void)launch_idct_impl<float, uint8_t, true, true>(cf, static_cast<uint8_t*>(out), nullptr, c.g, nullptr, c.qp.q, 128.0f,
                                            false, s);
}
template <int kRecon, bool kStats, bool kFast>
void rt_fused(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kStats) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    (void)rt_detail::go_r<kRecon>(static_cast<const uint8_t*>(in), g_coef2[set_of(in)],
                                  kRecon == kRtReconNone ? nullptr : out, kStats ? g_sums : nullptr, c.g, c.qp,
                                  kFast, s);
}

template <int kRaw, bool kMemset = true>
void rt_raw(const void* in, void* out, const Ctx& c, hipStream_t s) {
    if (kMemset) (void)hipMemsetAsync(g_sums, 0, sizeof(RtSums), s);
    hipLaunchKernelGGL((roundtrip_kernel<kRtReconU8, true, true, kRaw, false, 512>), roundtrip_grid(c.g, 512), dim3(512), 0, s,
                       static_cast<const uint8_t*>(in), g_coef2[set_of(in)], out, g_sums, c.g, c.qp);
}

int main(int argc, char** argv) {
    // frame: "N" (N x N) or "HxW"
    int n = 8192, hgt = 8192;
    if (argc > 1) {
        n = hgt = atoi(argv[1]);
        if (const char* x = strchr(argv[1], 'x')) n = atoi(x + 1);
    }
    const int iters = argc > 2 ? atoi(argv[2]) : 64;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const std::string only = argc > 4 ? argv[4] : "all";
    const int nsets = argc > 5 ? atoi(argv[5]) : 4;  // rotating buffer sets (>= 3: the checks use sets 1..3)
    // device allocation: 0 hipMalloc per buffer, 1 hipExtMallocWithFlags(hipDeviceMallocContiguous)
    const int amode = argc > 6 ? atoi(argv[6]) : 0;
    auto dalloc = [&](auto** p, size_t bytes) {
        void* v = nullptr;
        if (amode == 1) {
            CK(hipExtMallocWithFlags(&v, bytes, hipDeviceMallocContiguous));
        } else {
            CK(hipMalloc(&v, bytes));
        }
        *p = static_cast<std::remove_pointer_t<decltype(p)>>(v);
    };
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

    // per set: u8 frame, its fp32 quantised coefficients (the inverse's input), one output plane
    std::vector<uint8_t*> img(nsets);
    std::vector<float*> coef(nsets);
    std::vector<void*> out(nsets);
    std::vector<uint8_t> h(px);
    srand(42);
    for (size_t i = 0; i < px; ++i) h[i] = (uint8_t)(rand() % 256);
    for (int s = 0; s < nsets; ++s) {
        dalloc(&img[s], px);
        dalloc(&coef[s], px * 4);
        dalloc(&out[s], px * 4);
        std::vector<uint8_t> hs(px);
        for (size_t i = 0; i < px; ++i) hs[i] = h[(i * 7919u + 13u * s) % px];
        CK(hipMemcpy(img[s], hs.data(), px, hipMemcpyHostToDevice));
        hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kProdVar<uint8_t, float>>),
                           grid_for(c.g, false, c.cus, kBlock<kProdVar<uint8_t, float>>),
                           dim3(kBlock<kProdVar<uint8_t, float>>), 0, 0, img[s], coef[s], nullptr, c.g, nullptr, c.qp,
                           128.0f);
    }
    CK(hipDeviceSynchronize());
    g_img = img;
    g_coef2.resize(nsets);
    for (int s = 0; s < nsets; ++s) dalloc(&g_coef2[s], px * 4);
    CK(hipMalloc(&g_sums, sizeof(RtSums)));

    constexpr unsigned N = kVarNT, W512 = 2u << 12, W1024 = 3u << 12, LL = ab::kVarLdsLoad, OR = kOctRestage;
    constexpr unsigned F = kVarFastDiv, IP = kVarI8Pack;
    constexpr unsigned I8 = F | N | W512 | IP;  // the product's int8 forward
    std::vector<Variant> vars = {
        {"inv", "inv f32->u8 tile (product)", inv_tile<kProdVar<float, uint8_t>>, true},
        {"inv", "inv f32->u8 tile lds-load", inv_tile<kProdVar<float, uint8_t> | LL>, true},
        {"inv", "inv f32->u8 octet", inv_octet<N | OR>, true},
        {"inv", "inv f32->u8 duo b512", inv_duo<N | W512>, true},
        {"inv", "inv f32->u8 duo b256", inv_duo<N>, true},
        {"inv", "inv f32->u8 duo b512 plain st", inv_duo<W512>, true},
        {"i8", "fwd u8->i8 (product)", i8_fwd<I8>, true},
        {"i8", "fwd u8->i8 xor+sdwa byte convert", i8_fwd<I8 | ab::kVarXorCvt>, true},
        {"i8", "fwd u8->i8 b256", i8_fwd<F | N | IP>, true},
        {"i8", "fwd u8->i8 b1024", i8_fwd<F | N | IP | W1024>, true},
        {"i8", "fwd u8->i8 lds 1 wg/cu (2 w/simd)", i8_fwd<I8, 84 * 1024>, true},
        {"i8", "fwd u8->i8 lds 2 wg/cu (4 w/simd)", i8_fwd<I8, 64 * 1024>, true},
        {"i8", "fwd u8->i8 b256 lds 3 wg/cu (3 w/simd)", i8_fwd<F | N | IP, 48 * 1024>, true},
        {"i8", "fwd u8->i8 b256 lds 4 wg/cu (4 w/simd)", i8_fwd<F | N | IP, 40 * 1024>, true},
        {"i8", "fwd u8->i8 two sets per wave", i8_fwd_two<I8>, true},
        {"i8", "fwd u8->i8 two sets per wave b256", i8_fwd_two<F | N | IP>, true},
        {"i8", "fwd u8->i8 persistent+prefetch", i8_fwd_persist<I8>, true},
        {"i8", "fwd u8->i8 persistent+prefetch b256", i8_fwd_persist<F | N | IP>, true},
        {"i8", "fwd u8->i8 (product) again", i8_fwd<I8>, true},
        {"rt", "rt two kernels fwd+inv->u8 (10 B/px)", rt_two_kernels, true},
        {"rt", "rt fused u8 recon + sums (6 B/px)", rt_fused<kRtReconU8, true, true>, true},
        {"rt", "rt fused u8 recon (6 B/px)", rt_fused<kRtReconU8, false, true>, true},
        {"rt", "rt fused u8 recon + sums, raw in VGPRs", rt_raw<0>, true},
        {"rt", "rt fused u8 recon + sums, raw re-read", rt_raw<1>, true},
        {"rt", "rt fused u8 recon + sums, raw in LDS", rt_raw<2>, true},
        {"rt", "rt sums, no memset (accumulate)", rt_raw<2, false>, true},
        {"rt", "rt sums, no memset (accumulate) again", rt_raw<2, false>, true},
        {"rt", "rt fused u8 recon + sums, raw in LDS again", rt_raw<2>, true},
        {"rt", "rt fused sums only (5 B/px)", rt_fused<kRtReconNone, true, true>, false},
        {"rt", "rt fused f32 recon + sums (9 B/px)", rt_fused<kRtReconF32, true, true>, false},
        {"rt", "rt fused u8 recon + sums, IEEE/fp32 q", rt_fused<kRtReconU8, true, false>, true},
        {"wide", "fwd u8->f32 tile (product)", f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"wide", "fwd u8->f32 tile panel 4096 px", f32_fwd<kProdVar<uint8_t, float> | F | ab::kVarPanel>, true},
        {"wide", "fwd u8->f32 tile nt loads", f32_fwd<kProdVar<uint8_t, float> | F | ab::kVarNTLoad>, true},
        {"wide", "fwd u8->f32 tile b256", f32_fwd<(kProdVar<uint8_t, float> & ~(3u << 12)) | F>, true},
        {"wide", "fwd u8->f32 tile b1024", f32_fwd<(kProdVar<uint8_t, float> & ~(3u << 12)) | W1024 | F>, true},
        {"wide", "fwd u8->f32 tile lds 1 wg/cu (2 w/simd)", f32_fwd<kProdVar<uint8_t, float> | F, 100 * 1024>, true},
        {"wide", "fwd u8->f32 tile lds 2 wg/cu (4 w/simd)", f32_fwd<kProdVar<uint8_t, float> | F, 60 * 1024>, true},
        {"wide", "fwd u8->f32 tile lds 3 wg/cu (6 w/simd)", f32_fwd<kProdVar<uint8_t, float> | F, 36 * 1024>, true},
        {"wide", "fwd u8->f32 tile b256 lds 2 wg/cu (2 w/simd)", f32_fwd<(kProdVar<uint8_t, float> & ~(3u << 12)) | F, 60 * 1024>, true},
        {"wide", "fwd u8->f32 tile b256 lds 3 wg/cu (3 w/simd)", f32_fwd<(kProdVar<uint8_t, float> & ~(3u << 12)) | F, 40 * 1024>, true},
        {"wide", "fwd u8->f32 tile two sets/wave", f32_fwd_two<kProdVar<uint8_t, float> | F>, true},
        {"wide", "fwd u8->f32 tile two sets/wave b256", f32_fwd_two<(kProdVar<uint8_t, float> & ~(3u << 12)) | F>, true},
        {"wide", "fwd u8->f32 tile persistent+prefetch", f32_fwd_persist<kProdVar<uint8_t, float> | F>, true},
        {"wide", "fwd u8->f32 tile (product) again", f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"tlb", "fwd u8->f32 library kernel", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"tlb", "fwd u8->f32 library kernel again", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"tlb8", "fwd u8->i8 library kernel", prod_i8_fwd<I8>, true},
        {"mfma", "fwd u8->i8 library tile kernel", prod_i8_fwd<I8>, true},
        {"mfma", "fwd u8->i8 MFMA first pass", mfma_i8_fwd<true>, true},
        {"mfma", "fwd u8->i8 MFMA first pass, IEEE quotient", mfma_i8_fwd<false>, true},
        {"mfma", "fwd u8->i8 library tile kernel again", prod_i8_fwd<I8>, true},
        // linear 4 KiB input reads staged through LDS (kbench_linread.hpp) against the library kernel
        {"lin", "fwd u8->f32 library (b512)", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"lin", "fwd u8->f32 linear reads via LDS (b1024)", lin_f32_fwd, true},
        {"lin", "fwd u8->f32 library b1024", prod_f32_fwd<(kProdVar<uint8_t, float> & ~(3u << 12)) | W1024 | F>, true},
        {"lin", "fwd u8->f32 library (b512) again", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"lin", "fwd u8->f32 linear reads via LDS again", lin_f32_fwd, true},
        // linear reads through an LDS-DMA double buffer (kbench_dma.hpp): waves per workgroup x workgroups per CU
        {"dma", "fwd u8->f32 library (b512)", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"dma", "fwd u8->f32 dma 8w x 2/cu", dma_f32_fwd<8, 2>, true},
        {"dma", "fwd u8->f32 dma 8w x 1/cu", dma_f32_fwd<8, 1>, true},
        {"dma", "fwd u8->f32 dma 4w x 4/cu", dma_f32_fwd<4, 4>, true},
        {"dma", "fwd u8->f32 dma 4w x 2/cu", dma_f32_fwd<4, 2>, true},
        {"dma", "fwd u8->f32 dma 16w x 1/cu", dma_f32_fwd<16, 1>, true},
        {"dma", "fwd u8->f32 dma 8w not persistent", dma_f32_fwd<8, 64>, true},
        {"dma", "fwd u8->f32 library (b512) again", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"dma", "fwd u8->f32 dma 8w x 2/cu again", dma_f32_fwd<8, 2>, true},
        // copysign as v_bitop3_b32 (library) against v_bfi_b32 (the ab:: copy)
        {"b3", "fwd u8->i8 ab copy (bfi)", i8_fwd<I8>, true},
        {"b3", "fwd u8->i8 library (bitop3)", prod_i8_fwd<I8>, true},
        {"b3", "fwd u8->i8 ab copy (bfi) again", i8_fwd<I8>, true},
        {"b3", "fwd u8->i8 library (bitop3) again", prod_i8_fwd<I8>, true},
        {"b3f", "fwd u8->f32 ab copy (bfi)", f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"b3f", "fwd u8->f32 library (bitop3)", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"b3f", "fwd u8->f32 ab copy (bfi) again", f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"b3f", "fwd u8->f32 library (bitop3) again", prod_f32_fwd<kProdVar<uint8_t, float> | F>, true},
        {"i8", "fwd u8->i8 no load (diag)", i8_fwd<I8 | ab::kVarNoLoad>, false},
        {"i8", "fwd u8->i8 no store (diag)", i8_fwd<I8 | ab::kVarNoStore>, false},
        {"i8", "fwd u8->i8 math only (diag)", i8_fwd<I8 | ab::kVarNoLoad | ab::kVarNoStore>, false},
    };
    vars.erase(std::remove_if(vars.begin(), vars.end(),
                              [&](const Variant& v) { return only != "all" && v.group != only; }),
               vars.end());
    auto src = [&](const Variant& v, int s) -> const void* {
        return v.group == "inv" ? static_cast<const void*>(coef[s]) : static_cast<const void*>(img[s]);
    };
    // correctness: each variant against its group's first entry, on set 1
    {
        std::vector<uint8_t> ref(px * 4), got(px * 4);
        std::string cur;
        for (auto& v : vars) {
            const size_t nb = v.group == "wide" || v.group == "tlb" || v.group == "b3f" || v.group == "lin" || v.group == "dma" ? px * 4 : px;  // fp32 output plane
            CK(hipMemset(out[2], 0xa5, nb));
            v.launch(src(v, 1), out[2], c, 0);
            const hipError_t le = hipGetLastError();
            if (le != hipSuccess) {
                printf("check %-40s LAUNCH FAILED: %s (skipped)\n", v.name.c_str(), hipGetErrorString(le));
                v.launch = nullptr;
                continue;
            }
            CK(hipDeviceSynchronize());
            if (v.group != cur) {
                cur = v.group;
                CK(hipMemcpy(ref.data(), out[2], nb, hipMemcpyDeviceToHost));
                printf("check %-40s reference of group %s\n", v.name.c_str(), cur.c_str());
                continue;
            }
            if (!v.check) continue;
            CK(hipMemcpy(got.data(), out[2], nb, hipMemcpyDeviceToHost));
            const bool ok = memcmp(ref.data(), got.data(), nb) == 0;
            printf("check %-40s %s\n", v.name.c_str(), ok ? "bit-exact" : "MISMATCH");
            if (!ok) return 1;
        }
    }
    // round trip: fused coefficients == two-kernel coefficients, sums == host sums of the recon
    if (only == "all" || only == "rt") {
        std::vector<float> c2(px), cf(px), rf(px), rf2(px);
        std::vector<uint8_t> r8(px), x(px);
        rt_two_kernels(img[1], out[2], c, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(c2.data(), g_coef2[1], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r8.data(), out[2], px, hipMemcpyDeviceToHost));
        CK(hipMemcpy(x.data(), img[1], px, hipMemcpyDeviceToHost));
        (void)launch_idct_impl<float, float, true, true>(g_coef2[1], static_cast<float*>(out[3]), nullptr, c.g, nullptr,
                                              c.qp.q, 128.0f, false, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(rf.data(), out[3], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemset(g_coef2[1], 0xff, px * 4));
        CK(hipMemset(out[3], 0xff, px * 4));
        rt_fused<kRtReconF32, true, true>(img[1], out[3], c, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(cf.data(), g_coef2[1], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rf2.data(), out[3], px * 4, hipMemcpyDeviceToHost));
        const bool cok = memcmp(c2.data(), cf.data(), px * 4) == 0;
        const bool rok = memcmp(rf.data(), rf2.data(), px * 4) == 0;
        RtSums hs;
        CK(hipMemcpy(&hs, g_sums, sizeof(hs), hipMemcpyDeviceToHost));
        unsigned long long e8 = 0, xx = 0;
        double ef = 0;
        for (size_t i = 0; i < px; ++i) {
            const long d = (long)x[i] - (long)r8[i];
            e8 += (unsigned long long)(d * d);
            xx += (unsigned long long)x[i] * x[i];
            const double df = (double)x[i] - (double)rf[i];
            ef += df * df;
        }
        const double ef_dev = (double)hs.sse_f32_fx / 65536.0;
        printf("check rt coefficients fused == two kernels: %s\n", cok ? "bit-exact" : "MISMATCH");
        printf("check rt fp32 recon fused == inverse kernel: %s\n", rok ? "bit-exact" : "MISMATCH");
        printf("check rt sums: sse_u8 %llu vs host %llu, sum_x2 %llu vs %llu, sse_f32 %.6f vs %.6f (rel %.2e)\n",
               hs.sse_u8, e8, hs.sum_x2, xx, ef_dev, ef, std::fabs(ef_dev - ef) / ef);
        if (!cok || !rok || hs.sse_u8 != e8 || hs.sum_x2 != xx || std::fabs(ef_dev - ef) > 1e-6 * ef) return 1;
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(vars.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            if (!vars[v].launch) continue;
            for (int w = 0; w < 2 * nsets; ++w) vars[v].launch(src(vars[v], w % nsets), out[w % nsets], c, 0);
            for (int i = 0; i < iters; i += 4 * nsets) {
                CK(hipEventRecord(a, 0));
                for (int k = 0; k < 4 * nsets; ++k) vars[v].launch(src(vars[v], k % nsets), out[k % nsets], c, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                us[v].push_back(ms * 1e3f / (4 * nsets));
            }
        }
    }
    printf("%-42s %10s %10s %9s %8s\n", "variant", "median_us", "min_us", "B/px", "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = us[v];
        if (t.empty()) continue;
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        double bpp = vars[v].group == "inv" || vars[v].group == "wide" || vars[v].group == "tlb" || vars[v].group == "b3f" || vars[v].group == "lin" || vars[v].group == "dma" ? 5.0 : 2.0;
        if (vars[v].group == "rt") {
            const std::string& nm = vars[v].name;
            bpp = nm.find("(10 B") != std::string::npos  ? 10.0
                  : nm.find("(9 B") != std::string::npos ? 9.0
                  : nm.find("(5 B") != std::string::npos ? 5.0
                                                         : 6.0;
        }
        const double gbs = bpp * px / (med * 1e-6) / 1e9;
        printf("%-42s %10.2f %10.2f %9.0f %8.3f\n", vars[v].name.c_str(), med, t[0], bpp, gbs / 8000.0);
    }
    return 0;
}
