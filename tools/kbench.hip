// kbench.hip -- development micro-benchmark: A/B of the forward kernel
// variants on one 8192x8192 uint8 frame -> fp32 quantised coefficients, with
// rotating buffer sets (> 1 GB) so the Infinity Cache cannot serve the
// stream, plus copy kernels with the same traffic (1 B read + 4 B written per
// pixel) as the practical HBM ceiling.  Every variant's output is compared
// bit-for-bit with the plain variant's.  Interleaved rounds in one process
// (cdna_hip_programming.md rule 24).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//          -I../include -I../cuda-dct-idct_amd/csrc kbench.hip -o kbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hpdct_kernels_impl.hpp"

using namespace hpdct;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

// same access pattern as the tile kernel: per lane 8 x uint2 loads, 16 x float4 stores
__global__ __launch_bounds__(256) void copy_tilepattern(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                        TileGrid g) {
    const uint32_t tile = blockIdx.x * 256u + threadIdx.x;
    if (tile >= g.ntiles) return;
    const uint32_t ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
    const uint64_t base = (uint64_t)ty * 8u * g.width + (uint64_t)tx * 8u;
    uint2 r[8];
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + i * g.width);
    for (int i = 0; i < 8; ++i) {
        float4* d = reinterpret_cast<float4*>(out + base + i * g.width);
        d[0] = make_float4(byte_f32(r[i].x, 0), byte_f32(r[i].x, 1), byte_f32(r[i].x, 2), byte_f32(r[i].x, 3));
        d[1] = make_float4(byte_f32(r[i].y, 0), byte_f32(r[i].y, 1), byte_f32(r[i].y, 2), byte_f32(r[i].y, 3));
    }
}

// perfectly coalesced: each lane reads 4 B and writes one float4, grid-stride
__global__ __launch_bounds__(256) void copy_linear(const uint32_t* __restrict__ in, float4* __restrict__ out,
                                                   uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n4; i += stride) {
        const uint32_t w = in[i];
        out[i] = make_float4(byte_f32(w, 0), byte_f32(w, 1), byte_f32(w, 2), byte_f32(w, 3));
    }
}

struct Variant {
    std::string name;
    void (*launch)(const uint8_t*, float*, const TileGrid&, const QParams&, uint32_t cus, hipStream_t);
    bool f32_input = false;  // reads the fp32 frame set instead of the uint8 one
};

template <unsigned kVar>
void launch_var(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus, hipStream_t s) {
    const dim3 grid = grid_for(g, (kVar & kVarPersist) != 0, cus, kBlock<kVar>);
    hipLaunchKernelGGL((fdct_kernel<uint8_t, float, true, true, false, kVar>), grid, dim3(kBlock<kVar>), 0, s, in,
                       out, nullptr, g, nullptr, qp, 128.0f);
}

template <unsigned kVar, uint32_t kWavesPerCU>
void launch_var_occ(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    const uint32_t sets = (g.ntiles + 63u) / 64u;
    uint32_t blocks = std::min<uint32_t>((sets + 3) / 4, cus * kWavesPerCU / 4);
    hipLaunchKernelGGL((fdct_kernel<uint8_t, float, true, true, false, kVar>), dim3(blocks), dim3(kBlockThreads), 0,
                       s, in, out, nullptr, g, nullptr, qp, 128.0f);
}

// other kernels of the path: buffers reinterpreted (inputs are valid for every type:
// u8 pixels, small ints as int8, fp32 read from the fp32 output of a previous run)
template <typename TI, typename TO, unsigned kVar>
void launch_fwd_any(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    hipLaunchKernelGGL((fdct_kernel<TI, TO, true, true, false, kVar>), grid_for(g, false, cus, kBlock<kVar>),
                       dim3(kBlock<kVar>),
                       0, s, reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr, g, nullptr, qp,
                       128.0f);
}
template <typename TI, typename TO, unsigned kVar>
void launch_inv_any(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    hipLaunchKernelGGL((idct_kernel<TI, TO, true, true, kVar>), grid_for(g, false, cus, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), g, nullptr, qp.q, 128.0f);
}

void launch_copy_tile(const uint8_t* in, float* out, const TileGrid& g, const QParams&, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL(copy_tilepattern, dim3((g.ntiles + 255) / 256), dim3(256), 0, s, in, out, g);
}
void launch_copy_linear(const uint8_t* in, float* out, const TileGrid& g, const QParams&, uint32_t cus,
                        hipStream_t s) {
    const uint64_t n4 = (uint64_t)g.ntiles * 64 / 4;
    hipLaunchKernelGGL(copy_linear, dim3(cus * 8), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(in),
                       reinterpret_cast<float4*>(out), n4);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const int iters = argc > 2 ? atoi(argv[2]) : 50;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const int nsets = 4;
    const size_t px = (size_t)n * n;
    TileGrid g{(uint32_t)(px / 64), (uint32_t)(n / 8), (uint64_t)n};
    QParams qp;
    for (int i = 0; i < 64; ++i) {
        qp.q.v[i] = kDefaultQ.v[i];
        qp.r.v[i] = 1.0f / kDefaultQ.v[i];
    }
    int dev = 0;
    CK(hipGetDevice(&dev));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));

    std::vector<uint8_t*> in(nsets), inf(nsets);
    std::vector<float*> out(nsets);
    std::vector<uint8_t> h(px);
    srand(42);
    for (size_t i = 0; i < px; ++i) h[i] = (uint8_t)(rand() % 256);
    for (int s = 0; s < nsets; ++s) {
        CK(hipMalloc(&in[s], px * 4));  // large enough for the fp32-input kernels
        CK(hipMemset(in[s], 0, px * 4));
        CK(hipMalloc(&out[s], px * 4));
        CK(hipMemcpy(in[s], h.data(), px, hipMemcpyHostToDevice));
        // fp32 frames (pixel values 0..255 as float) for the fp32-input kernels
        std::vector<float> hf(px);
        for (size_t i = 0; i < px; ++i) hf[i] = (float)h[(i * 7919u + s) % px];
        CK(hipMalloc(&inf[s], px * 4));
        CK(hipMemcpy(inf[s], hf.data(), px * 4, hipMemcpyHostToDevice));
    }
    constexpr unsigned F = kVarFastDiv, X = kVarXorCvt, L = kVarLdsStore, N = kVarNT, P = kVarPersist;
    constexpr unsigned B = L | N | F, R = kVarRowMajor, S = kVarLdsSwz, W512 = 2u << 12, W1024 = 3u << 12;
    constexpr unsigned LL = kVarLdsLoad;
    std::vector<Variant> vars = {
        {"copy_linear(5B/px ceiling)", launch_copy_linear},
        {"product (b512+lds+nt+fast)", launch_var<B | W512>},
    };
    std::vector<Variant> other = {
        {"fwd f32->f32 lds+nt b512 (8B/px)", launch_fwd_any<float, float, L | N | W512>, true},
        {"fwd f32->f32 +ldsload", launch_fwd_any<float, float, L | N | W512 | LL>, true},
        {"inv f32->f32 lds+nt b512 (8B/px)", launch_inv_any<float, float, L | N | W512>, true},
        {"inv f32->f32 +ldsload", launch_inv_any<float, float, L | N | W512 | LL>, true},
        {"fwd f32->f32 plain b256", launch_fwd_any<float, float, 0>, true},
        {"fwd f32->f32 nt-only b512", launch_fwd_any<float, float, N | W512>, true},
    };
    // correctness: every DCT variant equal to "plain" bit for bit
    std::vector<float> ref(px), got(px);
    launch_var<0>(in[0], out[0], g, qp, cus, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), out[0], px * 4, hipMemcpyDeviceToHost));
    for (size_t v = 2; v < vars.size(); ++v) {
        CK(hipMemset(out[1], 0xff, px * 4));
        vars[v].launch(in[0], out[1], g, qp, cus, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), out[1], px * 4, hipMemcpyDeviceToHost));
        const bool ok = memcmp(ref.data(), got.data(), px * 4) == 0;
        printf("check %-32s %s\n", vars[v].name.c_str(), ok ? "bit-exact" : "MISMATCH");
        if (!ok) return 1;
    }
    // pairs (other[2k], other[2k+1]) must agree bit for bit on a real fp32 frame (in[1])
    for (size_t v = 0; v + 1 < other.size(); v += 2) {
        CK(hipMemset(out[2], 0xab, px * 4));
        CK(hipMemset(out[3], 0xcd, px * 4));
        other[v].launch(other[v].f32_input ? inf[1] : in[1], out[2], g, qp, cus, 0);
        other[v + 1].launch(other[v + 1].f32_input ? inf[1] : in[1], out[3], g, qp, cus, 0);
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> A(px * 4), Bv(px * 4);
        CK(hipMemcpy(A.data(), out[2], px * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(Bv.data(), out[3], px * 4, hipMemcpyDeviceToHost));
        const size_t nb = other[v].name.find("->u8") != std::string::npos ? px : px * 4;
        const bool ok = memcmp(A.data(), Bv.data(), nb) == 0;
        printf("check %-32s == %-24s %s\n", other[v + 1].name.c_str(), other[v].name.c_str(),
               ok ? "bit-exact" : "MISMATCH");
        if (!ok) return 1;
    }
    vars.insert(vars.end(), other.begin(), other.end());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(vars.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            auto src = [&](int i) { return vars[v].f32_input ? inf[i % nsets] : in[i % nsets]; };
            for (int w = 0; w < 5; ++w) vars[v].launch(src(w), out[w % nsets], g, qp, cus, 0);
            for (int i = 0; i < iters; ++i) {
                CK(hipEventRecord(a, 0));
                vars[v].launch(src(i), out[i % nsets], g, qp, cus, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                us[v].push_back(ms * 1e3f);
            }
        }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
        printf("per-set median %-32s", vars[v].name.c_str());
        for (int st = 0; st < nsets; ++st) {
            std::vector<float> t;
            for (size_t k = 0; k < us[v].size(); ++k)
                if ((int)((k % iters) % nsets) == st) t.push_back(us[v][k]);
            std::sort(t.begin(), t.end());
            printf(" %8.2f", t[t.size() / 2]);
        }
        printf("\n");
    }
    printf("%-34s %10s %10s %10s %8s\n", "variant", "median_us", "min_us", "GB/s(5B)", "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = us[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        const double gbs = 5.0 * px / (med * 1e-6) / 1e9;
        printf("%-34s %10.2f %10.2f %10.1f %8.3f\n", vars[v].name.c_str(), med, t[0], gbs, gbs / 8000.0);
    }
    return 0;
}
