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

#include "hpdct_launch.hpp"
#include "kbench_variants.hpp"
#include "hpdct_duo.hpp"

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

// ---------------------------------------------------------------------------
// A/B: the north_star's sketch -- one wavefront per 8x8 tile, lane (r, c) =
// pixel, row/column passes through wavefront shuffles (ds_bpermute), u8 rows
// loaded wide and staged in LDS, T rows per lane in VGPRs (the FMA constants
// differ per lane, so no zero-term skipping), outputs staged in LDS and
// written as 1 KiB-contiguous non-temporal stores.  Each wave walks strips of
// 8 horizontally adjacent tiles (64 px x 8 rows).  Same arithmetic: the output
// is checked bit-for-bit against the product kernel.
template <bool kUnroll>
__global__ __launch_bounds__(256) void wave_per_tile_kernel(const uint8_t* __restrict__ img, float* __restrict__ out,
                                                            TileGrid g, QParams qp) {
    __shared__ uint2 sin[4][64];        // per wave: 8 rows x 8 tiles x 8 B
    __shared__ float sout[4][8 * 64];   // per wave: 8 rows x 64 floats
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t r = lane >> 3, c = lane & 7u;
    float trow[8], tcol[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        trow[i] = kBuiltinT.v[r * 8 + i];  // column pass: T[r][i]
        tcol[i] = kBuiltinT.v[c * 8 + i];  // row pass: T[c][i]
    }
    const float qv = qp.q.v[r * 8 + c], rv = qp.r.v[r * 8 + c];
    const uint32_t strips = g.ntiles / 8u;  // tiles_x multiple of 8 assumed (checked by the launcher)
    const uint32_t strip = (blockIdx.x * 4u + w);
    if (strip >= strips) return;
    const uint32_t t0 = strip * 8u;
    const uint32_t ty = t0 / g.tiles_x, tx = t0 - ty * g.tiles_x;
    const uint64_t base = (uint64_t)ty * 8u * g.width + (uint64_t)tx * 8u;
    // lane l loads tile (l & 7), row (l >> 3): 8 rows x 64 contiguous bytes
    sin[w][r * 8 + c] = *reinterpret_cast<const uint2*>(img + base + r * g.width + 8u * c);
    __builtin_amdgcn_wave_barrier();
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(sin[w]);
    auto tile = [&](int k) {
        const float x = (float)sb[r * 64 + 8 * k + c] - 128.0f;
        float p = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float xi = __int_as_float(__builtin_amdgcn_ds_bpermute((int)((i * 8 + c) << 2), __float_as_int(x)));
            p = __builtin_fmaf(trow[i], xi, p);
        }
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float pi = __int_as_float(__builtin_amdgcn_ds_bpermute((int)((r * 8 + i) << 2), __float_as_int(p)));
            s = __builtin_fmaf(pi, tcol[i], s);
        }
        sout[w][r * 64 + 8 * k + c] = quantise<kVarFastDiv>(s, qv, rv);  // the product's verified quotient
    };
    if constexpr (kUnroll) {
        unroll<8>([&](auto k) { tile(k); });
    } else {
#pragma unroll 1
        for (int k = 0; k < 8; ++k) tile(k);
    }
    __builtin_amdgcn_wave_barrier();
    // 8 rows x 256 B: two rows per 1 KiB... each lane stores float4 j of row (j / 16)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t j = h * 64u + lane;   // float4 index in the 8 x 16 strip
        const uint32_t row = j >> 4, col4 = j & 15u;
        const float4 v = reinterpret_cast<const float4*>(sout[w])[row * 16 + col4];
        float4* dst = reinterpret_cast<float4*>(out + base + row * g.width) + col4;
        __builtin_nontemporal_store(v.x, &dst->x);
        __builtin_nontemporal_store(v.y, &dst->y);
        __builtin_nontemporal_store(v.z, &dst->z);
        __builtin_nontemporal_store(v.w, &dst->w);
    }
}

template <bool kUnroll>
void launch_wave_per_tile(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                          hipStream_t s) {
    const uint32_t strips = g.ntiles / 8u;
    hipLaunchKernelGGL(wave_per_tile_kernel<kUnroll>, dim3((strips + 3) / 4), dim3(256), 0, s, in, out, g, qp);
}

struct Variant {
    std::string name;
    void (*launch)(const uint8_t*, float*, const TileGrid&, const QParams&, uint32_t cus, hipStream_t);
    bool f32_input = false;  // reads the fp32 frame set instead of the uint8 one
};

template <unsigned kVar>
void launch_var(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus, hipStream_t s) {
    const dim3 grid = grid_for(g, (kVar & ab::kVarPersist) != 0, cus, kBlock<kVar>);
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar>), grid, dim3(kBlock<kVar>), 0, s, in,
                       out, nullptr, g, nullptr, qp, 128.0f);
}

template <unsigned kVar, uint32_t kWavesPerCU>
void launch_var_occ(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    const uint32_t sets = (g.ntiles + 63u) / 64u;
    uint32_t blocks = std::min<uint32_t>((sets + 3) / 4, cus * kWavesPerCU / 4);
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar>), dim3(blocks), dim3(kBlockThreads), 0,
                       s, in, out, nullptr, g, nullptr, qp, 128.0f);
}

// other kernels of the path: buffers reinterpreted (inputs are valid for every type:
// u8 pixels, small ints as int8, fp32 read from the fp32 output of a previous run)
template <typename TI, typename TO, unsigned kVar>
void launch_fwd_any(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<TI, TO, true, true, false, kVar>), grid_for(g, false, cus, kBlock<kVar>),
                       dim3(kBlock<kVar>),
                       0, s, reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr, g, nullptr, qp,
                       128.0f);
}
template <typename TI, typename TO, unsigned kVar>
void launch_inv_any(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                    hipStream_t s) {
    hipLaunchKernelGGL((ab::idct_kernel<TI, TO, true, true, kVar>), grid_for(g, false, cus, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr, g, nullptr, qp.q, 128.0f);
}

template <typename TI, typename TO, unsigned kVar>
void launch_fwd_oct(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL((fdct_octet_kernel<TI, TO, true, true, false, kVar>), octet_grid(g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr,
                       g, nullptr, qp, 128.0f);
}
template <typename TI, typename TO, unsigned kVar>
void launch_inv_oct(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL((idct_octet_kernel<TI, TO, true, true, kVar>), octet_grid(g, kBlock<kVar>), dim3(kBlock<kVar>),
                       0, s, reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr, g, nullptr, qp.q,
                       128.0f);
}

// compat-path shape: runtime T (device buffer), X-128 written back (to a scratch plane here)
float* g_T = nullptr;
float* g_wb = nullptr;
template <unsigned kVar>
void launch_fwd_compat_tile(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                            hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<float, float, true, false, true, kVar>), grid_for(g, false, 0, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp, 128.0f);
}
template <unsigned kVar>
void launch_fwd_compat_duo(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                           hipStream_t s) {
    hipLaunchKernelGGL((fdct_duo_kernel<true, false, true, kVar>), duo_grid(g, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp, 128.0f);
}
template <unsigned kVar>
void launch_fwd_compat_oct(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                           hipStream_t s) {
    hipLaunchKernelGGL((fdct_octet_kernel<float, float, true, false, true, kVar>), octet_grid(g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp, 128.0f);
}
// cublasDCTv2 order: runtime T, X-128 / q*Q written back (to the scratch plane)
template <unsigned kVar>
void launch_cublas_fwd_tile(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                            hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<float, float, true, false, true, kVar | kVarRowFirst>),
                       grid_for(g, false, 0, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp, 128.0f);
}
template <unsigned kVar>
void launch_cublas_fwd_duo(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                           hipStream_t s) {
    hipLaunchKernelGGL((rowfirst_duo_kernel<false, true, false, true, kVar>), duo_grid(g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp.q, 128.0f);
}
template <unsigned kVar>
void launch_cublas_inv_tile(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                            hipStream_t s) {
    hipLaunchKernelGGL((ab::idct_kernel<float, float, true, false, kVar | kVarRowFirst | kVarWbDequant>),
                       grid_for(g, false, 0, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp.q, 128.0f);
}
template <unsigned kVar>
void launch_cublas_inv_duo(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t,
                           hipStream_t s) {
    hipLaunchKernelGGL((rowfirst_duo_kernel<true, true, false, true, kVar>), duo_grid(g, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const float*>(in), out, g_wb, g, g_T, qp.q, 128.0f);
}
template <unsigned kVar>
void launch_fwd_duo(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL((fdct_duo_kernel<true, true, false, kVar>), duo_grid(g, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, nullptr, g, nullptr, qp, 128.0f);
}
template <unsigned kVar>
void launch_fwd_duo_rt(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL((fdct_duo_kernel<true, false, false, kVar>), duo_grid(g, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, nullptr, g, g_T, qp, 128.0f);
}
template <unsigned kVar>
void launch_inv_duo(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL((idct_duo_kernel<true, true, kVar>), duo_grid(g, kBlock<kVar>), dim3(kBlock<kVar>), 0, s,
                       reinterpret_cast<const float*>(in), out, nullptr, g, nullptr, qp.q, 128.0f);
}

template <typename TI, typename TO, unsigned kVar>
void launch_fwd_pers(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                     hipStream_t s) {
    hipLaunchKernelGGL((ab::fdct_kernel<TI, TO, true, true, false, kVar>), grid_for(g, true, cus, kBlock<kVar>),
                       dim3(kBlock<kVar>), 0, s, reinterpret_cast<const TI*>(in), reinterpret_cast<TO*>(out), nullptr,
                       g, nullptr, qp, 128.0f);
}

// the int8 forward's exact access pattern with no arithmetic: one lane per
// tile, 8 rows x 8 B loaded, the same 8 rows x 8 B stored (NT), 512-thread
// workgroups, one 64-tile set per wave
__global__ __launch_bounds__(512) void pattern_copy_u8(const uint8_t* __restrict__ in, int8_t* __restrict__ out,
                                                       TileGrid g) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 8u + threadIdx.x / 64u;
    const uint32_t tile = wave * 64u + lane;
    if (tile >= g.ntiles) return;
    const uint32_t by = tile / g.tiles_x, bx = tile - by * g.tiles_x;
    const uint64_t base = (uint64_t)by * 8u * g.width + (uint64_t)bx * 8u;
    uint2 r[8];
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + i * g.width);
    for (int i = 0; i < 8; ++i) {
        uint2* d = reinterpret_cast<uint2*>(out + base + i * g.width);
        __builtin_nontemporal_store(r[i].x ^ 0x80808080u, &d->x);
        __builtin_nontemporal_store(r[i].y ^ 0x80808080u, &d->y);
    }
}
void launch_pattern_copy(const uint8_t* in, float* out, const TileGrid& g, const QParams&, uint32_t, hipStream_t s) {
    hipLaunchKernelGGL(pattern_copy_u8, dim3((g.ntiles / 64 + 7) / 8), dim3(512), 0, s, in,
                       reinterpret_cast<int8_t*>(out), g);
}

// persistent int8 forward with next-set prefetch, kW waves per CU
template <unsigned kVar, uint32_t kW>
void launch_i8_pers_w(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t cus,
                      hipStream_t s) {
    const uint32_t per = kBlock<kVar> / 64u;
    const uint32_t sets = (g.ntiles + 63u) / 64u;
    const uint32_t blocks = std::min<uint32_t>((sets + per - 1) / per, cus * kW / per);
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>), dim3(blocks), dim3(kBlock<kVar>), 0,
                       s, in, reinterpret_cast<int8_t*>(out), nullptr, g, nullptr, qp, 128.0f);
}

template <unsigned kVar>
void launch_i8_two(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    const uint32_t sets = (g.ntiles + 63u) / 64u, per = kBlock<kVar> / 64u;
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, int8_t, true, true, false, kVar>), dim3(((sets + 1) / 2 + per - 1) / per),
                       dim3(kBlock<kVar>), 0, s, in, reinterpret_cast<int8_t*>(out), nullptr, g, nullptr, qp, 128.0f);
}
template <unsigned kVar>
void launch_f32_two(const uint8_t* in, float* out, const TileGrid& g, const QParams& qp, uint32_t, hipStream_t s) {
    const uint32_t sets = (g.ntiles + 63u) / 64u, per = kBlock<kVar> / 64u;
    hipLaunchKernelGGL((ab::fdct_kernel<uint8_t, float, true, true, false, kVar>), dim3(((sets + 1) / 2 + per - 1) / per),
                       dim3(kBlock<kVar>), 0, s, in, out, nullptr, g, nullptr, qp, 128.0f);
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

    {
        float th[64];
        for (int i = 0; i < 64; ++i) th[i] = kBuiltinT.v[i];
        CK(hipMalloc(&g_T, sizeof(th)));
        CK(hipMemcpy(g_T, th, sizeof(th), hipMemcpyHostToDevice));
        CK(hipMalloc(&g_wb, px * 4));
    }
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
    constexpr unsigned F = kVarFastDiv, X = ab::kVarXorCvt, L = kVarLdsStore, N = kVarNT, P = ab::kVarPersist;
    constexpr unsigned B = L | N | F, R = ab::kVarRowMajor, S = ab::kVarLdsSwz, W512 = 2u << 12, W1024 = 3u << 12;
    constexpr unsigned LL = ab::kVarLdsLoad;
    constexpr unsigned NL = ab::kVarNTLoad, IP = kVarI8Pack;
    constexpr unsigned PK = ab::kVarPacked, OR = kOctRestage;
    // u8 -> fp32 quantised (the headline kernel): each checked against "plain"
    std::vector<Variant> vars = {
        {"copy_linear(5B/px ceiling)", launch_copy_linear},
        {"u8->f32 tile (product)", launch_var<B | W512>},
        {"u8->f32 tile packed", launch_var<B | W512 | PK>},
        {"u8->f32 tile st sc1 nt", launch_var<B | W512 | ab::kVarStSc1>},
        {"u8->f32 tile st sc1", launch_var<(B & ~N) | W512 | ab::kVarStSc1>},
        {"u8->f32 tile st sc0sc1 nt", launch_var<B | W512 | ab::kVarStSc0Sc1>},
        {"u8->f32 tile st sc0sc1", launch_var<(B & ~N) | W512 | ab::kVarStSc0Sc1>},
        {"u8->f32 tile plain st", launch_var<(B & ~N) | W512>},
        {"u8->f32 octet", launch_fwd_oct<uint8_t, float, F | N | OR>},
        {"u8->f32 tile xcd-swz", launch_var<B | W512 | ab::kVarXcdSwz>},
        {"u8->f32 tile (product)", launch_var<B | W512>},
    };
    // pairs (2k, 2k+1), checked bit-exact against each other
    std::vector<Variant> other = {
        {"fwd f32 tile", launch_fwd_any<float, float, L | N | W512>, true},
        {"fwd f32 duo", launch_fwd_duo<N>, true},
        {"fwd f32 tile", launch_fwd_any<float, float, L | N | W512>, true},
        {"fwd f32 octet", launch_fwd_oct<float, float, N | OR>, true},
        {"fwd f32 duo", launch_fwd_duo<N>, true},
        {"fwd f32 duo runtime-T", launch_fwd_duo_rt<N>, true},
        {"fwd f32 duo", launch_fwd_duo<N>, true},
        {"fwd f32 duo tight", launch_fwd_duo<N | kDuoTight>, true},
        {"inv f32 tile", launch_inv_any<float, float, L | N | W512>, true},
        {"inv f32 duo", launch_inv_duo<N>, true},
        {"inv f32 tile", launch_inv_any<float, float, L | N | W512>, true},
        {"inv f32 octet", launch_inv_oct<float, float, N | OR>, true},
        {"compat fwd tile", launch_fwd_compat_tile<L | N | W512>, true},
        {"compat fwd duo", launch_fwd_compat_duo<N>, true},
        {"compat fwd tile", launch_fwd_compat_tile<L | N | W512>, true},
        {"compat fwd octet", launch_fwd_compat_oct<N | OR>, true},
        {"cublas fwd tile", launch_cublas_fwd_tile<L | N | W512>, true},
        {"cublas fwd duo", launch_cublas_fwd_duo<N>, true},
        {"cublas inv tile", launch_cublas_inv_tile<L | N | W512>, true},
        {"cublas inv duo", launch_cublas_inv_duo<N>, true},
        {"pattern copy u8->i8 (no math)", launch_pattern_copy},
        {"pattern copy u8->i8 (no math)", launch_pattern_copy},
        {"fwd u8->i8 tile", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP>},
        {"fwd u8->i8 two sets", launch_i8_two<F | N | W512 | IP | ab::kVarTwoSets>},
        {"fwd u8->i8 tile", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP>},
        {"fwd u8->i8 two sets b256", launch_i8_two<F | N | IP | ab::kVarTwoSets>},
        {"u8->f32 tile", launch_fwd_any<uint8_t, float, B | W512>},
        {"u8->f32 two sets", launch_f32_two<B | W512 | ab::kVarTwoSets>},
        {"fwd u8->i8 tile", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP>},
        {"fwd u8->i8 tile packed", launch_fwd_any<uint8_t, int8_t, F | N | W512 | PK>},
        {"fwd u8->i8 tile", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP>},
        {"fwd u8->i8 octet", launch_fwd_oct<uint8_t, int8_t, F | N>},
        {"inv i8->u8 tile", launch_inv_any<int8_t, uint8_t, N | W512>},
        {"inv i8->u8 octet", launch_inv_oct<int8_t, uint8_t, N>},
        {"fwd u8->i8 tile", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP>},
        {"fwd u8->i8 tile xcd-swz", launch_fwd_any<uint8_t, int8_t, F | N | W512 | IP | ab::kVarXcdSwz>},
        {"inv i8->u8 tile", launch_inv_any<int8_t, uint8_t, N | W512>},
        {"inv i8->u8 tile xcd-swz", launch_inv_any<int8_t, uint8_t, N | W512 | ab::kVarXcdSwz>},
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
        const size_t nb = (other[v].name.find("->u8") != std::string::npos ||
                           other[v].name.find("->i8") != std::string::npos) ? px : px * 4;
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
            // back-to-back region (no per-launch sync: small frames would time the
            // launch latency), average per launch; repeated in blocks of nsets
            for (int i = 0; i < iters; i += nsets) {
                CK(hipEventRecord(a, 0));
                for (int k = 0; k < 8 * nsets; ++k) vars[v].launch(src(k), out[k % nsets], g, qp, cus, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                for (int k = 0; k < nsets; ++k) us[v].push_back(ms * 1e3f / (8 * nsets));
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
