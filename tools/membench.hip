// membench.hip -- development micro-benchmark of the HBM ceilings that bound
// the DCT kernels on MI355X: pure read, pure write, and the 1-B-in / 4-B-out
// streaming mix of the uint8 -> fp32 forward pass, with plain and
// non-temporal stores, several per-lane widths and grid sizes.  Buffers
// rotate over 16 sets (1 GiB of u8 inputs) so the 256 MiB Infinity Cache does
// not serve the reads.  usage: membench [n=8192] [iters=40] [all|u8|f32] [sets=16]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

__device__ __forceinline__ float4 cvt4(uint32_t w) {
    return make_float4((float)(w & 255u), (float)((w >> 8) & 255u), (float)((w >> 16) & 255u), (float)(w >> 24));
}

template <bool kNT>
__device__ __forceinline__ void st4(float4* p, float4 v) {
    if constexpr (kNT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}

// 1 B in -> 4 B out, each lane 4 px per step (1 KiB contiguous store per wave-instr)
template <bool kNT>
__global__ __launch_bounds__(256) void mix_w4(const uint32_t* __restrict__ in, float4* __restrict__ out, uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n4; i += stride) st4<kNT>(&out[i], cvt4(in[i]));
}

// 16 px per lane per step: 1 uint4 load, 4 float4 stores, each store instruction 1 KiB contiguous
template <bool kNT>
__global__ __launch_bounds__(256) void mix_w16(const uint4* __restrict__ in, float4* __restrict__ out, uint64_t n16) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;
    for (uint64_t c = wave; c * 64u < n16; c += nw) {  // chunk of 64 uint4 = 1 KiB in, 4 KiB out
        const uint64_t j = c * 64u + lane;
        if (j >= n16) break;
        const uint4 w = in[j];
        // output of chunk c: 256 float4; the lane's 4 float4 are at 4*lane..4*lane+3 in the natural layout;
        // re-map so each store instruction k covers float4 [64k, 64k+64) contiguously.
        // value for position p = 64k + lane comes from lane p/4, word p%4 -> shuffle via ds_bpermute.
        uint32_t words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = 64 * k + (int)lane;
            const int src_lane = p >> 2;
            const int word = p & 3;
            uint32_t v0 = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)words[0]);
            uint32_t v1 = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)words[1]);
            uint32_t v2 = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)words[2]);
            uint32_t v3 = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)words[3]);
            const uint32_t v = word == 0 ? v0 : word == 1 ? v1 : word == 2 ? v2 : v3;
            st4<kNT>(&out[c * 256u + p], cvt4(v));
        }
    }
}

// 1 B in -> 4 B out, each wave one contiguous run of kRun pixels (kRun/256
// store instructions of 1 KiB), no grid-stride interleaving between waves
template <uint32_t kRun>
__global__ __launch_bounds__(256) void mix_run(const uint32_t* __restrict__ in, float4* __restrict__ out, uint64_t n4) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i0 = wave * (kRun / 4);
    if (i0 >= n4) return;
    uint32_t w[kRun / 256];
#pragma unroll
    for (uint32_t k = 0; k < kRun / 256; ++k) w[k] = in[i0 + 64u * k + lane];
#pragma unroll
    for (uint32_t k = 0; k < kRun / 256; ++k) st4<true>(&out[i0 + 64u * k + lane], cvt4(w[k]));
}

// The headline kernel's access pattern without its arithmetic (n x n u8 ->
// fp32, n a multiple of 4096): wave w of the grid owns 64-tile set w (8 rows x
// 512 px): 8 row loads of 512 B (8 B per lane), 16 NT stores of 1 KiB (two
// per 2 KiB output row).  8 waves per workgroup.
// kOrder 0: consecutive waves along the tile row; 1: consecutive waves down
// the tile rows (column strips of 512 px).  kWg threads per workgroup.
template <int kOrder, uint32_t kWg>
__global__ __launch_bounds__(kWg) void pat_rows8(const uint8_t* __restrict__ in, float* __restrict__ out, uint32_t n) {
    const uint32_t wave = blockIdx.x * (kWg / 64u) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t spr = n / 512u, trows = n / 8u;
    const uint32_t ty = kOrder == 0 ? wave / spr : wave % trows, sx = kOrder == 0 ? wave - ty * spr : wave / trows;
    const uint64_t base = (uint64_t)ty * 8u * n + (uint64_t)sx * 512u;
    uint2 r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + (uint64_t)i * n + 8u * lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float4* row = reinterpret_cast<float4*>(out + base + (uint64_t)i * n);
        st4<true>(row + lane, cvt4(r[i].x));
        st4<true>(row + 64u + lane, cvt4(r[i].y));
    }
}

// The int8 forward's access pattern without its arithmetic: 8 row loads and 8
// NT row stores of 512 B (8 B per lane) per 64-tile set.
__global__ __launch_bounds__(512) void pat_rows8_i8(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                    uint32_t n) {
    const uint32_t wave = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t spr = n / 512u, ty = wave / spr, sx = wave - ty * spr;
    const uint64_t base = (uint64_t)ty * 8u * n + (uint64_t)sx * 512u;
    uint2 r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + (uint64_t)i * n + 8u * lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint2* p = reinterpret_cast<uint2*>(out + base + (uint64_t)i * n + 8u * lane);
        __builtin_nontemporal_store(r[i].x ^ 0x80808080u, &p->x);
        __builtin_nontemporal_store(r[i].y ^ 0x80808080u, &p->y);
    }
}

// Half-and-half patterns (the values are not a transform; bandwidth only):
// kLinRead: each wave loads 4 KiB contiguous (wave w -> bytes [4096w, +4096),
// 4 x 1 KiB) instead of the set's 8 row pieces; kLinWrite: each wave stores
// 16 KiB contiguous (floats [4096w, +4096)) instead of the set's 8 x 2 KiB.
template <bool kLinRead, bool kLinWrite>
__global__ __launch_bounds__(512) void pat_half(const uint8_t* __restrict__ in, float* __restrict__ out, uint32_t n) {
    const uint32_t wave = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t spr = n / 512u, ty = wave / spr, sx = wave - ty * spr;
    const uint64_t base = (uint64_t)ty * 8u * n + (uint64_t)sx * 512u;
    const uint64_t lin = (uint64_t)wave * 4096u;
    uint2 r[8];
    if constexpr (kLinRead) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = *reinterpret_cast<const uint4*>(in + lin + 1024u * k + 16u * lane);
            r[2 * k] = make_uint2(v.x, v.y);
            r[2 * k + 1] = make_uint2(v.z, v.w);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + (uint64_t)i * n + 8u * lane);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float4* row = kLinWrite ? reinterpret_cast<float4*>(out + lin + 512u * i)
                                : reinterpret_cast<float4*>(out + base + (uint64_t)i * n);
        st4<true>(row + lane, cvt4(r[i].x));
        st4<true>(row + 64u + lane, cvt4(r[i].y));
    }
}

// Two sets per wave: 8 row loads of 1 KiB (16 B per lane), 8 x 4 KiB of
// output (4 NT stores of 1 KiB per row).  8 waves per workgroup.
__global__ __launch_bounds__(512) void pat_rows8x2(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                   uint32_t n) {
    const uint32_t wave = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t spr = n / 1024u, ty = wave / spr, sx = wave - ty * spr;
    const uint64_t base = (uint64_t)ty * 8u * n + (uint64_t)sx * 1024u;
    uint4 r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint4*>(in + base + (uint64_t)i * n + 16u * lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float4* row = reinterpret_cast<float4*>(out + base + (uint64_t)i * n);
        st4<true>(row + lane, cvt4(r[i].x));
        st4<true>(row + 64u + lane, cvt4(r[i].y));
        st4<true>(row + 128u + lane, cvt4(r[i].z));
        st4<true>(row + 192u + lane, cvt4(r[i].w));
    }
}

// The same workgroup footprint (8 rows x 4096 px) with the work split by row:
// wave w of the workgroup loads row w (4 KiB, 1 KiB per instruction) and
// stores it (16 KiB, 1 KiB per instruction).
__global__ __launch_bounds__(512) void pat_rowwave(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                   uint32_t n) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t bpr = n / 4096u, ty = blockIdx.x / bpr, bx = blockIdx.x - ty * bpr;
    const uint64_t base = ((uint64_t)ty * 8u + w) * n + (uint64_t)bx * 4096u;
    uint4 r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = *reinterpret_cast<const uint4*>(in + base + 1024u * k + 16u * lane);
    float4* row = reinterpret_cast<float4*>(out + base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        st4<true>(row + 256u * k + lane, cvt4(r[k].x));
        st4<true>(row + 256u * k + 64u + lane, cvt4(r[k].y));
        st4<true>(row + 256u * k + 128u + lane, cvt4(r[k].z));
        st4<true>(row + 256u * k + 192u + lane, cvt4(r[k].w));
    }
}

// write-only, each wave one contiguous run of kRun floats
template <uint32_t kRun>
__global__ __launch_bounds__(256) void write_run(float4* __restrict__ out, uint64_t n4) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i0 = wave * (kRun / 4);
    if (i0 >= n4) return;
#pragma unroll
    for (uint32_t k = 0; k < kRun / 256; ++k) st4<true>(&out[i0 + 64u * k + lane], make_float4(1.f, 2.f, 3.f, 4.f));
}

// fp32 -> fp32 (4 B in + 4 B out per px), 16 B per lane each way, grid-stride
template <bool kNT>
__global__ __launch_bounds__(256) void copy_f32(const float4* __restrict__ in, float4* __restrict__ out, uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n4; i += stride) {
        float4 v = in[i];
        v.x -= 128.f; v.y -= 128.f; v.z -= 128.f; v.w -= 128.f;
        st4<kNT>(&out[i], v);
    }
}

// 1 B in / 1 B out (the int8 forward's traffic mix): grid-stride copy of
// 8-byte (uint2) or 16-byte (uint4) lane pieces
template <typename V, bool kNT>
__global__ __launch_bounds__(256) void copy_bytes(const V* __restrict__ in, V* __restrict__ out, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
        const V v = in[i];
        if constexpr (kNT) {
            if constexpr (sizeof(V) == 8) {
                __builtin_nontemporal_store(v.x, &out[i].x);
                __builtin_nontemporal_store(v.y, &out[i].y);
            } else {
                __builtin_nontemporal_store(v.x, &out[i].x);
                __builtin_nontemporal_store(v.y, &out[i].y);
                __builtin_nontemporal_store(v.z, &out[i].z);
                __builtin_nontemporal_store(v.w, &out[i].w);
            }
        } else {
            out[i] = v;
        }
    }
}

template <bool kNT>
__global__ __launch_bounds__(256) void write_only(float4* __restrict__ out, uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n4; i += stride)
        st4<kNT>(&out[i], make_float4((float)i, 1.f, 2.f, 3.f));
}

__global__ __launch_bounds__(256) void read_only(const uint4* __restrict__ in, uint64_t n16, uint32_t* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += stride) {
        const uint4 w = in[i];
        acc ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// calibration kernels for the PMC byte counters (known byte counts, the
// access widths of the DCT kernels: dwordx2 loads, dwordx4 loads, dwordx4
// and dwordx2 non-temporal stores)
__global__ __launch_bounds__(256) void calib_read_x2(const uint2* __restrict__ in, uint64_t n8, uint32_t* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n8; i += stride) {
        const uint2 w = in[i];
        acc ^= w.x ^ w.y;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void calib_write_x2_nt(uint2* __restrict__ out, uint64_t n8) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n8; i += stride) {
        __builtin_nontemporal_store((uint32_t)i, &out[i].x);
        __builtin_nontemporal_store((uint32_t)(i >> 32), &out[i].y);
    }
}

// tile pattern (the DCT kernel's): per lane 8 rows x (8 B in, 32 B out)
template <bool kNT>
__global__ __launch_bounds__(256) void tile_mix(const uint8_t* __restrict__ in, float* __restrict__ out, uint32_t ntiles,
                                                uint32_t tiles_x, uint64_t width) {
    const uint32_t tile = blockIdx.x * 256u + threadIdx.x;
    if (tile >= ntiles) return;
    const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const uint64_t base = (uint64_t)ty * 8u * width + (uint64_t)tx * 8u;
    uint2 r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint2*>(in + base + i * width);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float4* d = reinterpret_cast<float4*>(out + base + i * width);
        st4<kNT>(d, cvt4(r[i].x));
        st4<kNT>(d + 1, cvt4(r[i].y));
    }
}

static int calib(int cus) {
    // 256 MiB buffers, each kernel 5 times: FETCH_SIZE / WRITE_SIZE per
    // dispatch divided by these byte counts = the counter's calibration
    const size_t bytes = 256ull << 20;
    void *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    for (int i = 0; i < 5; ++i) {
        hipLaunchKernelGGL(calib_read_x2, dim3(cus * 8), dim3(256), 0, 0, (const uint2*)(i & 1 ? a : b), bytes / 8,
                           sink);
        hipLaunchKernelGGL(read_only, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)(i & 1 ? a : b), bytes / 16,
                           sink);
        hipLaunchKernelGGL(write_only<true>, dim3(cus * 8), dim3(256), 0, 0, (float4*)(i & 1 ? a : b), bytes / 16);
        hipLaunchKernelGGL(write_only<false>, dim3(cus * 8), dim3(256), 0, 0, (float4*)(i & 1 ? b : a), bytes / 16);
        hipLaunchKernelGGL(calib_write_x2_nt, dim3(cus * 8), dim3(256), 0, 0, (uint2*)(i & 1 ? a : b), bytes / 8);
    }
    CK(hipDeviceSynchronize());
    printf("calibration kernels: 5 x {calib_read_x2, read_only(x4), write_only nt, write_only plain, "
           "calib_write_x2_nt}, "
           "%zu bytes each\n", bytes);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "calib") == 0) {
        int dev = 0, cus = 0;
        CK(hipGetDevice(&dev));
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        return calib(cus);
    }
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const int iters = argc > 2 ? atoi(argv[2]) : 40;
    // rotating buffer sets: the INPUT bytes of all sets must exceed the 256 MiB
    // Infinity Cache by a wide margin, or the reads are served from it (NT
    // stores do not allocate there; 4 sets of 64 MiB u8 inputs fit exactly).
    const int nsets = argc > 4 ? atoi(argv[4]) : 16;
    const size_t px = (size_t)n * n;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint8_t*> in(nsets);
    std::vector<float*> out(nsets);
    for (int s = 0; s < nsets; ++s) {
        CK(hipMalloc(&in[s], px));
        CK(hipMalloc(&out[s], px * 4));
        CK(hipMemset(in[s], s + 1, px));
    }
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    struct Case {
        std::string name;
        double bytes;
        std::function<void(int)> run;
    };
    std::vector<Case> cases;
    const uint64_t n4 = px / 4, n16 = px / 16;
    for (int gm : {1, 2, 4, 8, 16, 32}) {
        const unsigned grid = cus * gm;
        cases.push_back({"mix_w4 plain g" + std::to_string(gm), 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(mix_w4<false>, dim3(grid), dim3(256), 0, 0,
                                                (const uint32_t*)in[s], (float4*)out[s], n4);
                         }});
        cases.push_back({"mix_w4 nt    g" + std::to_string(gm), 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(mix_w4<true>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)in[s],
                                                (float4*)out[s], n4);
                         }});
    }
    for (int gm : {4, 8, 16}) {
        const unsigned grid = cus * gm;
        cases.push_back({"mix_w16 plain g" + std::to_string(gm), 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(mix_w16<false>, dim3(grid), dim3(256), 0, 0, (const uint4*)in[s],
                                                (float4*)out[s], n16);
                         }});
        cases.push_back({"mix_w16 nt    g" + std::to_string(gm), 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(mix_w16<true>, dim3(grid), dim3(256), 0, 0, (const uint4*)in[s],
                                                (float4*)out[s], n16);
                         }});
    }
    for (int gm : {2, 4, 8, 16}) {
        const unsigned grid = cus * gm;
        cases.push_back({"copy_f32 plain g" + std::to_string(gm), 8.0 * px, [=](int s) {
                             hipLaunchKernelGGL(copy_f32<false>, dim3(grid), dim3(256), 0, 0,
                                                (const float4*)out[(s + 1) % nsets], (float4*)out[s], n4);
                         }});
        cases.push_back({"copy_f32 nt    g" + std::to_string(gm), 8.0 * px, [=](int s) {
                             hipLaunchKernelGGL(copy_f32<true>, dim3(grid), dim3(256), 0, 0,
                                                (const float4*)out[(s + 1) % nsets], (float4*)out[s], n4);
                         }});
    }
    cases.push_back({"mix_run 4096 px/wave nt", 5.0 * px, [=](int s) {
                         hipLaunchKernelGGL(mix_run<4096>, dim3((unsigned)(px / 4096 / 4)), dim3(256), 0, 0,
                                            (const uint32_t*)in[s], (float4*)out[s], n4);
                     }});
    cases.push_back({"mix_run 1024 px/wave nt", 5.0 * px, [=](int s) {
                         hipLaunchKernelGGL(mix_run<1024>, dim3((unsigned)(px / 1024 / 4)), dim3(256), 0, 0,
                                            (const uint32_t*)in[s], (float4*)out[s], n4);
                     }});
    cases.push_back({"mix_run 16384 px/wave nt", 5.0 * px, [=](int s) {
                         hipLaunchKernelGGL(mix_run<16384>, dim3((unsigned)(px / 16384 / 4)), dim3(256), 0, 0,
                                            (const uint32_t*)in[s], (float4*)out[s], n4);
                     }});
    cases.push_back({"write_run 4096/wave nt", 4.0 * px, [=](int s) {
                         hipLaunchKernelGGL(write_run<4096>, dim3((unsigned)(px / 4096 / 4)), dim3(256), 0, 0,
                                            (float4*)out[s], n4);
                     }});
    cases.push_back({"write_run 16384/wave nt", 4.0 * px, [=](int s) {
                         hipLaunchKernelGGL(write_run<16384>, dim3((unsigned)(px / 16384 / 4)), dim3(256), 0, 0,
                                            (float4*)out[s], n4);
                     }});
    const uint32_t ntiles = px / 64, tiles_x = n / 8;
    cases.push_back({"tile_mix plain", 5.0 * px, [=](int s) {
                         hipLaunchKernelGGL(tile_mix<false>, dim3((ntiles + 255) / 256), dim3(256), 0, 0, in[s],
                                            out[s], ntiles, tiles_x, (uint64_t)n);
                     }});
    cases.push_back({"tile_mix nt", 5.0 * px, [=](int s) {
                         hipLaunchKernelGGL(tile_mix<true>, dim3((ntiles + 255) / 256), dim3(256), 0, 0, in[s],
                                            out[s], ntiles, tiles_x, (uint64_t)n);
                     }});
    for (int gm : {1, 2, 4, 8, 16}) {
        const unsigned grid = cus * gm;
        cases.push_back({"write_only plain g" + std::to_string(gm), 4.0 * px, [=](int s) {
                             hipLaunchKernelGGL(write_only<false>, dim3(grid), dim3(256), 0, 0, (float4*)out[s], n4);
                         }});
        cases.push_back({"write_only nt    g" + std::to_string(gm), 4.0 * px, [=](int s) {
                             hipLaunchKernelGGL(write_only<true>, dim3(grid), dim3(256), 0, 0, (float4*)out[s], n4);
                         }});
        cases.push_back({"read_only 4B/px  g" + std::to_string(gm), 4.0 * px, [=](int s) {
                             hipLaunchKernelGGL(read_only, dim3(grid), dim3(256), 0, 0, (const uint4*)out[s], n4 / 1,
                                                sink);
                         }});
    }
    for (int gm : {4, 8, 16}) {
        const unsigned grid = cus * gm;
        cases.push_back({"copy_u8 x8 plain g" + std::to_string(gm), 2.0 * px, [=](int s) {
                             hipLaunchKernelGGL((copy_bytes<uint2, false>), dim3(grid), dim3(256), 0, 0,
                                                (const uint2*)in[s], (uint2*)out[s], (uint64_t)px / 8);
                         }});
        cases.push_back({"copy_u8 x8 nt    g" + std::to_string(gm), 2.0 * px, [=](int s) {
                             hipLaunchKernelGGL((copy_bytes<uint2, true>), dim3(grid), dim3(256), 0, 0,
                                                (const uint2*)in[s], (uint2*)out[s], (uint64_t)px / 8);
                         }});
        cases.push_back({"copy_u8 x16 nt   g" + std::to_string(gm), 2.0 * px, [=](int s) {
                             hipLaunchKernelGGL((copy_bytes<uint4, true>), dim3(grid), dim3(256), 0, 0,
                                                (const uint4*)in[s], (uint4*)out[s], (uint64_t)px / 16);
                         }});
    }
    cases.push_back({"hipMemcpyD2D 1B/px (r+w)", 2.0 * px, [=](int s) {
                         CK(hipMemcpyAsync(out[s], in[(s + 1) % nsets], px, hipMemcpyDeviceToDevice, 0));
                     }});
    cases.push_back({"hipMemcpyD2D 4B/px (r+w)", 8.0 * px, [=](int s) {
                         CK(hipMemcpyAsync(out[s], out[(s + 1) % nsets], px * 4, hipMemcpyDeviceToDevice, 0));
                     }});
    if (n % 4096 == 0) {
        cases.push_back({"pat rows8 (headline pattern)", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_rows8<0, 512>), dim3((unsigned)(px / 4096 / 8)), dim3(512), 0, 0,
                                                (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rows8 i8 (int8 pattern)", 2.0 * px, [=](int s) {
                             hipLaunchKernelGGL(pat_rows8_i8, dim3((unsigned)(px / 4096 / 8)), dim3(512), 0, 0,
                                                (const uint8_t*)in[s], (uint8_t*)out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat linear reads + tile writes", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_half<true, false>), dim3((unsigned)(px / 4096 / 8)), dim3(512), 0,
                                                0, (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat tile reads + linear writes", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_half<false, true>), dim3((unsigned)(px / 4096 / 8)), dim3(512), 0,
                                                0, (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat linear reads + linear writes", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_half<true, true>), dim3((unsigned)(px / 4096 / 8)), dim3(512), 0,
                                                0, (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rows8 x2 (two sets per wave)", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(pat_rows8x2, dim3((unsigned)(px / 8192 / 8)), dim3(512), 0, 0,
                                                (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rows8 wg1024", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_rows8<0, 1024>), dim3((unsigned)(px / 4096 / 16)), dim3(1024), 0,
                                                0, (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rows8 wg256", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_rows8<0, 256>), dim3((unsigned)(px / 4096 / 4)), dim3(256), 0,
                                                0, (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rows8 column strips", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL((pat_rows8<1, 512>), dim3((unsigned)(px / 4096 / 8)), dim3(512), 0, 0,
                                                (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"pat rowwave (row per wave)", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(pat_rowwave, dim3((unsigned)(px / 4096 / 8)), dim3(512), 0, 0,
                                                (const uint8_t*)in[s], out[s], (uint32_t)n);
                         }});
        cases.push_back({"mix_run 4096 px/wave nt (pat)", 5.0 * px, [=](int s) {
                             hipLaunchKernelGGL(mix_run<4096>, dim3((unsigned)(px / 4096 / 4)), dim3(256), 0, 0,
                                                (const uint32_t*)in[s], (float4*)out[s], n4);
                         }});
    }
    cases.push_back({"hipMemsetD32 4B/px", 4.0 * px, [=](int s) { CK(hipMemsetD32Async((hipDeviceptr_t)out[s], 7, px, 0)); }});

    if (argc > 3 && strcmp(argv[3], "mix") == 0) {
        std::vector<Case> keep;
        for (auto& c : cases)
            if (c.name.find("mix") != std::string::npos || c.name.find("write") != std::string::npos ||
                c.name.find("Memset") != std::string::npos)
                keep.push_back(c);
        cases.swap(keep);
    }
    if (argc > 3 && strcmp(argv[3], "pat") == 0) {
        std::vector<Case> keep;
        for (auto& c : cases)
            if (c.name.find("pat") != std::string::npos || c.name.find("mix_w4 nt    g8") != std::string::npos ||
                c.name.find("copy_u8 x8 nt    g8") != std::string::npos)
                keep.push_back(c);
        cases.swap(keep);
    }
    if (argc > 3 && strcmp(argv[3], "u8") == 0) {
        std::vector<Case> keep;
        for (auto& c : cases)
            if (c.name.find("copy_u8") != std::string::npos || c.name.find("1B/px") != std::string::npos)
                keep.push_back(c);
        cases.swap(keep);
    }
    if (argc > 3 && strcmp(argv[3], "f32") == 0) {
        std::vector<Case> keep;
        for (auto& c : cases)
            if (c.name.find("copy_f32") != std::string::npos || c.name.find("D2D") != std::string::npos ||
                c.name.find("mix_w4 nt    g4") != std::string::npos)
                keep.push_back(c);
        cases.swap(keep);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(cases.size());
    for (int r = 0; r < 3; ++r)
        for (size_t c = 0; c < cases.size(); ++c) {
            for (int w = 0; w < 3; ++w) cases[c].run(w % nsets);
            for (int i = 3; i < iters + 3; ++i) {  // sets not touched by the warm-up first
                CK(hipEventRecord(a, 0));
                cases[c].run(i % nsets);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                us[c].push_back(ms * 1e3f);
            }
        }
    printf("%-30s %10s %10s %10s %7s\n", "case", "median_us", "min_us", "GB/s", "frac8T");
    for (size_t c = 0; c < cases.size(); ++c) {
        auto t = us[c];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        const double gbs = cases[c].bytes / (med * 1e-6) / 1e9;
        printf("%-30s %10.2f %10.2f %10.1f %7.3f\n", cases[c].name.c_str(), med, t[0], gbs, gbs / 8000.0);
    }
    return 0;
}
