// hpdct_baselines.hip -- A/B baselines, NOT the
// product path: the reference's two GPU work decompositions of the same
// arithmetic, written for gfx950, so the README's comparison (HpApprDCT vs
// fastApprDCT vs CPU, README.md:46-60) can be re-measured on MI355X beside the
// fused kernel.  Same fp32 FMA order, IEEE division and roundf as the oracle,
// so their outputs are bit-identical to the product's.
//
//   HPDCT_BASELINE_REFERENCE_3PASS  main_newAppr.cu:252-291: three launches
//     (X-=128 in place; one 64-thread workgroup per tile with T, the tile and
//     P staged in LDS and a barrier between the passes; round(C/Q)), each
//     launch a (W/8) x (H/8) grid of 8x8 workgroups.
//   HPDCT_BASELINE_FASTAPPR_3PASS   main_fastAppr.cu:303-359: the same three
//     launches, but the middle one gives each thread one tile ROW (8 tiles per
//     64-thread workgroup, T and the 8 tiles in LDS, the thread's P row in
//     registers).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hpdct_baseline.h"
#include "hpdct_kernels.h"

namespace {

struct Q64 {
    float v[64];
};

// element index of thread (tx, ty) of workgroup (bx, by) in a W-wide image
__device__ __forceinline__ uint64_t pix(uint32_t w) {
    return (static_cast<uint64_t>(blockIdx.y) * 8u + threadIdx.y) * w + blockIdx.x * 8u + threadIdx.x;
}

__global__ __launch_bounds__(64) void shift_kernel(float* __restrict__ img, uint32_t w, float delta) {
    const uint64_t i = pix(w);
    img[i] = img[i] + delta;
}

__global__ __launch_bounds__(64) void quant_kernel(const float* __restrict__ c, float* __restrict__ out, uint32_t w,
                                                   Q64 q) {
    const uint64_t i = pix(w);
    out[i] = __builtin_roundf(c[i] / q.v[threadIdx.y * 8 + threadIdx.x]);
}

// one 64-thread workgroup per tile: thread (x = tx, v = ty)
__global__ __launch_bounds__(64) void tile_dct_kernel(const float* __restrict__ img, const float* __restrict__ t,
                                                      float* __restrict__ out, uint32_t w) {
    __shared__ float st[64], sx[64], sp[64];
    const uint32_t tx = threadIdx.x, ty = threadIdx.y;
    const uint64_t i = pix(w);
    st[ty * 8 + tx] = t[ty * 8 + tx];
    sx[ty * 8 + tx] = img[i];
    __syncthreads();
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s = __builtin_fmaf(st[ty * 8 + k], sx[k * 8 + tx], s);  // P = T.X
    sp[ty * 8 + tx] = s;
    __syncthreads();
    s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s = __builtin_fmaf(sp[ty * 8 + k], st[tx * 8 + k], s);  // C = P.T^T
    out[i] = s;
}

// one thread per tile row: workgroup = 8 tiles (ty) x 8 rows (tx), 1-D grid
__global__ __launch_bounds__(64) void row_dct_kernel(const float* __restrict__ img, const float* __restrict__ t,
                                                     float* __restrict__ out, uint32_t w, uint32_t ntiles,
                                                     uint32_t tiles_x) {
    __shared__ float st[64];
    __shared__ float tiles[8][64];
    const uint32_t r = threadIdx.x, k = threadIdx.y;
    st[k * 8 + r] = t[k * 8 + r];
    const uint32_t tile = blockIdx.x * 8u + k;
    const bool live = tile < ntiles;
    uint64_t base = 0;
    if (live) {
        const uint32_t by = tile / tiles_x, bx = tile - by * tiles_x;
        base = static_cast<uint64_t>(by) * 8u * w + bx * 8u;
#pragma unroll
        for (int c = 0; c < 8; ++c) tiles[k][r * 8 + c] = img[base + static_cast<uint64_t>(r) * w + c];
    }
    __syncthreads();
    if (!live) return;
    float prow[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // P[r][c] = sum_j T[r][j] X[j][c]
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = __builtin_fmaf(st[r * 8 + j], tiles[k][j * 8 + c], s);
        prow[c] = s;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // C[r][u] = sum_j P[r][j] T[u][j]
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = __builtin_fmaf(prow[j], st[u * 8 + j], s);
        out[base + static_cast<uint64_t>(r) * w + u] = s;
    }
}

}  // namespace

extern "C" hpdct_status hpdct_baseline_forward(hpdct_baseline kind, float* d_image, float* d_tmp, float* d_result,
                                               int64_t height, int64_t width, const float* d_transform,
                                               void* stream) {
    if (!d_image || !d_tmp || !d_result || !d_transform) return HPDCT_ERROR_INVALID_VALUE;
    if (height <= 0 || width <= 0 || height % 8 || width % 8 || width / 8 >= (int64_t(1) << 31) || height / 8 > 65535)
        return HPDCT_ERROR_INVALID_VALUE;
    if (kind != HPDCT_BASELINE_REFERENCE_3PASS && kind != HPDCT_BASELINE_FASTAPPR_3PASS)
        return HPDCT_ERROR_UNSUPPORTED;
    const uint32_t w = static_cast<uint32_t>(width);
    const dim3 grid(static_cast<uint32_t>(width / 8), static_cast<uint32_t>(height / 8)), block(8, 8);
    hipStream_t s = static_cast<hipStream_t>(stream);
    float qv[64];
    if (hpdct_get_quant_table(qv) != HPDCT_SUCCESS) return HPDCT_ERROR_INVALID_VALUE;
    Q64 q;
    for (int i = 0; i < 64; ++i) q.v[i] = qv[i];
    hipLaunchKernelGGL(shift_kernel, grid, block, 0, s, d_image, w, -128.0f);
    if (kind == HPDCT_BASELINE_REFERENCE_3PASS) {
        hipLaunchKernelGGL(tile_dct_kernel, grid, block, 0, s, d_image, d_transform, d_tmp, w);
    } else {
        const uint32_t tiles_x = w / 8, ntiles = static_cast<uint32_t>(height / 8) * tiles_x;
        hipLaunchKernelGGL(row_dct_kernel, dim3((ntiles + 7) / 8), block, 0, s, d_image, d_transform, d_tmp, w,
                           ntiles, tiles_x);
    }
    hipLaunchKernelGGL(quant_kernel, grid, block, 0, s, d_tmp, d_result, w, q);
    return hipGetLastError() == hipSuccess ? HPDCT_SUCCESS : HPDCT_ERROR_DEVICE;
}
