// mfma_probe.hip -- development probe (not the product): operand layout,
// numerics and issue rate of the f32-input MFMA shapes on gfx950, for a
// matrix-core form of the DCT's exact fp32 FMA chains.
//   1. layout of v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4 blocks, k = 1):
//      every (block, i, j) of D checked against fmaf(A, B, C) under the
//      hypothesis  A: lane 4b+i,  B: lane 4b+j,  D: VGPR i, lane 4b+j;
//   2. exactness: D == fmaf(a, b, c) bit for bit on random, tiny, huge,
//      signed-zero and integer-valued operands (the DCT's operands);
//   3. an 8-step chain D = fma(a7, b7, ... fma(a0, b0, +0)) == the scalar chain;
//   4. issue rate: back-to-back dependent / independent instructions timed with
//      s_memtime inside one wave.
// usage: mfma_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one MFMA per wave: a[64], b[64], c[4][64] -> d[4][64]
__global__ void one_mfma(const float* a, const float* b, const float* c, float* d) {
    const int l = threadIdx.x;
    f32x4 acc = {c[0 * 64 + l], c[1 * 64 + l], c[2 * 64 + l], c[3 * 64 + l]};
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[r * 64 + l] = acc[r];
}

// 8-step chain from +0: a[k*64 + l], b[k*64 + l]
__global__ void chain8(const float* a, const float* b, float* d) {
    const int l = threadIdx.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[k * 64 + l], b[k * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[r * 64 + l] = acc[r];
}

// issue timing: kChains independent accumulators, kIters rounds of dependent MFMAs
template <int kChains>
__global__ void rate(float x, float* out, long long* cyc, int iters) {
    f32x4 acc[kChains];
    for (int c = 0; c < kChains; ++c) acc[c] = f32x4{x, x + 1, x + 2, x + 3};
    const float a = x * 0.5f + threadIdx.x, b = x * 0.25f;
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[c], 0, 0, 0);
    }
    const long long t1 = __builtin_readcyclecounter();
    float s = 0;
    for (int c = 0; c < kChains; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static uint32_t bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static float pick(uint32_t& s, int kind) {
    s = s * 1664525u + 1013904223u;
    const float u = (float)((s >> 8) & 0xffffff) / 16777216.0f;
    switch (kind) {
        case 0: return (u - 0.5f) * 600.0f;                        // DCT-like magnitudes
        case 1: return std::ldexp(u - 0.5f, -130);                  // subnormal range
        case 2: return std::ldexp(u + 0.5f, 100) * (s & 1 ? -1 : 1);  // huge
        case 3: return (s & 2) ? -0.0f : 0.0f;                      // signed zeros
        default: return (float)((int)((s >> 9) & 255) - 128);       // integer pixels - 128
    }
}

int main() {
    float *da, *db, *dc, *dd;
    CK(hipMalloc(&da, 8 * 64 * 4));
    CK(hipMalloc(&db, 8 * 64 * 4));
    CK(hipMalloc(&dc, 4 * 64 * 4));
    CK(hipMalloc(&dd, 4 * 64 * 4));
    std::vector<float> a(8 * 64), b(8 * 64), c(4 * 64), d(4 * 64);
    uint32_t seed = 12345;
    long bad_layout = 0, bad_exact = 0, checked = 0;
    for (int trial = 0; trial < 400; ++trial) {
        const int ka = trial % 5, kb = (trial / 5) % 5, kc = (trial / 25) % 5;
        for (int l = 0; l < 64; ++l) {
            a[l] = pick(seed, ka);
            b[l] = pick(seed, kb);
        }
        for (int i = 0; i < 256; ++i) c[i] = pick(seed, kc);
        CK(hipMemcpy(da, a.data(), 64 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, b.data(), 64 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dc, c.data(), 256 * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(one_mfma, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
        CK(hipMemcpy(d.data(), dd, 256 * 4, hipMemcpyDeviceToHost));
        for (int blk = 0; blk < 16; ++blk)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    const float want = std::fma(a[4 * blk + i], b[4 * blk + j], c[i * 64 + 4 * blk + j]);
                    const float got = d[i * 64 + 4 * blk + j];
                    ++checked;
                    if (bits(want) != bits(got)) {
                        if (std::isnan(want) && std::isnan(got)) continue;
                        // distinguish a layout error (value matches another slot) from rounding
                        if (std::fabs(want - got) > 1e-3f * (std::fabs(want) + 1.0f)) {
                            ++bad_layout;
                        } else {
                            ++bad_exact;
                        }
                        if (bad_layout + bad_exact < 6)
                            printf("mismatch trial %d blk %d i %d j %d: want %a got %a\n", trial, blk, i, j, want,
                                   got);
                    }
                }
    }
    printf("4x4x1_16b layout/exactness: %ld elements, %ld layout mismatches, %ld rounding mismatches\n", checked,
           bad_layout, bad_exact);

    // 8-step chains with integer pixels and T-like constants
    long chain_bad = 0, chain_n = 0;
    for (int trial = 0; trial < 200; ++trial) {
        for (int k = 0; k < 8; ++k)
            for (int l = 0; l < 64; ++l) {
                a[k * 64 + l] = pick(seed, trial % 2 ? 4 : 0);
                b[k * 64 + l] = (float)((int)(pick(seed, 4))) * 0.0027621358f;
            }
        CK(hipMemcpy(da, a.data(), 512 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, b.data(), 512 * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(chain8, dim3(1), dim3(64), 0, 0, da, db, dd);
        CK(hipMemcpy(d.data(), dd, 256 * 4, hipMemcpyDeviceToHost));
        for (int blk = 0; blk < 16; ++blk)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    float s = 0.0f;
                    for (int k = 0; k < 8; ++k) s = std::fma(a[k * 64 + 4 * blk + i], b[k * 64 + 4 * blk + j], s);
                    ++chain_n;
                    if (bits(s) != bits(d[i * 64 + 4 * blk + j])) ++chain_bad;
                }
    }
    printf("8-step chains from +0: %ld elements, %ld mismatches vs the scalar fmaf chain\n", chain_n, chain_bad);

    float* dout;
    long long* dcyc;
    CK(hipMalloc(&dout, 64 * 4));
    CK(hipMalloc(&dcyc, 8));
    const int iters = 4096;
    for (int pass = 0; pass < 2; ++pass) {
        long long cyc[3];
        hipLaunchKernelGGL(rate<1>, dim3(1), dim3(64), 0, 0, 1.0f, dout, dcyc, iters);
        CK(hipMemcpy(&cyc[0], dcyc, 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(rate<4>, dim3(1), dim3(64), 0, 0, 1.0f, dout, dcyc, iters);
        CK(hipMemcpy(&cyc[1], dcyc, 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(rate<8>, dim3(1), dim3(64), 0, 0, 1.0f, dout, dcyc, iters);
        CK(hipMemcpy(&cyc[2], dcyc, 8, hipMemcpyDeviceToHost));
        if (pass)
            printf("4x4x1_16b cycles per instruction (one wave): dependent %.2f, 4 chains %.2f, 8 chains %.2f\n",
                   (double)cyc[0] / iters, (double)cyc[1] / (4.0 * iters), (double)cyc[2] / (8.0 * iters));
    }
    return (bad_layout || bad_exact || chain_bad) ? 1 : 0;
}
