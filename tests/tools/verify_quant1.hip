// verify_quant1.hip -- exhaustive on-device check of two SHORTER quantiser
// forms against the reference's round(C / Q) (utils_kernels.cu:42: IEEE fp32
// division, then roundf = round half away from zero).  For every integer
// divisor Q in 1..255 and EVERY fp32 x with 0 <= x <= XMAX (the forms are odd
// in x), with r = RN(1/Q) and b = copysign(0.49999997f, x):
//   F  trunc(fma(x, r, b))            one rounding of x*r + b (3 VALU with the
//                                     copysign; the int8 output folds the
//                                     trunc into its truncating convert)
//   M  trunc(RN(x * r) + b)           the 1-op quotient, then the verified
//                                     3-op roundf (4 VALU)
// against the product's 6-op form (3-op quotient, exact by verify_fastdiv).
// Prints, per divisor, the mismatch count of each form and its smallest
// mismatching x (a form is exact for that divisor on |x| below it), and a final line
// "exact divisors F: <bitmask hex>" (bit q-1 set when F is exact for Q = q):
// the table the library uses to enable F (csrc/hpdct_quant_tables.h).
//   usage: verify_quant1 [xmax=4096]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__device__ __forceinline__ float rha(float x) { return __builtin_truncf(x + __builtin_copysignf(0.49999997f, x)); }

__global__ void check(uint32_t umax, unsigned long long* badf, unsigned long long* badm, uint32_t* minf,
                      uint32_t* minm) {
    const float Q = (float)(blockIdx.y + 1);
    const float r = 1.0f / Q;
    unsigned long long nf = 0, nm = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u <= umax; u += stride) {
        const float x = __uint_as_float(u);
        const float ref = rha(x / Q);
        const float b = __builtin_copysignf(0.49999997f, x);
        const float f = __builtin_truncf(__builtin_fmaf(x, r, b));
        const float m = __builtin_truncf(x * r + b);
        const bool bf = __float_as_uint(f) != __float_as_uint(ref), bm = __float_as_uint(m) != __float_as_uint(ref);
        nf += bf;
        nm += bm;
        if (bf) atomicMin(&minf[blockIdx.y], u);  // positive floats order like their bit patterns
        if (bm) atomicMin(&minm[blockIdx.y], u);
        if (u > umax - stride) break;  // avoid u wrap-around
    }
    if (nf) atomicAdd(&badf[blockIdx.y], nf);
    if (nm) atomicAdd(&badm[blockIdx.y], nm);
}

int main(int argc, char** argv) {
    const float xmax = argc > 1 ? strtof(argv[1], nullptr) : 4096.0f;
    uint32_t umax;
    memcpy(&umax, &xmax, 4);
    unsigned long long *bf, *bm;
    uint32_t *mf, *mm;
    if (hipMalloc(&bf, 255 * 8) || hipMalloc(&bm, 255 * 8) || hipMalloc(&mf, 255 * 4) || hipMalloc(&mm, 255 * 4))
        return 2;
    (void)hipMemset(bf, 0, 255 * 8);
    (void)hipMemset(bm, 0, 255 * 8);
    (void)hipMemset(mf, 0xff, 255 * 4);
    (void)hipMemset(mm, 0xff, 255 * 4);
    hipLaunchKernelGGL(check, dim3(4096, 255), dim3(256), 0, 0, umax, bf, bm, mf, mm);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long hf[255], hm[255];
    uint32_t hmf[255], hmm[255];
    (void)hipMemcpy(hf, bf, sizeof(hf), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hm, bm, sizeof(hm), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hmf, mf, sizeof(hmf), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hmm, mm, sizeof(hmm), hipMemcpyDeviceToHost);
    auto fl = [](uint32_t u) {
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    uint64_t mask[4] = {0, 0, 0, 0};
    int exact_f = 0, exact_m = 0;
    for (int q = 1; q <= 255; ++q) {
        if (hf[q - 1] || hm[q - 1])
            printf("Q=%3d: F %llu mismatches (smallest x %.9g), M %llu mismatches (smallest x %.9g)\n", q, hf[q - 1],
                   hf[q - 1] ? fl(hmf[q - 1]) : 0.0f, hm[q - 1], hm[q - 1] ? fl(hmm[q - 1]) : 0.0f);
        if (!hf[q - 1]) {
            mask[(q - 1) / 64] |= 1ull << ((q - 1) % 64);
            ++exact_f;
        }
        exact_m += !hm[q - 1];
    }
    printf("xmax %g (%u values per divisor): F exact for %d of 255 divisors, M exact for %d\n", xmax, umax + 1,
           exact_f, exact_m);
    printf("exact divisors F: 0x%016llx 0x%016llx 0x%016llx 0x%016llx\n", (unsigned long long)mask[0],
           (unsigned long long)mask[1], (unsigned long long)mask[2], (unsigned long long)mask[3]);
    return 0;
}
