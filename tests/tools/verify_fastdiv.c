/*
 * verify_fastdiv.c -- exhaustive proof that the kernel's 3-operation
 * division  q0 = x*r; e = fma(-q0, Q, x); q = fma(e, r, q0)   (r = RN(1/Q))
 * returns exactly the IEEE fp32 quotient RN(x/Q) for EVERY float x with
 * |x| <= XMAX, for each divisor Q given on the command line (default: every
 * integer 1..255, which covers the reference's JPEG table, main_newAppr.cu:60-68).
 * Also reports whether roundf(q) == roundf(x/Q) where q differs.
 * Sign symmetry: every step is odd in x under round-to-nearest, so only
 * x >= 0 is enumerated.  Build: gcc -O3 -march=native -fopenmp -ffp-contract=off
 * Usage: verify_fastdiv [--stride S] [Q ...]   (--stride S checks every S-th
 * bit pattern: the sampled mode of tests/test_tools.py; default exhaustive)
 * Exhaustive CPU result for the 47 JPEG divisors: verify_fastdiv.cpu.log.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
    const float XMAX = 4096.0f;
    uint32_t umax; memcpy(&umax, &XMAX, 4);
    int nq = 0; float qs[512];
    long long stride = 1;
    int a0 = 1;
    if (argc > 2 && strcmp(argv[1], "--stride") == 0) { stride = atoll(argv[2]); a0 = 3; }
    if (argc > a0) { for (int i = a0; i < argc && nq < 512; ++i) qs[nq++] = strtof(argv[i], NULL); }
    else { for (int i = 1; i <= 255; ++i) qs[nq++] = (float)i; }
    long long total_bad = 0, total_round_bad = 0;
    for (int k = 0; k < nq; ++k) {
        const float Q = qs[k];
        const float r = 1.0f / Q;
        long long bad = 0, rbad = 0;
        #pragma omp parallel for reduction(+:bad,rbad) schedule(static)
        for (long long u = 0; u <= (long long)umax; u += stride) {
            const float x = f_of((uint32_t)u);
            const float ref = x / Q;
            const float q0 = x * r;
            const float e = fmaf(-q0, Q, x);
            const float q = fmaf(e, r, q0);
            if (q != ref) {
                bad++;
                const float a = roundf(q), b = roundf(ref);
                uint32_t ab, bb;
                memcpy(&ab, &a, 4);
                memcpy(&bb, &b, 4);
                if (ab != bb) rbad++;
            }
        }
        if (bad) printf("Q=%g: %lld quotient mismatches (%lld change roundf)\n", Q, bad, rbad);
        total_bad += bad; total_round_bad += rbad;
    }
    printf("checked %d divisors x %llu floats: %lld quotient mismatches, %lld rounding mismatches\n",
           nq, ((long long)umax + stride) / stride, total_bad, total_round_bad);
    return total_round_bad ? 1 : 0;
}
