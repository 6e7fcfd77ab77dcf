/*
 * verify_fastdiv.c -- exhaustive proof that the kernel's 3-operation
 * division  q0 = x*r; e = fma(-q0, Q, x); q = fma(e, r, q0)   (r = RN(1/Q))
 * returns exactly the IEEE fp32 quotient RN(x/Q) for EVERY float x with
 * |x| <= XMAX, for each divisor Q given on the command line (default: every
 * integer 1..255, which covers the reference's JPEG table, main_newAppr.cu:60-68).
 * Also reports whether roundf(q) == roundf(x/Q) where q differs.
 * Sign symmetry: every step is odd in x under round-to-nearest, so only
 * x >= 0 is enumerated.  Build: gcc -O3 -march=native -fopenmp -ffp-contract=off
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
    if (argc > 1) { for (int i = 1; i < argc && nq < 512; ++i) qs[nq++] = strtof(argv[i], NULL); }
    else { for (int i = 1; i <= 255; ++i) qs[nq++] = (float)i; }
    long long total_bad = 0, total_round_bad = 0;
    for (int k = 0; k < nq; ++k) {
        const float Q = qs[k];
        const float r = 1.0f / Q;
        long long bad = 0, rbad = 0;
        #pragma omp parallel for reduction(+:bad,rbad) schedule(static)
        for (long long u = 0; u <= (long long)umax; ++u) {
            const float x = f_of((uint32_t)u);
            const float ref = x / Q;
            const float q0 = x * r;
            const float e = fmaf(-q0, Q, x);
            const float q = fmaf(e, r, q0);
            if (q != ref) { bad++; if (roundf(q) != roundf(ref)) rbad++; }
        }
        if (bad) printf("Q=%g: %lld quotient mismatches (%lld change roundf)\n", Q, bad, rbad);
        total_bad += bad; total_round_bad += rbad;
    }
    printf("checked %d divisors x %u floats: %lld quotient mismatches, %lld rounding mismatches\n",
           nq, umax + 1, total_bad, total_round_bad);
    return total_bad ? 1 : 0;
}
