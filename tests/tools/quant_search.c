/* quant_search.c -- search for more 3-operation quantiser forms for the
 * DEFAULT JPEG table (the positions where F and H of verify_quant_pos.c are
 * not exact).  The form is the same shape,
 *     trunc(fma(x, r', copysign(b, x)))
 * but with a per-position reciprocal r' near RN(1/Q) (RN(1/Q) + k ulps,
 * |k| <= KR) and a per-position bias b near 0.5 (b = 0.5 - j 2^-25 for
 * j = 0..JB, or 0.5 + j 2^-24 for j = 1..JB).  A (r', b) pair is exact at a
 * position when it gives roundf(x / Q) (IEEE division, then round half away)
 * for EVERY fp32 x in [Q/4, bound] (odd forms; below Q/4 all give 0), the
 * same exhaustive check as verify_quant_pos.c.  Development tool: prints, per
 * position, the first exact (k, j) found and the table of results.
 *
 * Build: gcc -O2 -mfma -ffp-contract=off -fno-fast-math -fopenmp quant_search.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define TA ((float)0.35355339)
#define TH ((float)0.5)
#define TB ((float)0.4472136)
#define TC ((float)0.2236068)
#define TD ((float)0.70710678)
static const float kT[64] = {
    TA, TA,  TA,  TA,  TA,  TA,  TA,  TA,  TH, TH,  0,  0,   0,   0,   -TH, -TH, TB, TC,  -TC, -TB, -TB, -TC,
    TC, TB,  0,   0,   -TD, 0,   0,   TD,  0,  0,   TA, -TA, -TA, TA,  TA,  -TA, -TA, TA, TH, -TH, 0,   0,
    0,  0,   TH,  -TH, TC,  -TB, TB,  -TC, -TC, TB, -TB, TC, 0,  0,   0,   -TD, TD,  0,   0,   0};
static const float kQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                             14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                             18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const uint64_t kF = 0x43169a554274082dull, kH = 0xa8894480a800a000ull;

#define KR 3
#define JB 24

static float fbits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t ubits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static double position_bound(int v, int u) {
    double nv = 0, nu = 0;
    for (int i = 0; i < 8; ++i) nv += fabs((double)kT[v * 8 + i]), nu += fabs((double)kT[u * 8 + i]);
    return 128.0 * nv * nu * (1.0 + ldexp(1.0, -16));
}
/* 1 when trunc(fma(x, r, +-b)) == roundf(x / Q) for every x in [Q/4, bound] */
static int exact(float Q, double bound, float r, float b) {
    const uint32_t u0 = ubits(Q / 4.0f), u1 = ubits((float)bound) + 1u;
    for (uint32_t u = u0; u <= u1; ++u) {
        const float x = fbits(u);
        if (ubits(truncf(__builtin_fmaf(x, r, b))) != ubits(roundf(x / Q))) return 0;
    }
    return 1;
}

int main(void) {
    int found_k[64], found_j[64];
    float found_r[64], found_b[64];
#pragma omp parallel for schedule(dynamic)
    for (int p = 0; p < 64; ++p) {
        found_k[p] = found_j[p] = 999;
        if (((kF | kH) >> p) & 1u) continue;
        const float Q = kQ[p], r0 = 1.0f / Q;
        const double bound = position_bound(p / 8, p % 8);
        for (int k = 0; k <= KR && found_k[p] == 999; ++k)
            for (int sk = (k ? -1 : 1); sk <= 1 && found_k[p] == 999; sk += 2) {
                const float r = fbits(ubits(r0) + sk * k);
                for (int j = -JB; j <= JB && found_k[p] == 999; ++j) {
                    const float b = j <= 0 ? 0.5f + ldexpf((float)j, -25) : 0.5f + ldexpf((float)j, -24);
                    if (exact(Q, bound, r, b)) {
                        found_k[p] = sk * k, found_j[p] = j, found_r[p] = r, found_b[p] = b;
                    }
                }
            }
    }
    int n = 0;
    uint64_t mask = 0;
    for (int p = 0; p < 64; ++p) {
        if (((kF | kH) >> p) & 1u) continue;
        if (found_k[p] != 999) {
            ++n, mask |= 1ull << p;
            printf("pos %2d (v %d u %d, Q %3.0f): r = RN(1/Q) %+d ulp = %.9g (0x%08x), bias %.9g (0x%08x)\n", p, p / 8,
                   p % 8, kQ[p], found_k[p], found_r[p], ubits(found_r[p]), found_b[p], ubits(found_b[p]));
        } else {
            printf("pos %2d (v %d u %d, Q %3.0f): none within %d ulp of r and %d bias steps\n", p, p / 8, p % 8, kQ[p],
                   KR, JB);
        }
    }
    printf("new 3-op positions: %d of %d; mask 0x%016llx\n", n, 64 - __builtin_popcountll(kF | kH),
           (unsigned long long)mask);
    return 0;
}
