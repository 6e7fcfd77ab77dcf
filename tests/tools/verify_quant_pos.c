/* verify_quant_pos.c -- per-position proof of the shorter quantiser forms for
 * the DEFAULT JPEG table with uint8 input and the built-in T (the only case
 * the library uses them in; csrc/hpdct_quant_forms.h).
 *
 * The reference quantises with round(C / Q) (utils_kernels.cu:42: IEEE fp32
 * division, then roundf = round half away from zero).  With uint8 pixels
 * X' = X - 128 lies in [-128, 127], so the coefficient at (v, u) is bounded by
 *     |C[v][u]| <= 128 * ||T_v||_1 * ||T_u||_1 * (1 + 2^-16)
 * (the factor covers the fp32 rounding of the two 8-term FMA chains, whose
 * relative growth is below 16 * 2^-24).  For every position this program
 * checks, over EVERY fp32 x in [Q/4, bound] (the forms are odd in x; below
 * Q/4 all of them and the reference give 0, since x*r + 0.49999997 < 0.75),
 * with r = RN(1/Q):
 *   F  trunc(fma(x, r, copysign(0.49999997f, x)))   3 VALU (fp32 out; int8
 *                                                    folds the trunc)
 *   H  trunc(fma(x, r, copysign(0.5f, x)))           3 VALU, another bias
 *   M  trunc(RN(x * r) + copysign(0.49999997f, x))   4 VALU (reported only:
 *                                                    H covers every position
 *                                                    M does)
 * against roundf(x / Q), and prints the table of exact forms.  The library
 * takes F where it is exact, else H, else the verified 6-op form (3-op
 * quotient, exact for |C| <= 4096 and every integer Q: verify_fastdiv, then
 * the 3-op roundf).
 *
 *   verify_quant_pos           table + per-position smallest failing x
 *   verify_quant_pos --masks   only the masks line
 * Build: gcc -O2 -mfma -ffp-contract=off -fno-fast-math -fopenmp (tests/test_quant_forms.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

/* T and Q exactly as csrc/hpdct_tables.h (main_newAppr.cu:60-81): (float)(double)literal */
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

double position_bound(int v, int u) {
    double nv = 0, nu = 0;
    for (int i = 0; i < 8; ++i) {
        nv += fabs((double)kT[v * 8 + i]);
        nu += fabs((double)kT[u * 8 + i]);
    }
    return 128.0 * nv * nu * (1.0 + ldexp(1.0, -16));
}

/* smallest x in [Q/4, bound] where the form differs from the reference, or 0 */
static float first_fail(float Q, double bound, int form) {
    const float r = 1.0f / Q;
    const uint32_t u0 = ubits(Q / 4.0f), u1 = ubits((float)bound) + 1u;
    for (uint32_t u = u0; u <= u1; ++u) {
        const float x = fbits(u);
        const float ref = roundf(x / Q);
        const float b = copysignf(0.49999997f, x);
        float got;
        if (form == 0) {
            got = truncf(__builtin_fmaf(x, r, b));
        } else if (form == 2) {
            got = truncf(__builtin_fmaf(x, r, copysignf(0.5f, x)));
        } else {
            volatile float p = x * r; /* one rounding, not fused (-ffp-contract=off as well) */
            got = truncf(p + b);
        }
        if (ubits(got) != ubits(ref)) return x;
    }
    return 0.0f;
}

int main(int argc, char** argv) {
    const int masks_only = argc > 1 && strcmp(argv[1], "--masks") == 0;
    uint64_t fok = 0, hok = 0, mok = 0;
    float ff[64], fh[64], fm[64];
#pragma omp parallel for schedule(dynamic)
    for (int p = 0; p < 64; ++p) {
        const double b = position_bound(p / 8, p % 8);
        ff[p] = first_fail(kQ[p], b, 0);
        fh[p] = first_fail(kQ[p], b, 2);
        fm[p] = first_fail(kQ[p], b, 1);
    }
    for (int p = 0; p < 64; ++p) {
        if (ff[p] == 0.0f) fok |= 1ull << p;
        if (fh[p] == 0.0f) hok |= 1ull << p;
        if (fm[p] == 0.0f) mok |= 1ull << p;
    }
    const uint64_t use_h = hok & ~fok; /* the library's choice: F first, then H */
    if (!masks_only) {
        printf("pos  v u    Q   bound     F (first fail)      H (first fail)      M (first fail)\n");
        for (int p = 0; p < 64; ++p)
            printf("%3d  %d %d  %3.0f  %7.2f   %-3s %-14.9g   %-3s %-14.9g   %-3s %-14.9g\n", p, p / 8, p % 8, kQ[p],
                   position_bound(p / 8, p % 8), ff[p] == 0.0f ? "ok" : "no", ff[p], fh[p] == 0.0f ? "ok" : "no",
                   fh[p], fm[p] == 0.0f ? "ok" : "no", fm[p]);
        printf("F exact at %d positions, H at %d, M at %d; F or H at %d of 64; M-only positions: %d\n",
               __builtin_popcountll(fok), __builtin_popcountll(hok), __builtin_popcountll(mok),
               __builtin_popcountll(fok | hok), __builtin_popcountll(mok & ~(fok | hok)));
    }
    printf("masks F 0x%016llx H 0x%016llx\n", (unsigned long long)fok, (unsigned long long)use_h);
    return 0;
}
