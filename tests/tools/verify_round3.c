/*
 * verify_round3.c -- exhaustive check, over all 2^32 fp32 bit patterns, that
 *     truncf(x + copysignf(0.49999997f, x))      (0.49999997f = 0x3EFFFFFF)
 * is bit-identical to roundf(x) (round half away from zero, the reference's
 * divide_matrices, utils_kernels.cu:42).  NaN inputs only need to stay NaN.
 * Build: gcc -O2 -ffp-contract=off verify_round3.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    const float c = 0.49999997f;
    uint32_t cb;
    memcpy(&cb, &c, 4);
    if (cb != 0x3EFFFFFFu) { printf("constant bits %08x\n", cb); return 2; }
    unsigned long long bad = 0, n = 0;
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; ++u) {
        uint32_t b = (uint32_t)u;
        float x;
        memcpy(&x, &b, 4);
        const float r = roundf(x);
        const float y = truncf(x + copysignf(c, x));
        uint32_t rb, yb;
        memcpy(&rb, &r, 4);
        memcpy(&yb, &y, 4);
        if (isnan(x)) { if (!isnan(y)) ++bad; }
        else if (rb != yb) { if (bad < 10) printf("x=%a round=%a got=%a\n", x, r, y); ++bad; }
        ++n;
    }
    printf("checked %llu patterns: %llu mismatches\n", n, bad);
    return bad != 0;
}
