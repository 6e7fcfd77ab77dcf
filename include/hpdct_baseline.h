/*
 * hpdct_baseline.h -- A/B baselines of the reference's own GPU work
 * decompositions (NOT the product path).
 *
 * hpdct_baseline_forward runs, on the given stream, the three launches of
 *   HPDCT_BASELINE_REFERENCE_3PASS  dct_all_blocks_cuda, main_newAppr.cu:252-291
 *                                   (HpApprDCT: one 8x8 workgroup per tile)
 *   HPDCT_BASELINE_FASTAPPR_3PASS   dct_all_blocks_cuda, main_fastAppr.cu:303-359
 *                                   (fastApprDCT: one thread per tile row)
 * with the reference's data types and side effects: fp32 image in HBM,
 * mutated in place to X-128; d_tmp an H*W fp32 scratch plane (the reference
 * allocates it per call); d_result the fp32 quantised coefficients; the
 * caller's device T; the library's quant table.  Same arithmetic as
 * hpdct_forward, so the results are bit-identical to it.
 */
#ifndef HPDCT_BASELINE_H
#define HPDCT_BASELINE_H

#include "hpdct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum hpdct_baseline {
    HPDCT_BASELINE_REFERENCE_3PASS = 0,
    HPDCT_BASELINE_FASTAPPR_3PASS = 1
} hpdct_baseline;

hpdct_status hpdct_baseline_forward(hpdct_baseline kind, float* d_image, float* d_tmp, float* d_result,
                                    int64_t height, int64_t width, const float* d_transform, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HPDCT_BASELINE_H */
