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

/* Measurement floors and ceilings (bench.py only; no reference counterpart,
 * never called by the product path).
 *
 * hpdct_floor_probe: the floors of the uint8 -> fp32 forward of a height x
 * width frame (bench.py's C2 leg).  HPDCT_PROBE_EMPTY launches an empty kernel
 * on the grid and workgroup size that forward uses (d_in, d_out unused, may be
 * NULL), HPDCT_PROBE_COPY the same grid copying the frame's bytes:
 * d_out[i] = (float)d_in[i], 1 B read + 4 B non-temporal write per pixel and
 * no transform.  Device pointers d_in 8-byte, d_out 16-byte aligned. */
typedef enum hpdct_probe_kind { HPDCT_PROBE_EMPTY = 0, HPDCT_PROBE_COPY = 1 } hpdct_probe_kind;
hpdct_status hpdct_floor_probe(hpdct_probe_kind kind, const uint8_t* d_in, float* d_out, int64_t height,
                               int64_t width, void* stream);

/* hpdct_copy_ceiling: the memory ceiling of a streaming kernel over n pixels,
 * the bytes of the kernel it stands beside and no arithmetic: every pixel
 * reads one in_type element of d_in and writes one out0_type element to
 * d_out0 and, when d_out1 is not NULL, one out1_type element to d_out1
 * (HPDCT_U8 / HPDCT_I8: 1 B, HPDCT_F32: 4 B; values converted, non-temporal
 * stores).  Access widths follow the path's kernels: a lane moves 4 pixels per
 * instruction when any plane is fp32 (1 KiB contiguous per fp32 instruction),
 * 8 pixels (8 B) when every plane is 1 B.  One-wave workgroups of 2,048
 * pixels each; cap_waves > 0 reserves LDS so that at most that many are
 * resident per CU (0: the hardware's limit).  n a positive multiple of 2048;
 * d_in and the outputs 16-byte aligned; d_out1 may be d_in (an in-place
 * write-back, as the drop-in kernels' X-128 and q*Q planes); async on
 * `stream`.  bench.py times it over each kernel's own planes at a few caps
 * and reports the fastest as that kernel's ceiling. */
hpdct_status hpdct_copy_ceiling(const void* d_in, hpdct_dtype in_type, void* d_out0, hpdct_dtype out0_type,
                                void* d_out1, hpdct_dtype out1_type, int64_t n, int cap_waves, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HPDCT_BASELINE_H */
