/*
 * hpdct_compat.h -- the reference's own call surface, served by libhpdct.so.
 *
 * C++ linkage on purpose: these are the exact symbols the reference's drivers
 * bind (checked with g++ name mangling):
 *   _Z19dct_all_blocks_cudaPfiiPKfS_     dct_all_blocks_cuda
 *   _Z20idct_all_blocks_cudaPKfiiS0_Pf   idct_all_blocks_cuda
 *   _Z14dct_all_blocksPfiiPKfS_P13cublasContext    dct_all_blocks   (cublasDCTv2)
 *   _Z15idct_all_blocksPfiiPKfS_P13cublasContext   idct_all_blocks  (cublasDCTv2)
 *
 * Semantics kept from the reference (main_newAppr.cu:252-332):
 *   - all four pointers are DEVICE pointers owned by the caller; T is the
 *     caller's 64-float transform (d_B in main_newAppr.cu:88-95);
 *   - parameter order (image, HEIGHT, WIDTH, T, result);
 *   - the forward pass leaves X-128 in image_matrix (in-place
 *     sub_matrix_scalar, main_newAppr.cu:273);
 *   - legacy null stream, synchronous on return, prints
 *     "DCT (W,H): x ms" / "IDCT (W,H): x ms" (main_newAppr.cu:287,328);
 *   - a HIP error prints "<msg> : <line>" and exits with EXIT_FAILURE
 *     (CHECK_CUDA, main_newAppr.cu:9-17).
 * Deliberate differences:
 *   - Q is library-owned: hpdct_set_quant_table() replaces the caller-TU
 *     `__constant__ const_quant_matrix` + cudaMemcpyToSymbol
 *     (main_newAppr.cu:19,70); the default is the same JPEG table;
 *   - W or H not a positive multiple of 8 is rejected with a message and
 *     EXIT_FAILURE instead of silently computing garbage;
 *   - one fused kernel per call, no per-call device allocation.
 * Set HPDCT_COMPAT_QUIET=1 in the environment to suppress the timing line.
 *
 * cublasDCTv2 surface (main_cublass_2.cu:36-37,197-311): same conventions,
 * plus its pass order (row pass X.T^T first, inverse D.T first) and its
 * in-place effects (X-128 left in the image, q*Q left in the coefficient
 * buffer).  The cuBLAS handle is accepted and never dereferenced: the
 * arithmetic runs in the library's own kernel.  Its summation order inside
 * cuBLAS is not knowable here, so parity with a cuBLAS build is
 * tolerance-only.  `struct cublasContext` is only the opaque tag
 * cuBLAS's cublasHandle_t points to; it is named here so the mangled symbols
 * match the reference's callers, nothing of cuBLAS is declared or used.
 */
#ifndef HPDCT_COMPAT_H
#define HPDCT_COMPAT_H

#include "hpdct.h"

#ifdef __cplusplus
struct cublasContext;  // opaque handle tag (never dereferenced)

void dct_all_blocks_cuda(float* image_matrix, const int img_height, const int img_width,
                         const float* transform_matrix, float* result);
void idct_all_blocks_cuda(const float* image_matrix, const int img_height, const int img_width,
                          const float* transform_matrix, float* result);
void dct_all_blocks(float* image_matrix, int img_height, int img_width, const float* transform_matrix, float* result,
                    cublasContext* handle);
void idct_all_blocks(float* image_matrix, int img_height, int img_width, const float* transform_matrix, float* result,
                     cublasContext* handle);
#endif

#endif /* HPDCT_COMPAT_H */
