// hpdct_compat.cpp -- the reference's C++ call surface (include/hpdct_compat.h)
// on top of the native C-ABI.  Behaviour follows dct_all_blocks_cuda /
// idct_all_blocks_cuda (main_newAppr.cu:252-332): device pointers owned by
// the caller, caller's T, null stream, synchronous, one timing line on
// stdout, print-and-exit on any runtime error (CHECK_CUDA, :9-17).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "hpdct_compat.h"

namespace {

// CHECK_CUDA equivalent (main_newAppr.cu:9-17): "<msg> : <line>", exit.
#define HPDCT_CHECK_HIP(call)                                        \
    do {                                                             \
        hipError_t err_ = (call);                                    \
        if (err_ != hipSuccess) {                                    \
            printf("%s : %d", hipGetErrorString(err_), __LINE__);    \
            exit(EXIT_FAILURE);                                      \
        }                                                            \
    } while (0)

void check_status(hpdct_status st, int line) {
    if (st == HPDCT_SUCCESS) return;
    printf("%s : %d", hpdct_last_error_string(), line);
    exit(EXIT_FAILURE);
}

bool quiet() {
    const char* q = getenv("HPDCT_COMPAT_QUIET");
    return q && q[0] && q[0] != '0';
}

void check_shape(int img_height, int img_width) {
    if (img_height <= 0 || img_width <= 0 || (img_height % 8) || (img_width % 8)) {
        printf("image size (%d,%d) is not a positive multiple of 8 : %d", img_width, img_height, __LINE__);
        exit(EXIT_FAILURE);
    }
}

template <typename Launch>
void timed(const char* tag, int img_width, int img_height, Launch&& launch) {
    hipEvent_t start, stop;
    HPDCT_CHECK_HIP(hipEventCreate(&start));
    HPDCT_CHECK_HIP(hipEventCreate(&stop));
    HPDCT_CHECK_HIP(hipEventRecord(start, nullptr));
    launch();
    HPDCT_CHECK_HIP(hipEventRecord(stop, nullptr));
    HPDCT_CHECK_HIP(hipEventSynchronize(stop));
    float ms = 0.0f;
    HPDCT_CHECK_HIP(hipEventElapsedTime(&ms, start, stop));
    if (!quiet()) printf("%s (%d,%d): %f ms\n", tag, img_width, img_height, ms);
    HPDCT_CHECK_HIP(hipEventDestroy(start));
    HPDCT_CHECK_HIP(hipEventDestroy(stop));
}

}  // namespace

// main_newAppr.cu:252-291.  Leaves X-128 in image_matrix like the reference's
// in-place sub_matrix_scalar (:273); result = round((T.(X-128).T^T) / Q).
void dct_all_blocks_cuda(float* image_matrix, const int img_height, const int img_width,
                         const float* transform_matrix, float* result) {
    check_shape(img_height, img_width);
    timed("DCT", img_width, img_height, [&] {
        check_status(hpdct_forward(image_matrix, HPDCT_F32, result, HPDCT_F32, img_height, img_width,
                                   transform_matrix, HPDCT_FLAG_WRITEBACK_SHIFT, nullptr),
                     __LINE__);
    });
}

// main_newAppr.cu:293-332.  result = T^T.(q*Q).T + 128, image_matrix untouched.
void idct_all_blocks_cuda(const float* image_matrix, const int img_height, const int img_width,
                          const float* transform_matrix, float* result) {
    check_shape(img_height, img_width);
    timed("IDCT", img_width, img_height, [&] {
        check_status(hpdct_inverse(image_matrix, HPDCT_F32, result, HPDCT_F32, img_height, img_width,
                                   transform_matrix, 0u, nullptr),
                     __LINE__);
    });
}

// cublasDCTv2 surface (main_cublass_2.cu:197-252): row pass first, X-128 left
// in image_matrix, result = round((T.(X-128).T^T)/Q).  The handle is unused.
void dct_all_blocks(float* image_matrix, const int img_height, const int img_width, const float* transform_matrix,
                    float* result, cublasContext* /*handle*/) {
    check_shape(img_height, img_width);
    timed("DCT", img_width, img_height, [&] {
        check_status(hpdct_forward(image_matrix, HPDCT_F32, result, HPDCT_F32, img_height, img_width,
                                   transform_matrix, HPDCT_FLAG_WRITEBACK_SHIFT | HPDCT_FLAG_ROW_FIRST, nullptr),
                     __LINE__);
    });
}

// main_cublass_2.cu:257-311: q*Q left in image_matrix (in-place
// multiply_matrices, :285), result = T^T.(q*Q).T + 128 with D.T computed first.
void idct_all_blocks(float* image_matrix, const int img_height, const int img_width, const float* transform_matrix,
                     float* result, cublasContext* /*handle*/) {
    check_shape(img_height, img_width);
    timed("IDCT", img_width, img_height, [&] {
        check_status(hpdct_inverse(image_matrix, HPDCT_F32, result, HPDCT_F32, img_height, img_width,
                                   transform_matrix, HPDCT_FLAG_ROW_FIRST | HPDCT_FLAG_WRITEBACK_DEQUANT, nullptr),
                     __LINE__);
    });
}
