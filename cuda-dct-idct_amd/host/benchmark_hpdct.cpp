// benchmark_hpdct.cpp -- HIP-native counterpart of the reference's
// Benchmark_code/benchmark_newAppr.cu (main, :33-119): same CLI
// (`benchmark_hpdct <width/height>`), same synthetic input (srand(42),
// rand()%256 stored as float, :44-51), same Q/T tables, same call sequence
// (H2D -> dct_all_blocks_cuda -> D2H -> idct_all_blocks_cuda -> D2H) and the
// same stdout lines "DCT (W,H): x ms" / "IDCT (W,H): x ms", printed by the
// library's compat entry points.  An optional second argument repeats the
// whole sequence (image re-uploaded each time, since the forward leaves X-128
// in it) to average warm calls; the first call of a process includes loading
// the kernels' code object.
//
// `benchmark_hpdct <n> [runs] --gpus N [--int8]` is the build's own C4 mode
// (shard_bench.hpp): the n x n frame row-sharded over N GPUs of this process,
// RCCL gather to device 0 (include/hpdct_dist.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpdct_compat.h"

#define CHECK_HIP(call)                                               \
    {                                                                 \
        hipError_t err = call;                                        \
        if (err != hipSuccess) {                                      \
            printf("%s : %d", hipGetErrorString(err), __LINE__);      \
            exit(EXIT_FAILURE);                                       \
        }                                                             \
    }

#include "shard_bench.hpp"

int main(int argc, char* argv[]) {
    // options of the sharded mode, anywhere after the size
    int gpus = 0;
    bool int8 = false;
    int npos = 0;
    char* pos[2] = {NULL, NULL};
    for (int i = 1; i < argc; ++i) {
        if (strcmp(argv[i], "--gpus") == 0 && i + 1 < argc) {
            gpus = atoi(argv[++i]);
        } else if (strcmp(argv[i], "--int8") == 0) {
            int8 = true;
        } else if (npos < 2) {
            pos[npos++] = argv[i];
        } else {
            npos = 3;
        }
    }
    if (npos != 1 && npos != 2) {
        printf("Use: %s <width/height> [runs] [--gpus N [--int8]]\n", argv[0]);
        return 1;
    }
    const size_t n = strtoul(pos[0], NULL, 10);
    const long runs = npos == 2 ? strtol(pos[1], NULL, 10) : 1;
    if (gpus > 0) return run_sharded(n, gpus, int8, runs);
    const size_t width = n, height = n;
    const size_t px = width * height;

    float* image = (float*)malloc(px * sizeof(float));
    srand(42);
    for (size_t i = 0; i < px; ++i) image[i] = (float)(rand() % 256);

    float transform[64];
    hpdct_default_transform(transform);  // the T of benchmark_newAppr.cu:67-75
    // Q: the library's default table is the one of benchmark_newAppr.cu:54-62

    float* result = (float*)malloc(px * sizeof(float));
    float *d_A, *d_B, *d_C, *d_E;
    CHECK_HIP(hipMalloc(&d_A, px * sizeof(float)));
    CHECK_HIP(hipMalloc(&d_B, 64 * sizeof(float)));
    CHECK_HIP(hipMalloc(&d_C, px * sizeof(float)));
    CHECK_HIP(hipMemcpy(d_B, transform, 64 * sizeof(float), hipMemcpyHostToDevice));
    CHECK_HIP(hipMalloc(&d_E, px * sizeof(float)));

    for (long r = 0; r < (runs > 0 ? runs : 1); ++r) {
        CHECK_HIP(hipMemcpy(d_A, image, px * sizeof(float), hipMemcpyHostToDevice));
        dct_all_blocks_cuda(d_A, (int)height, (int)width, d_B, d_C);
        CHECK_HIP(hipMemcpy(result, d_C, px * sizeof(float), hipMemcpyDeviceToHost));
        idct_all_blocks_cuda(d_C, (int)height, (int)width, d_B, d_E);
        CHECK_HIP(hipMemcpy(result, d_E, px * sizeof(float), hipMemcpyDeviceToHost));
    }

    CHECK_HIP(hipFree(d_A));
    CHECK_HIP(hipFree(d_B));
    CHECK_HIP(hipFree(d_C));
    CHECK_HIP(hipFree(d_E));
    free(result);
    free(image);
    return 0;
}
