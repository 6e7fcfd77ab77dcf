// main_hpdct.cpp -- HIP-native counterpart of the reference's interactive
// driver main_newAppr.cu (main, :26-168): `main_hpdct <input> <output>`.
// Loads a grayscale image (PGM, or JPEG when built with libjpeg), prints the
// top-left 8x8 of the input, of the quantised DCT and of the IDCT, converts
// back to uint8 (clamp + truncate, utils.cu:18-24) and writes the result
// (JPEG quality 100 as :136, or PGM).  Images whose sides are not multiples of
// 8 are cropped to the largest multiple of 8 (the reference would compute
// garbage on them).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "hpdct_compat.h"
#include "image_io.hpp"

#define CHECK_HIP(call)                                               \
    {                                                                 \
        hipError_t err = call;                                        \
        if (err != hipSuccess) {                                      \
            printf("%s : %d", hipGetErrorString(err), __LINE__);      \
            exit(EXIT_FAILURE);                                       \
        }                                                             \
    }

static void print_tile(const char* title, const float* m, int width) {
    printf("%s\n", title);
    for (int i = 0; i < 8; i++) {
        for (int j = 0; j < 8; j++) printf("%f ", m[i * width + j]);
        printf("\n");
    }
    printf("\n\n");
}

int main(int argc, char* argv[]) {
    if (argc != 3) {
        fprintf(stderr, "Usage: %s <input_image> <output_image> \n", argv[0]);
        return 1;
    }
    std::vector<uint8_t> src;
    int w0 = 0, h0 = 0;
    if (!hpdct_io::load_gray(argv[1], src, w0, h0)) {
        fprintf(stderr, "Error: Unable to open file %s\n", argv[1]);
        exit(EXIT_FAILURE);
    }
    const int width = w0 & ~7, height = h0 & ~7;
    if (width == 0 || height == 0) {
        fprintf(stderr, "Error: image smaller than 8x8\n");
        exit(EXIT_FAILURE);
    }
    const size_t px = (size_t)width * height;
    std::vector<uint8_t> gray(px);
    for (int r = 0; r < height; ++r)
        for (int c = 0; c < width; ++c) gray[(size_t)r * width + c] = src[(size_t)r * w0 + c];

    std::vector<float> image(px), result(px);
    hpdct_u8_to_f32(gray.data(), image.data(), (int64_t)px);  // convertToFloat
    char title[160];
    snprintf(title, sizeof(title), "Printing the 8x8 of image[] (matrix from the jpeg image w:%d h:%d)", width,
             height);
    print_tile(title, image.data(), width);

    float transform[64];
    hpdct_default_transform(transform);
    float *d_A, *d_B, *d_C, *d_E;
    CHECK_HIP(hipMalloc(&d_A, px * sizeof(float)));
    CHECK_HIP(hipMalloc(&d_B, 64 * sizeof(float)));
    CHECK_HIP(hipMalloc(&d_C, px * sizeof(float)));
    CHECK_HIP(hipMalloc(&d_E, px * sizeof(float)));
    CHECK_HIP(hipMemcpy(d_A, image.data(), px * sizeof(float), hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_B, transform, 64 * sizeof(float), hipMemcpyHostToDevice));

    dct_all_blocks_cuda(d_A, height, width, d_B, d_C);
    CHECK_HIP(hipMemcpy(result.data(), d_C, px * sizeof(float), hipMemcpyDeviceToHost));
    print_tile("Printing the 8x8 of result[] (matrix coming from the dct)", result.data(), width);

    idct_all_blocks_cuda(d_C, height, width, d_B, d_E);
    CHECK_HIP(hipMemcpy(result.data(), d_E, px * sizeof(float), hipMemcpyDeviceToHost));
    print_tile("Printing the 8x8 of result[] (matrix coming from the idct)", result.data(), width);

    std::vector<uint8_t> out(px);
    hpdct_f32_to_u8(result.data(), out.data(), (int64_t)px);  // convertToUnsignedChar
    printf("Printing the 8x8 of U_C[] (unsignedchar)\n");
    for (int i = 0; i < 8; i++) {
        for (int j = 0; j < 8; j++) printf("%d ", out[(size_t)i * width + j]);
        printf("\n");
    }
    printf("\n\n");

    if (hpdct_io::save_gray(argv[2], out.data(), width, height, 100)) {
        printf("Image saved successfully to %s\n", argv[2]);
    } else {
        fprintf(stderr, "Error: Failed to save image\n");
    }
    CHECK_HIP(hipFree(d_A));
    CHECK_HIP(hipFree(d_B));
    CHECK_HIP(hipFree(d_C));
    CHECK_HIP(hipFree(d_E));
    return 0;
}
