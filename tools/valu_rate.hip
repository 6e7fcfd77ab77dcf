// valu_rate.hip -- issue rate of the VALU instructions the tile kernels are
// made of, on gfx950.  Each kernel runs 8 independent chains of one
// instruction per lane (inline asm, so the compiler cannot fold or reorder
// them away), 8 waves per SIMD on every CU; the time per wave-instruction per
// SIMD is reported in nanoseconds and relative to v_fmac_f32.
//
//   valu_rate [iters=2048] [reps=5]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

// one op on accumulator a (in/out) with the loop-invariant operands b, c
#define OP_KERNEL(NAME, ASM)                                                                  \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t seed) {    \
        uint32_t b = seed ^ threadIdx.x, c = 0x3f000000u + (seed & 0xff);                     \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,        \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                       \
        for (int i = 0; i < iters; ++i) {                                                     \
            asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                    \
        }                                                                                     \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
    }

OP_KERNEL(k_fmac, "v_fmac_f32 %0, %1, %2")
OP_KERNEL(k_fma3, "v_fma_f32 %0, %1, %2, %0")
OP_KERNEL(k_add, "v_add_f32 %0, %0, %1")
OP_KERNEL(k_mul, "v_mul_f32 %0, %0, %1")
OP_KERNEL(k_subrev, "v_subrev_f32 %0, %1, %0")
OP_KERNEL(k_cvt_ub0, "v_cvt_f32_ubyte0 %0, %0")
OP_KERNEL(k_cvt_ub3, "v_cvt_f32_ubyte3 %0, %0")
OP_KERNEL(k_cvt_f32_i32, "v_cvt_f32_i32 %0, %0")
OP_KERNEL(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %0")
OP_KERNEL(k_cvt_u32_f32, "v_cvt_u32_f32 %0, %0")
OP_KERNEL(k_cvt_rpi, "v_cvt_rpi_i32_f32 %0, %0")
OP_KERNEL(k_cvt_i32_sdwa, "v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD")
OP_KERNEL(k_cvt_f32_sdwa_sext, "v_cvt_f32_i32_sdwa %0, sext(%0) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2")
OP_KERNEL(k_min_u32_sdwa, "v_min_u32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD")
OP_KERNEL(k_cvt_pk_u8, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
OP_KERNEL(k_bfi, "v_bfi_b32 %0, %1, %0, %2")
OP_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP_KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
OP_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 8, %1")
OP_KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
OP_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
OP_KERNEL(k_bfe_i32, "v_bfe_i32 %0, %0, 8, 8")
OP_KERNEL(k_trunc, "v_trunc_f32 %0, %0")
OP_KERNEL(k_rndne, "v_rndne_f32 %0, %0")
OP_KERNEL(k_med3, "v_med3_f32 %0, %0, %1, %2")
OP_KERNEL(k_fmamk, "v_fmamk_f32 %0, %0, 0x3e9e0000, %1")
OP_KERNEL(k_dot4, "v_dot4_u32_u8 %0, %1, %2, %0")
OP_KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
OP_KERNEL(k_add_f32_abs, "v_add_f32 %0, |%0|, %1")
OP_KERNEL(k_pk_add, "v_pk_add_u16 %0, %0, %1")
OP_KERNEL(k_cvt_pk_i16_i32, "v_cvt_pk_i16_i32 %0, %0, %1")
OP_KERNEL(k_ashr_pk_i8, "v_ashr_pk_i8_i32 %0, %0, %1, 0")
OP_KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca")
OP_KERNEL(k_mov, "v_mov_b32 %0, %1")
OP_KERNEL(k_mov_dpp_ror8, "v_mov_b32_dpp %0, %1 row_ror:8 row_mask:0xf bank_mask:0x3")
OP_KERNEL(k_mov_dpp_ror8_self, "v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xc")
OP_KERNEL(k_add_u32_dpp, "v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
OP_KERNEL(k_fmac_dpp, "v_fmac_f32_dpp %0, %1, %2 row_ror:8 row_mask:0xf bank_mask:0xf")

// 64-bit operands (register pairs): packed fp32 and the 64-bit address add
#define OP64_KERNEL(NAME, ASM)                                                                \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t seed) {    \
        uint64_t b = (uint64_t)(seed ^ threadIdx.x) * 0x100000001ull, c = 0x3f0000003f000000ull; \
        uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,        \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                       \
        for (int i = 0; i < iters; ++i) {                                                     \
            asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                    \
            asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                    \
        }                                                                                     \
        const uint64_t x = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                             \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)x ^ (uint32_t)(x >> 32);              \
    }
OP64_KERNEL(k_pk_fma_f32, "v_pk_fma_f32 %0, %1, %2, %0")
OP64_KERNEL(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
OP64_KERNEL(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
OP64_KERNEL(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")

// v_permlane32_swap_b32: both operands in and out, 4 pairs x 2 per iteration
__global__ __launch_bounds__(256) void k_permlane32_swap(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a0), "+v"(a1));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a2), "+v"(a3));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a4), "+v"(a5));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a6), "+v"(a7));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a1), "+v"(a2));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a3), "+v"(a4));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a5), "+v"(a6));
        asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a7), "+v"(a0));
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

struct K {
    const char* name;
    void (*fn)(uint32_t*, int, uint32_t);
};

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 8;  // 8 x 4 waves per CU = 8 waves per SIMD
    uint32_t* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    const K ks[] = {{"v_fmac_f32", k_fmac},
                    {"v_fma_f32 (VOP3)", k_fma3},
                    {"v_pk_fma_f32", k_pk_fma_f32},
                    {"v_pk_add_f32", k_pk_add_f32},
                    {"v_pk_mul_f32", k_pk_mul_f32},
                    {"v_lshl_add_u64", k_lshl_add_u64},
                    {"v_permlane32_swap_b32", k_permlane32_swap},
                    {"v_mov_b32", k_mov},
                    {"v_mov_b32_dpp row_ror:8 bank_mask:0x3", k_mov_dpp_ror8},
                    {"v_mov_b32_dpp self row_ror:8 bank_mask:0xc", k_mov_dpp_ror8_self},
                    {"v_add_u32_dpp row_shr:1", k_add_u32_dpp},
                    {"v_fmac_f32_dpp row_ror:8", k_fmac_dpp},
                    {"v_add_f32", k_add},
                    {"v_mul_f32", k_mul},
                    {"v_subrev_f32", k_subrev},
                    {"v_fmamk_f32", k_fmamk},
                    {"v_add_f32 |a|", k_add_f32_abs},
                    {"v_cvt_f32_ubyte0", k_cvt_ub0},
                    {"v_cvt_f32_ubyte3", k_cvt_ub3},
                    {"v_cvt_f32_i32", k_cvt_f32_i32},
                    {"v_cvt_i32_f32", k_cvt_i32_f32},
                    {"v_cvt_u32_f32", k_cvt_u32_f32},
                    {"v_cvt_rpi_i32_f32", k_cvt_rpi},
                    {"v_cvt_i32_f32_sdwa BYTE_1", k_cvt_i32_sdwa},
                    {"v_cvt_f32_i32_sdwa sext BYTE_2", k_cvt_f32_sdwa_sext},
                    {"v_min_u32_sdwa BYTE_1", k_min_u32_sdwa},
                    {"v_cvt_pk_u8_f32", k_cvt_pk_u8},
                    {"v_bfi_b32", k_bfi},
                    {"v_perm_b32", k_perm},
                    {"v_and_or_b32", k_and_or},
                    {"v_lshl_or_b32", k_lshl_or},
                    {"v_xor_b32", k_xor},
                    {"v_add_u32", k_add_u32},
                    {"v_bfe_i32", k_bfe_i32},
                    {"v_trunc_f32", k_trunc},
                    {"v_rndne_f32", k_rndne},
                    {"v_med3_f32", k_med3},
                    {"v_dot4_u32_u8", k_dot4},
                    {"v_cndmask_b32", k_cndmask},
                    {"v_pk_add_u16", k_pk_add},
                    {"v_cvt_pk_i16_i32", k_cvt_pk_i16_i32},
                    {"v_ashr_pk_i8_i32", k_ashr_pk_i8},
                    {"v_bitop3_b32", k_bitop3}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // warm the clocks
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_fmac, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
    CK(hipDeviceSynchronize());
    const double winst_per_simd = (double)blocks * 4 * iters * 8 / (cus * 4);  // wave-instructions per SIMD
    double ref = 0;
    printf("%-34s %10s %12s %8s\n", "instruction", "us", "ns/winst/SIMD", "vs fmac");
    for (const K& k : ks) {
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, iters, 7u + r);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ns = t[t.size() / 2] * 1e6 / winst_per_simd;
        if (ref == 0) ref = ns;
        printf("%-34s %10.1f %12.3f %8.2f\n", k.name, t[t.size() / 2] * 1e3, ns, ns / ref);
    }
    return 0;
}
