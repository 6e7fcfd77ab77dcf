// shard_bench.hpp -- `benchmark_hpdct <n> [runs] --gpus N [--int8]`: BASELINE
// config C4 from ONE process driving N GPUs (no fork, no exec): an n x n
// synthetic frame (pixel i = splitmix64(42, i) & 255, generated on each
// device for its own rows) row-sharded over the devices, the fused forward on
// every slab, then the RCCL gather of the coefficient slabs to device 0
// (include/hpdct_dist.h: ncclCommInitAll, ncclSend/ncclRecv in one group).
// The gathered frame is compared byte for byte with a one-GPU forward of the
// whole frame on device 0, and the per-phase times are printed:
//   SHARD (W,H) x N: compute <max over devices> ms, gather <root> ms,
//   one-GPU <full frame> ms, compute speedup <x>, bit-exact <yes|NO>
// The reference has no multi-GPU mode; its driver's
// shape (benchmark_newAppr.cu:33-119: argv size, synthetic input, events
// around the work, one printed line per phase) is kept.
#pragma once

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "hpdct.h"
#include "hpdct_dist.h"

#define CHECK_HPDCT(call)                                                                          \
    {                                                                                              \
        hpdct_status st_ = call;                                                                   \
        if (st_ != HPDCT_SUCCESS) {                                                                \
            printf("%s : %d (%s)\n", hpdct_status_string(st_), __LINE__, hpdct_last_error_string()); \
            exit(EXIT_FAILURE);                                                                    \
        }                                                                                          \
    }

static int run_sharded(size_t n, int ngpus, bool int8, long runs) {
    int visible = 0;
    CHECK_HIP(hipGetDeviceCount(&visible));
    if (ngpus < 1 || ngpus > visible) {
        printf("--gpus %d but %d device(s) visible\n", ngpus, visible);
        return 1;
    }
    const hpdct_dtype ot = int8 ? HPDCT_I8 : HPDCT_F32;
    const size_t esz = int8 ? 1 : 4;
    const int64_t h = (int64_t)n, w = (int64_t)n;
    std::vector<int> devs(ngpus);
    for (int d = 0; d < ngpus; ++d) devs[d] = d;
    std::vector<hpdct_comm> comms(ngpus);
    CHECK_HPDCT(hpdct_comm_init_all(comms.data(), ngpus, devs.data()));

    // every device rotates over enough slab copies that its inputs total >= 1 GiB,
    // 4x the 256 MiB Infinity Cache: each timed forward then reads HBM, not the
    // cache (at 8 GPUs a 16384^2 slab is 32 MiB)
    constexpr size_t kRotateBytes = size_t(1) << 30;
    struct Dev {
        hipStream_t s;
        std::vector<uint8_t*> slab;  // identical copies, rotated
        void* coef;
        int64_t first, rows;
        hipEvent_t e0, e1, e2;
    };
    std::vector<Dev> dv(ngpus);
    void* frame = nullptr;  // the gathered frame, on device 0
    for (int d = 0; d < ngpus; ++d) {
        Dev& x = dv[d];
        CHECK_HIP(hipSetDevice(d));
        CHECK_HIP(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking));
        CHECK_HPDCT(hpdct_shard_rows(h, ngpus, d, &x.first, &x.rows));
        const size_t slab_bytes = (size_t)x.rows * n;
        x.slab.resize(std::min<size_t>(64, (kRotateBytes + slab_bytes - 1) / slab_bytes));
        for (uint8_t*& p : x.slab) CHECK_HIP(hipMalloc(&p, slab_bytes));
        CHECK_HIP(hipMalloc(&x.coef, (size_t)x.rows * n * esz));
        if (d == 0) CHECK_HIP(hipMalloc(&frame, n * n * esz));
        CHECK_HIP(hipEventCreate(&x.e0));
        CHECK_HIP(hipEventCreate(&x.e1));
        CHECK_HIP(hipEventCreate(&x.e2));
        for (uint8_t* p : x.slab) CHECK_HPDCT(hpdct_fill_hash_u8(p, x.rows * w, 42, x.first * w, x.s));
    }
    float best_c = 1e30f, best_g = 1e30f;
    for (long r = 0; r < (runs > 0 ? runs : 1); ++r) {
        for (int d = 0; d < ngpus; ++d) {
            CHECK_HIP(hipSetDevice(d));
            CHECK_HIP(hipStreamSynchronize(dv[d].s));
            CHECK_HIP(hipEventRecord(dv[d].e0, dv[d].s));
            CHECK_HPDCT(hpdct_forward_slab(comms[d], dv[d].slab[r % dv[d].slab.size()], dv[d].coef, ot, h, w,
                                           dv[d].s));
            CHECK_HIP(hipEventRecord(dv[d].e1, dv[d].s));
        }
        CHECK_HPDCT(hpdct_group_start());
        for (int d = 0; d < ngpus; ++d)
            CHECK_HPDCT(hpdct_gather_rows(comms[d], dv[d].coef, d == 0 ? frame : nullptr, ot, h, w, 0, dv[d].s));
        CHECK_HPDCT(hpdct_group_end());
        float cmax = 0.0f, g0 = 0.0f;
        for (int d = 0; d < ngpus; ++d) {
            CHECK_HIP(hipSetDevice(d));
            CHECK_HIP(hipEventRecord(dv[d].e2, dv[d].s));
            CHECK_HIP(hipEventSynchronize(dv[d].e2));
            float c = 0.0f, g = 0.0f;
            CHECK_HIP(hipEventElapsedTime(&c, dv[d].e0, dv[d].e1));
            CHECK_HIP(hipEventElapsedTime(&g, dv[d].e1, dv[d].e2));
            cmax = std::max(cmax, c);
            if (d == 0) g0 = g;
        }
        best_c = std::min(best_c, cmax);
        best_g = std::min(best_g, g0);
    }
    // one GPU, whole frame, on device 0: the reference for bit-exactness and speedup
    CHECK_HIP(hipSetDevice(0));
    std::vector<uint8_t*> full_in(std::min<size_t>(64, (kRotateBytes + n * n - 1) / (n * n)));
    void* full_out = nullptr;
    for (uint8_t*& p : full_in) {
        CHECK_HIP(hipMalloc(&p, n * n));
        CHECK_HPDCT(hpdct_fill_hash_u8(p, h * w, 42, 0, dv[0].s));
    }
    CHECK_HIP(hipMalloc(&full_out, n * n * esz));
    float best_one = 1e30f;
    for (long r = 0; r < (runs > 0 ? runs : 1) + 1; ++r) {
        CHECK_HIP(hipEventRecord(dv[0].e0, dv[0].s));
        CHECK_HPDCT(hpdct_forward(full_in[r % full_in.size()], HPDCT_U8, full_out, ot, h, w, nullptr, 0u, dv[0].s));
        CHECK_HIP(hipEventRecord(dv[0].e1, dv[0].s));
        CHECK_HIP(hipEventSynchronize(dv[0].e1));
        float ms = 0.0f;
        CHECK_HIP(hipEventElapsedTime(&ms, dv[0].e0, dv[0].e1));
        if (r > 0) best_one = std::min(best_one, ms);  // the first launch loads the code object
    }
    std::vector<char> a(n * n * esz), b(n * n * esz);
    CHECK_HIP(hipMemcpy(a.data(), frame, a.size(), hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(b.data(), full_out, b.size(), hipMemcpyDeviceToHost));
    const bool same = memcmp(a.data(), b.data(), a.size()) == 0;
    printf("SHARD (%zu,%zu) x %d %s: compute %f ms, gather %f ms, one-GPU %f ms, compute speedup %.2f, bit-exact %s\n",
           n, n, ngpus, int8 ? "int8" : "fp32", best_c, best_g, best_one, best_one / best_c, same ? "yes" : "NO");
    for (uint8_t* p : full_in) CHECK_HIP(hipFree(p));
    CHECK_HIP(hipFree(full_out));
    for (int d = 0; d < ngpus; ++d) {
        CHECK_HIP(hipSetDevice(d));
        for (uint8_t* p : dv[d].slab) CHECK_HIP(hipFree(p));
        CHECK_HIP(hipFree(dv[d].coef));
        CHECK_HIP(hipEventDestroy(dv[d].e0));
        CHECK_HIP(hipEventDestroy(dv[d].e1));
        CHECK_HIP(hipEventDestroy(dv[d].e2));
        CHECK_HIP(hipStreamDestroy(dv[d].s));
        CHECK_HPDCT(hpdct_comm_destroy(comms[d]));
    }
    CHECK_HIP(hipSetDevice(0));
    CHECK_HIP(hipFree(frame));
    return same ? 0 : 1;
}
