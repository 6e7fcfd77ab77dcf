// asan_host_check.cpp -- the host-side code of the path under AddressSanitizer
// + UndefinedBehaviorSanitizer ("race detection /
// sanitizers"; the reference's only safety net is CHECK_CUDA,
// main_newAppr.cu:9-17).  CPU only: built by tests/tools/asan.mk with g++
// (-fsanitize=address,undefined on host code; the gfx950 kernel objects are
// linked unsanitised and never launched -- there is no GPU here).
//
// Exercised, every buffer heap-allocated at its exact size so an overrun is a
// sanitizer report:
//   * C-ABI host helpers (hpdct_api.cpp): fill_rand / u8<->f32 at ragged sizes,
//     against the oracle's restatements (oracle/hpdct_oracle.c, also sanitised);
//   * the library-owned quant table: set / get / reset from 8 threads (mutex);
//   * every argument-validation path of hpdct_forward / hpdct_inverse /
//     hpdct_roundtrip_u8 / hpdct_stream_forward / hpdct_fill_hash_u8 that
//     returns before device work, and the thread-local last-error string;
//   * the oracle's transforms, quality and generators at ragged sizes;
//   * host/image_io.hpp: PGM round trip and malformed headers (overflowing
//     dimensions, truncated data).
// Exit 0 = every check passed and no sanitizer report (reports abort).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "../../cuda-dct-idct_amd/host/image_io.hpp"
#include "hpdct.h"

using namespace hpdct_io;

extern "C" {
void oracle_default_quant(float* q);
void oracle_default_transform(float* t);
void oracle_fill_rand_u8(uint8_t* out, int64_t n, uint32_t seed);
void oracle_fill_hash_u8(uint8_t* out, int64_t n, uint64_t seed, int64_t first_index);
void oracle_u8_to_f32(const uint8_t* in, float* out, int64_t n);
void oracle_f32_to_u8(const float* in, uint8_t* out, int64_t n);
void oracle_fdct(const float* img, int64_t h, int64_t w, const float* T, const float* Q, float* out, int mode);
void oracle_fdct_u8(const uint8_t* img, int64_t h, int64_t w, const float* T, const float* Q, float* out, int mode);
void oracle_idct(const float* coef, int64_t h, int64_t w, const float* T, const float* Q, float* out, int mode);
void oracle_quality(const float* x, const float* y, int64_t n, double* peen, double* mse);
}

static int g_fail = 0;
#define CHECK(cond)                                                         \
    do {                                                                    \
        if (!(cond)) {                                                      \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

template <typename T>
static T* exact(size_t n) {  // heap block of exactly n elements
    return static_cast<T*>(malloc(n ? n * sizeof(T) : 1));
}

static void host_helpers() {
    for (int64_t n : {0, 1, 7, 63, 64, 65, 1000, 4097}) {
        uint8_t* a = exact<uint8_t>(n);
        uint8_t* b = exact<uint8_t>(n);
        hpdct_fill_rand_u8(a, n, 42);
        oracle_fill_rand_u8(b, n, 42);
        CHECK(n == 0 || memcmp(a, b, n) == 0);
        float* f = exact<float>(n);
        float* g = exact<float>(n);
        hpdct_u8_to_f32(a, f, n);
        oracle_u8_to_f32(a, g, n);
        CHECK(n == 0 || memcmp(f, g, n * sizeof(float)) == 0);
        for (int64_t i = 0; i < n; ++i) f[i] = (float)(i % 300) - 20.5f;  // out-of-range values too
        hpdct_f32_to_u8(f, a, n);
        oracle_f32_to_u8(f, b, n);
        CHECK(n == 0 || memcmp(a, b, n) == 0);
        free(a), free(b), free(f), free(g);
    }
    float t[64], t2[64], q[64], q2[64];
    hpdct_default_transform(t);
    oracle_default_transform(t2);
    hpdct_default_quant_table(q);
    oracle_default_quant(q2);
    CHECK(memcmp(t, t2, sizeof t) == 0 && memcmp(q, q2, sizeof q) == 0);
    CHECK(strstr(hpdct_version(), "gfx950") != nullptr);
    for (int s = -1; s < 8; ++s) CHECK(hpdct_status_string((hpdct_status)s) != nullptr);
}

static void quant_table_threads() {
    std::vector<std::thread> th;
    for (int k = 0; k < 8; ++k) {
        th.emplace_back([k] {
            float q[64], got[64];
            for (int it = 0; it < 200; ++it) {
                for (int i = 0; i < 64; ++i) q[i] = (float)(1 + (i + k + it) % 200);
                CHECK(hpdct_set_quant_table(q) == HPDCT_SUCCESS);
                CHECK(hpdct_get_quant_table(got) == HPDCT_SUCCESS);
                // some thread's complete table (or the default after a reset), never a mix
                bool whole = true, dflt = true;
                for (int i = 1; i < 64; ++i) whole &= ((int)got[i] - (int)got[0] + 200) % 200 == i % 200;
                float d[64];
                hpdct_default_quant_table(d);
                for (int i = 0; i < 64; ++i) dflt &= got[i] == d[i];
                CHECK(whole || dflt);
                if (it % 50 == 0) CHECK(hpdct_set_quant_table(nullptr) == HPDCT_SUCCESS);
            }
        });
    }
    for (auto& t : th) t.join();
    float bad[64];
    for (int i = 0; i < 64; ++i) bad[i] = 1.0f;
    bad[9] = 0.0f;
    CHECK(hpdct_set_quant_table(bad) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_get_quant_table(nullptr) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_set_quant_table(nullptr) == HPDCT_SUCCESS);
}

static void validation_paths() {
    void* a = (void*)(uintptr_t)(1 << 20);
    void* b = (void*)(uintptr_t)(1u << 30);
    void* c = (void*)((uintptr_t)1 << 31);
    auto* s = (hpdct_roundtrip_sums*)((uintptr_t)1 << 32);
    const int64_t bad[][2] = {{0, 8}, {8, 0}, {12, 8}, {8, 20}, {-8, 8}, {7, 7}, {INT64_MAX, 8}, {8, INT64_MIN}};
    for (auto& hw : bad) {
        CHECK(hpdct_forward(a, HPDCT_U8, b, HPDCT_F32, hw[0], hw[1], nullptr, 0, nullptr) == HPDCT_ERROR_INVALID_VALUE);
        CHECK(strlen(hpdct_last_error_string()) > 0);
        CHECK(hpdct_inverse(a, HPDCT_F32, b, HPDCT_F32, hw[0], hw[1], nullptr, 0, nullptr) ==
              HPDCT_ERROR_INVALID_VALUE);
        CHECK(hpdct_roundtrip_u8((uint8_t*)a, (float*)b, c, HPDCT_U8, s, hw[0], hw[1], nullptr) ==
              HPDCT_ERROR_INVALID_VALUE);
    }
    CHECK(hpdct_forward(nullptr, HPDCT_U8, b, HPDCT_F32, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_forward(a, HPDCT_I8, b, HPDCT_F32, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_forward(a, HPDCT_U8, b, HPDCT_U8, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_forward(a, (hpdct_dtype)99, b, HPDCT_F32, 8, 8, nullptr, 0, nullptr) != HPDCT_SUCCESS);
    CHECK(hpdct_forward(a, HPDCT_U8, b, HPDCT_F32, 8, 8, nullptr, 0x80, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_forward((char*)a + 4, HPDCT_F32, b, HPDCT_F32, 8, 8, nullptr, 0, nullptr) ==
          HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_forward(a, HPDCT_F32, (char*)a + 64, HPDCT_F32, 8, 8, nullptr, 0, nullptr) ==
          HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_inverse(a, HPDCT_U8, b, HPDCT_F32, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_inverse(a, HPDCT_F32, b, HPDCT_I8, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_roundtrip_u8(nullptr, (float*)b, c, HPDCT_U8, s, 8, 8, nullptr) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_roundtrip_u8((uint8_t*)a, (float*)b, c, HPDCT_I8, s, 8, 8, nullptr) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_roundtrip_u8((uint8_t*)a, (float*)b, (char*)b + 64, HPDCT_U8, nullptr, 8, 8, nullptr) ==
          HPDCT_ERROR_INVALID_VALUE);
    CHECK(strstr(hpdct_last_error_string(), "overlap") != nullptr);
    CHECK(hpdct_roundtrip_u8_accumulate((uint8_t*)a, (float*)b, c, HPDCT_U8, nullptr, 8, 8, nullptr) ==
          HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_roundtrip_u8_accumulate((uint8_t*)a, (float*)b, c, HPDCT_U8, s, 12, 8, nullptr) ==
          HPDCT_ERROR_INVALID_VALUE);
    float ones[64];
    for (float& v : ones) v = 1.0f;
    CHECK(hpdct_set_quant_table(ones) == HPDCT_SUCCESS);
    CHECK(hpdct_forward(a, HPDCT_U8, b, HPDCT_I8, 8, 8, nullptr, 0, nullptr) == HPDCT_ERROR_RANGE);
    CHECK(hpdct_set_quant_table(nullptr) == HPDCT_SUCCESS);
    CHECK(hpdct_fill_hash_u8(nullptr, 64, 42, 0, nullptr) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_fill_hash_u8((uint8_t*)a, -1, 42, 0, nullptr) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_set_mapping((hpdct_mapping)7) == HPDCT_ERROR_INVALID_VALUE);

    // hpdct_forward_frames: the pointer-table checks (exact-size host tables;
    // the device pointers are never dereferenced on the host)
    {
        const uint8_t** fin = exact<const uint8_t*>(3);
        void** fout = exact<void*>(3);
        fin[0] = (const uint8_t*)(uintptr_t(1) << 20), fin[1] = (const uint8_t*)(uintptr_t(1) << 21), fin[2] = fin[0];
        fout[0] = (void*)(uintptr_t(1) << 30), fout[1] = (void*)((uintptr_t(1) << 30) + (1u << 22));
        fout[2] = (void*)(uintptr_t(1) << 31);
        CHECK(hpdct_forward_frames(fin, fout, HPDCT_F32, 0, 64, 64, nullptr) == HPDCT_SUCCESS);
        CHECK(hpdct_forward_frames(fin, fout, HPDCT_F32, -3, 64, 64, nullptr) == HPDCT_ERROR_INVALID_VALUE);
        CHECK(hpdct_forward_frames(nullptr, fout, HPDCT_F32, 3, 64, 64, nullptr) == HPDCT_ERROR_INVALID_VALUE);
        CHECK(hpdct_forward_frames(fin, fout, HPDCT_U8, 3, 64, 64, nullptr) == HPDCT_ERROR_UNSUPPORTED);
        fout[1] = (void*)((uintptr_t(1) << 30) + 64);  // overlaps out 0
        CHECK(hpdct_forward_frames(fin, fout, HPDCT_F32, 3, 64, 64, nullptr) == HPDCT_ERROR_INVALID_VALUE);
        CHECK(strstr(hpdct_last_error_string(), "overlap") != nullptr);
        fout[1] = nullptr;
        CHECK(hpdct_forward_frames(fin, fout, HPDCT_I8, 3, 64, 64, nullptr) == HPDCT_ERROR_INVALID_VALUE);
        free(fin);
        free(fout);
    }

    // hpdct_stream_forward: every check that precedes stream creation
    std::vector<uint8_t> px(64 * 64);
    std::vector<float> out(64 * 64);
    const uint8_t* frames[3] = {px.data(), nullptr, px.data()};
    void* outs[3] = {out.data(), out.data(), out.data()};
    float ms = -1;
    CHECK(hpdct_stream_forward(nullptr, outs, 1, 64, 64, HPDCT_F32, 2, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, nullptr, 1, 64, 64, HPDCT_F32, 2, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, outs, -1, 64, 64, HPDCT_F32, 2, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, outs, 1, 64, 64, HPDCT_F32, 0, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, outs, 1, 64, 64, HPDCT_F32, 17, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, outs, 1, 64, 64, HPDCT_U8, 2, &ms) == HPDCT_ERROR_UNSUPPORTED);
    CHECK(hpdct_stream_forward(frames, outs, 1, 60, 64, HPDCT_F32, 2, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(hpdct_stream_forward(frames, outs, 3, 64, 64, HPDCT_F32, 2, &ms) == HPDCT_ERROR_INVALID_VALUE);
    CHECK(strstr(hpdct_last_error_string(), "index 1") != nullptr);
    CHECK(hpdct_stream_forward(frames, outs, 0, 64, 64, HPDCT_F32, 2, &ms) == HPDCT_SUCCESS);
}

static void oracle_paths() {
    float T[64], Q[64];
    oracle_default_transform(T);
    oracle_default_quant(Q);
    const int64_t shapes[][2] = {{8, 8}, {16, 24}, {40, 8}, {8, 136}, {24, 24}};
    for (auto& hw : shapes) {
        const int64_t n = hw[0] * hw[1];
        uint8_t* img = exact<uint8_t>(n);
        oracle_fill_hash_u8(img, n, 42, 7);
        float* f = exact<float>(n);
        oracle_u8_to_f32(img, f, n);
        float* q = exact<float>(n);
        float* q2 = exact<float>(n);
        float* r = exact<float>(n);
        for (int mode = 0; mode < 4; ++mode) {
            oracle_fdct_u8(img, hw[0], hw[1], T, Q, q, mode);
            oracle_fdct(f, hw[0], hw[1], T, Q, q2, mode);
            CHECK(memcmp(q, q2, n * sizeof(float)) == 0);
            oracle_idct(q, hw[0], hw[1], T, Q, r, mode);
        }
        oracle_fdct_u8(img, hw[0], hw[1], T, Q, q, 0);
        oracle_idct(q, hw[0], hw[1], T, Q, r, 0);
        double peen = -1, mse = -1;
        oracle_quality(f, r, n, &peen, &mse);
        CHECK(peen >= 0 && mse >= 0);
        free(img), free(f), free(q), free(q2), free(r);
    }
}

static void write_file(const std::string& p, const std::string& bytes) {
    FILE* f = fopen(p.c_str(), "wb");
    fwrite(bytes.data(), 1, bytes.size(), f);
    fclose(f);
}

static void image_io_paths(const std::string& dir) {
    const int w = 24, h = 16;
    std::vector<uint8_t> px(w * h);
    for (int i = 0; i < w * h; ++i) px[i] = (uint8_t)(i * 7);
    const std::string p = dir + "/asan_rt.pgm";
    CHECK(save_pgm(p, px.data(), w, h));
    std::vector<uint8_t> back;
    int w2 = 0, h2 = 0;
    CHECK(load_gray(p, back, w2, h2) && w2 == w && h2 == h && back == px);
    const char* bad[] = {"P5 99999999999 8 255\n", "P5 8 8 255\n\x01\x02", "P5 -3 8 255\n", "P6 8 8 255\n",
                         "P5 70000 70000 255\n", "P5 8 8 0\n", "", "P5"};
    for (const char* b : bad) {
        write_file(p, b);
        CHECK(!load_pgm(p, back, w2, h2));
    }
    CHECK(!load_pgm(dir + "/does_not_exist.pgm", back, w2, h2));
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    host_helpers();
    quant_table_threads();
    validation_paths();
    oracle_paths();
    image_io_paths(dir);
    printf("asan_host_check: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
