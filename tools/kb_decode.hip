// kb_decode.hip -- A/B of the int8 -> fp32 decode kernel (csrc/hpdct_decode.hpp)
// at the C4 root's size: n int8 coefficients (default 16384^2), rotating
// buffer sets whose inputs total >= 1 GiB (4x the Infinity Cache), every
// variant checked byte for byte against the first, median of batch averages.
//   kb_decode [n=268435456] [iters=40] [rounds=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hpdct_decode.hpp"
#include "hpdct_launch.hpp"

using namespace hpdct;

int hpdct::mapping_mode() { return 0; }

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

typedef void (*Fn)(const int8_t*, float*, uint64_t, hipStream_t);

template <int kB, int kU>
void one_shot(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL((decode_i8_f32_kernel<kB, kU, false>), dim3((uint32_t)decode_blocks<kB, kU>(n, 0)), dim3(kB), 0,
                       s, in, out, n);
}
// one-wave workgroups, at most kCap resident per CU (dynamic-LDS reservation, as the headline)
template <int kU, uint32_t kCap>
void capped(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    auto* k = decode_i8_f32_kernel<64, kU, false>;
    static const size_t dyn = residency_cap_lds(static_lds_of(k), kCap);
    hipLaunchKernelGGL(k, dim3((uint32_t)decode_blocks<64, kU>(n, 0)), dim3(64), dyn, s, in, out, n);
}
// persistent: kWavesPerCU waves per CU walk the plane
template <int kB, int kU, uint32_t kWavesPerCU>
void persist(const int8_t* in, float* out, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL((decode_i8_f32_kernel<kB, kU, true>),
                       dim3((uint32_t)decode_blocks<kB, kU>(n, (uint64_t)device_cus() * kWavesPerCU)), dim3(kB), 0, s,
                       in, out, n);
}

void product(const int8_t* in, float* out, uint64_t n, hipStream_t s) { (void)launch_decode_i8_f32(in, out, n, s); }

struct V {
    const char* name;
    Fn fn;
};

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (uint64_t)16384 * 16384;
    const int iters = argc > 2 ? atoi(argv[2]) : 40;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const int nsets = std::max<int>(2, (int)((4ull << 28) / n + ((4ull << 28) % n != 0)));
    std::vector<V> vars = {
        {"b256 1 KiB/wave (round-4 first)", one_shot<256, 1>},
        {"product (hpdct_decode_i8_f32 launcher)", product},
        {"b256 2 KiB/wave", one_shot<256, 2>},
        {"b256 4 KiB/wave", one_shot<256, 4>},
        {"b512 1 KiB/wave", one_shot<512, 1>},
        {"b64 1 KiB cap 8 w/cu", capped<1, 8>},
        {"b64 1 KiB cap 10 w/cu", capped<1, 10>},
        {"b64 1 KiB cap 12 w/cu", capped<1, 12>},
        {"b64 1 KiB cap 14 w/cu", capped<1, 14>},
        {"b64 1 KiB cap 16 w/cu", capped<1, 16>},
        {"b64 1 KiB cap 12 w/cu again", capped<1, 12>},
        {"b64 2 KiB cap 8 w/cu", capped<2, 8>},
        {"b64 2 KiB cap 16 w/cu", capped<2, 16>},
        {"b256 1 KiB persistent 8 w/cu", persist<256, 1, 8>},
        {"b256 1 KiB persistent 16 w/cu", persist<256, 1, 16>},
        {"b256 2 KiB persistent 16 w/cu", persist<256, 2, 16>},
        {"product again", product},
    };
    std::vector<int8_t*> in(nsets);
    std::vector<float*> out(nsets);
    std::vector<int8_t> h(n);
    srand(42);
    for (uint64_t i = 0; i < n; ++i) h[i] = (int8_t)(rand() % 256);
    for (int k = 0; k < nsets; ++k) {
        CK(hipMalloc(&in[k], n));
        CK(hipMalloc(&out[k], n * 4));
        CK(hipMemcpy(in[k], h.data(), n, hipMemcpyHostToDevice));
    }
    // correctness: every variant against (float)q, ragged n included by the tail path
    std::vector<float> got(n);
    for (auto& v : vars) {
        CK(hipMemset(out[0], 0xa5, n * 4));
        v.fn(in[0], out[0], n, 0);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), out[0], n * 4, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; ++i) bad += got[i] != (float)h[i];
        printf("check %-36s %s\n", v.name, bad ? "MISMATCH" : "exact");
        if (bad) return 1;
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> us(vars.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int w = 0; w < 2 * nsets; ++w) vars[v].fn(in[w % nsets], out[w % nsets], n, 0);
            for (int i = 0; i < iters; i += nsets) {
                CK(hipEventRecord(a, 0));
                for (int k = 0; k < nsets; ++k) vars[v].fn(in[k], out[k], n, 0);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                us[v].push_back(ms * 1e3f / nsets);
            }
        }
    printf("n = %llu, %d sets\n%-36s %10s %10s %8s\n", (unsigned long long)n, nsets, "variant", "median_us", "min_us",
           "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = us[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        printf("%-36s %10.2f %10.2f %8.3f\n", vars[v].name, med, t[0], 5.0 * n / (med * 1e-6) / 8e12);
    }
    return 0;
}
