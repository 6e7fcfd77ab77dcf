// hpdct_tables.h -- the two constant tables of the HpApprDCT path, ONE copy
// shared by the kernels (hpdct_tile.hpp: immediates of the built-in T, the
// default Q) and the host C-ABI (hpdct_api.cpp: hpdct_default_transform /
// hpdct_default_quant_table, the library-owned Q's initial value).
//
// The reference stores double literals into float arrays
// (main_newAppr.cu:60-81, Benchmark_code/benchmark_newAppr.cu:54-75), so each
// entry is (float)(double)literal.  Pinned bit for bit against the literals
// extracted from the reference's own text: tests/golden/ref_tables.json
// (tests/golden/make_golden.py), tests/test_abi.py::test_tables_pinned_to_reference_text.
#pragma once

namespace hpdct {
namespace tables {

#define HPDCT_TA ((float)0.35355339)
#define HPDCT_TH ((float)0.5)
#define HPDCT_TB ((float)0.4472136)
#define HPDCT_TC ((float)0.2236068)
#define HPDCT_TD ((float)0.70710678)
// HpApprDCT transform matrix T (main_newAppr.cu:73-81)
inline constexpr float kT[64] = {
    HPDCT_TA,  HPDCT_TA,  HPDCT_TA,  HPDCT_TA,  HPDCT_TA,  HPDCT_TA,  HPDCT_TA,  HPDCT_TA,
    HPDCT_TH,  HPDCT_TH,  0.0f,      0.0f,      0.0f,      0.0f,      -HPDCT_TH, -HPDCT_TH,
    HPDCT_TB,  HPDCT_TC,  -HPDCT_TC, -HPDCT_TB, -HPDCT_TB, -HPDCT_TC, HPDCT_TC,  HPDCT_TB,
    0.0f,      0.0f,      -HPDCT_TD, 0.0f,      0.0f,      HPDCT_TD,  0.0f,      0.0f,
    HPDCT_TA,  -HPDCT_TA, -HPDCT_TA, HPDCT_TA,  HPDCT_TA,  -HPDCT_TA, -HPDCT_TA, HPDCT_TA,
    HPDCT_TH,  -HPDCT_TH, 0.0f,      0.0f,      0.0f,      0.0f,      HPDCT_TH,  -HPDCT_TH,
    HPDCT_TC,  -HPDCT_TB, HPDCT_TB,  -HPDCT_TC, -HPDCT_TC, HPDCT_TB,  -HPDCT_TB, HPDCT_TC,
    0.0f,      0.0f,      0.0f,      -HPDCT_TD, HPDCT_TD,  0.0f,      0.0f,      0.0f};
#undef HPDCT_TA
#undef HPDCT_TH
#undef HPDCT_TB
#undef HPDCT_TC
#undef HPDCT_TD

// JPEG luminance quantisation table (main_newAppr.cu:60-68)
inline constexpr float kQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                 14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                 18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};

}  // namespace tables
}  // namespace hpdct
