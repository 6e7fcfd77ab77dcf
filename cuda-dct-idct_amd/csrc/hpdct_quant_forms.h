// hpdct_quant_forms.h -- per-position quantiser forms for the DEFAULT JPEG
// table (main_newAppr.cu:60-68) with uint8 input, the built-in T and the
// reference's level shift of 128: the only case the kernels use them in
// (kVarJpegQ, hpdct_kernels_impl.hpp; chosen on the host by hpdct_api.cpp).
//
// The reference quantises with round(C / Q) (utils_kernels.cu:42: IEEE fp32
// division, then roundf).  With X - 128 in [-128, 127] the coefficient at
// (v, u) is bounded by 128 * |T_v|_1 * |T_u|_1 (* (1 + 2^-16) for the fp32
// chains), 256 .. 1024 depending on the position.  Below each position's
// bound, one of two 3-operation forms gives exactly the reference's value,
// with r = RN(1/Q):
//   F  trunc(fma(C, r, copysign(0.49999997f, C)))
//   H  trunc(fma(C, r, copysign(0.5f, C)))
// proved exhaustively over every fp32 C up to the bound by
// tests/tools/verify_quant_pos.c (run and compared with these masks by
// tests/test_quant_forms.py).  The other 25 positions keep the verified 6-op
// form: the 3-op quotient (exact for |C| <= 4096, verify_fastdiv) and the
// 3-op roundf.  39 of 64 positions take 3 operations instead of 6.
#pragma once

#include <stdint.h>

namespace hpdct {
namespace quantforms {

// bit p = v * 8 + u set: form F (bias 0.49999997) is exact at that position
inline constexpr uint64_t kJpegF = 0x43169a554274082dull;
// bit p set: form H (bias 0.5) at that position (F not exact there, H is)
inline constexpr uint64_t kJpegH = 0xa8894480a800a000ull;
static_assert((kJpegF & kJpegH) == 0, "one form per position");

enum : int { kFull = 0, kFormF = 1, kFormH = 2 };
constexpr int jpeg_form(int pos) {
    return ((kJpegF >> pos) & 1u) ? kFormF : ((kJpegH >> pos) & 1u) ? kFormH : kFull;
}
// the bias magnitude of a short form
constexpr float jpeg_bias(int pos) { return jpeg_form(pos) == kFormF ? 0.49999997f : 0.5f; }

}  // namespace quantforms
}  // namespace hpdct
