// hpdct_inv_i8.hip -- inverse kernels, int8 coefficients in (split from
// hpdct_inv.hip so the two halves compile in parallel).  Kernels: hpdct_kernels_impl.hpp.
#include "hpdct_launch.hpp"

namespace hpdct {
#define HPDCT_INV(TI, TO, DQ, BT)                                                                          \
    template <>                                                                                             \
    hipError_t launch_idct<TI, TO, DQ, BT>(const TI* a, TO* b, float* w, const TileGrid& g, const float* t,  \
                                           const Mat64& q, float sh, bool rf, hipStream_t s) {              \
        return launch_idct_impl<TI, TO, DQ, BT>(a, b, w, g, t, q, sh, rf, s);                               \
    }
#define HPDCT_INV_T(TI, TO, DQ) HPDCT_INV(TI, TO, DQ, true) HPDCT_INV(TI, TO, DQ, false)
HPDCT_INV_T(int8_t, float, true)
HPDCT_INV_T(int8_t, float, false)
HPDCT_INV_T(int8_t, uint8_t, true)
HPDCT_INV_T(int8_t, uint8_t, false)
}  // namespace hpdct
