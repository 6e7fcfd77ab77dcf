// hpdct_fwd_f32.hip -- forward kernels with fp32 input (the reference's own
// input type; compat path).  Kernels: hpdct_kernels_impl.hpp.
#include "hpdct_launch.hpp"

namespace hpdct {
#define HPDCT_FWD(TI, TO, QN, BT, WB)                                                                       \
    template <>                                                                                             \
    hipError_t launch_fdct<TI, TO, QN, BT, WB>(const TI* a, TO* b, float* c, const TileGrid& g, const float* t, \
                                               const QParams& q, float sh, int fd, bool rf, hipStream_t s) {  \
        return launch_fdct_impl<TI, TO, QN, BT, WB>(a, b, c, g, t, q, sh, fd, rf, s);                       \
    }
#define HPDCT_FWD_T(TI, TO, QN, WB) HPDCT_FWD(TI, TO, QN, true, WB) HPDCT_FWD(TI, TO, QN, false, WB)
HPDCT_FWD_T(float, float, true, false)
HPDCT_FWD_T(float, float, false, false)
HPDCT_FWD_T(float, float, true, true)
HPDCT_FWD_T(float, float, false, true)
}  // namespace hpdct
