// hpdct_fwd_f32.hip -- forward kernels with fp32 input (the reference's own
// input type; compat path).  Kernels: hpdct_kernels_impl.hpp.
#include "hpdct_kernels_impl.hpp"

namespace hpdct {
#define HPDCT_FWD(TI, TO, QN, BT, WB)                                                                              \
    template hipError_t launch_fdct<TI, TO, QN, BT, WB>(const TI*, TO*, float*, const TileGrid&, const float*,   \
                                                        const Mat64&, float, hipStream_t);
#define HPDCT_FWD_T(TI, TO, QN, WB) HPDCT_FWD(TI, TO, QN, true, WB) HPDCT_FWD(TI, TO, QN, false, WB)
HPDCT_FWD_T(float, float, true, false)
HPDCT_FWD_T(float, float, false, false)
HPDCT_FWD_T(float, float, true, true)
HPDCT_FWD_T(float, float, false, true)
}  // namespace hpdct
