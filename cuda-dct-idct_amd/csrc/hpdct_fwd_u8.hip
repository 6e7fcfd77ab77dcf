// hpdct_fwd_u8.hip -- forward kernels with uint8 input (one TU per input type
// so the instantiations build in parallel).  Kernels: hpdct_kernels_impl.hpp.
#include "hpdct_launch.hpp"

namespace hpdct {
#define HPDCT_FWD(TI, TO, QN, BT, WB)                                                                       \
    template <>                                                                                             \
    hipError_t launch_fdct<TI, TO, QN, BT, WB>(const TI* a, TO* b, float* c, const TileGrid& g, const float* t, \
                                               const QParams& q, float sh, int fd, bool rf, hipStream_t s) {  \
        return launch_fdct_impl<TI, TO, QN, BT, WB>(a, b, c, g, t, q, sh, fd, rf, s);                       \
    }
#define HPDCT_FWD_T(TI, TO, QN, WB) HPDCT_FWD(TI, TO, QN, true, WB) HPDCT_FWD(TI, TO, QN, false, WB)
HPDCT_FWD_T(uint8_t, float, true, false)
HPDCT_FWD_T(uint8_t, float, false, false)
HPDCT_FWD_T(uint8_t, int8_t, true, false)

hipError_t launch_fill_hash(uint8_t* out, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    return launch_fill_hash_impl(out, n, seed, first, s);
}
}  // namespace hpdct
