// hpdct_rt_duo.hip -- the two-lanes-per-tile round trip (hpdct_rt_duo.hpp)
// and the sums finish kernel.
#include "hpdct_rt_duo.hpp"

namespace hpdct {

hipError_t launch_rt_duo(const uint8_t* img, float* coef, void* recon, int recon_kind, unsigned long long* spread,
                         const TileGrid& g, const QParams& qp, int fast, hipStream_t s) {
    if (recon_kind == kRtReconF32) return launch_rt_duo_f32(img, coef, recon, spread, g, qp, fast, s);
    if (recon_kind == kRtReconU8) return rt_duo_detail::go_r<kRtReconU8>(img, coef, recon, spread, g, qp, fast, s);
    return rt_duo_detail::go_r<kRtReconNone>(img, coef, nullptr, spread, g, qp, fast, s);
}

hipError_t launch_rt_finish(RtSums* dst, unsigned long long* spread, bool accumulate, hipStream_t s) {
    hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, dst, spread, accumulate ? 1 : 0);
    return hipGetLastError();
}

}  // namespace hpdct
