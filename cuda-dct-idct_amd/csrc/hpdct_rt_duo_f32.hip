// hpdct_rt_duo_f32.hip -- the two-lanes-per-tile round trip with an fp32
// reconstruction (hpdct_rt_duo.hpp), in a translation unit of its own so the
// round-trip kernels compile in parallel.
#include "hpdct_rt_duo.hpp"

namespace hpdct {

hipError_t launch_rt_duo_f32(const uint8_t* img, float* coef, void* recon, unsigned long long* spread,
                             const TileGrid& g, const QParams& qp, int fast, hipStream_t s) {
    return rt_duo_detail::go_r<kRtReconF32>(img, coef, recon, spread, g, qp, fast, s);
}

}  // namespace hpdct
