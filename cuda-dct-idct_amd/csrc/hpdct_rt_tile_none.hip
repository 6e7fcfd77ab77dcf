// hpdct_rt_tile_none.hip -- the tile-per-lane round trip (hpdct_roundtrip.hpp)
// with the kRtReconNone reconstruction: every (sums, quotient) variant, in a
// translation unit of its own so the round-trip variants compile in parallel.
#include "hpdct_roundtrip.hpp"

namespace hpdct {

hipError_t launch_rt_tile_none(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g,
                           const QParams& qp, int fast, hipStream_t s) {
    return rt_detail::go_r<kRtReconNone>(img, coef, recon, sums, g, qp, fast, s);
}

}  // namespace hpdct
