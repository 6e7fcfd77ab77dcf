// hpdct_rt_tile_u8.hip -- the tile-per-lane round trip (hpdct_roundtrip.hpp)
// with the kRtReconU8 reconstruction: every (sums, quotient) variant, in a
// translation unit of its own so the round-trip variants compile in parallel.
#include "hpdct_roundtrip.hpp"

namespace hpdct {

hipError_t launch_rt_tile_u8(const uint8_t* img, float* coef, void* recon, RtSums* sums, const TileGrid& g,
                           const QParams& qp, int fast, hipStream_t s) {
    return rt_detail::go_r<kRtReconU8>(img, coef, recon, sums, g, qp, fast, s);
}

}  // namespace hpdct
