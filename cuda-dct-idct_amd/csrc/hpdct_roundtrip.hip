// hpdct_roundtrip.hip -- launcher of the one-pass round trip (hpdct_roundtrip.hpp).
#include "hpdct_roundtrip.hpp"

namespace hpdct {
hipError_t launch_roundtrip(const uint8_t* img, float* coef, void* recon, int recon_kind, RtSums* sums,
                            const TileGrid& g, const QParams& qp, int fast, bool zero_sums, hipStream_t s) {
    return launch_roundtrip_impl(img, coef, recon, recon_kind, sums, g, qp, fast, s, zero_sums);
}
}  // namespace hpdct
