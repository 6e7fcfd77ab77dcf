// hpdct_frames.hip -- forward over a list of uint8 frames, one launch per up
// to kMaxFramesPerLaunch frames (own TU so it builds in parallel).  Kernel:
// fdct_frames_kernel in hpdct_kernels_impl.hpp.
#include "hpdct_launch.hpp"

namespace hpdct {
template <>
hipError_t launch_fdct_frames<float>(const FrameTable<float>& ft, int n, const TileGrid& g, const QParams& q,
                                     int fd, hipStream_t s) {
    return launch_fdct_frames_impl<float>(ft, n, g, q, fd, s);
}
template <>
hipError_t launch_fdct_frames<int8_t>(const FrameTable<int8_t>& ft, int n, const TileGrid& g, const QParams& q,
                                      int fd, hipStream_t s) {
    return launch_fdct_frames_impl<int8_t>(ft, n, g, q, fd, s);
}
}  // namespace hpdct
