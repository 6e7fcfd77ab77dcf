// hpdct_rt_duo.hip -- the two-lanes-per-tile round trip (hpdct_rt_duo.hpp)
// and the sums finish kernel.
#include "hpdct_residency.hpp"
#include "hpdct_rt_duo.hpp"

namespace hpdct {

namespace {
template <int kQMode>
hipError_t fdct_duo_u8_go(const uint8_t* img, float* coef, const TileGrid& g, const QParams& qp, hipStream_t s) {
    static_assert(kDuoFwdBlock == 256, "fdct_duo_u8_kernel is built for 256-thread workgroups");
    auto* const kern = fdct_duo_u8_kernel<kQMode>;
    static const size_t st = static_lds_of(kern);
    hipLaunchKernelGGL(kern, roundtrip_duo_grid(g, kDuoFwdBlock), dim3(kDuoFwdBlock),
                       residency_cap_lds(st, kDuoFwdCapWgs), s, img, coef, g, qp);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_fdct_duo_u8(const uint8_t* img, float* coef, const TileGrid& g, const QParams& qp, int qmode,
                              hipStream_t s) {
    return qmode == 2 ? fdct_duo_u8_go<2>(img, coef, g, qp, s) : fdct_duo_u8_go<1>(img, coef, g, qp, s);
}

namespace {
template <int kQMode>
hipError_t fdct_duo_u8_frames_go(const FrameTable<float>& ft, int n, const TileGrid& g, const QParams& qp,
                                 hipStream_t s) {
    auto* const kern = fdct_duo_u8_frames_kernel<kQMode>;
    static const size_t st = static_lds_of(kern);
    const dim3 grid(roundtrip_duo_grid(g, kDuoFwdBlock).x, static_cast<uint32_t>(n));
    hipLaunchKernelGGL(kern, grid, dim3(kDuoFwdBlock), residency_cap_lds(st, kDuoFwdCapWgs), s, ft, g, qp);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_fdct_duo_u8_frames(const FrameTable<float>& ft, int n, const TileGrid& g, const QParams& qp,
                                     int qmode, hipStream_t s) {
    return qmode == 2 ? fdct_duo_u8_frames_go<2>(ft, n, g, qp, s) : fdct_duo_u8_frames_go<1>(ft, n, g, qp, s);
}

hipError_t launch_rt_duo(const uint8_t* img, float* coef, void* recon, int recon_kind, unsigned long long* spread,
                         const TileGrid& g, const QParams& qp, int fast, hipStream_t s) {
    if (recon_kind == kRtReconF32) return launch_rt_duo_f32(img, coef, recon, spread, g, qp, fast, s);
    if (recon_kind == kRtReconU8) return rt_duo_detail::go_r<kRtReconU8>(img, coef, recon, spread, g, qp, fast, s);
    // neither a reconstruction nor sums: the forward alone, capped
    if (!spread) return launch_fdct_duo_u8(img, coef, g, qp, fast, s);
    return rt_duo_detail::go_r<kRtReconNone>(img, coef, nullptr, spread, g, qp, fast, s);
}

hipError_t launch_rt_finish(RtSums* dst, unsigned long long* spread, bool accumulate, hipStream_t s) {
    hipLaunchKernelGGL(rt_spread_finish_kernel<>, dim3(1), dim3(64), 0, s, dst, spread, accumulate ? 1 : 0);
    return hipGetLastError();
}

}  // namespace hpdct
