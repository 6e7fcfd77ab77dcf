// hpdct_probe.hip -- floor probes for hpdct_floor_probe (include/hpdct.h): what
// a launch of the uint8 -> fp32 forward of a given frame costs with no
// transform in it.  Measurement only; the product path never calls them.
//
//   empty  an empty kernel on the forward's own grid and workgroup size: the
//          dispatch and wave-launch cost of that grid, no memory traffic
//   copy   the same grid moving the same bytes: 1 B read and 4 B written per
//          pixel (each byte converted to fp32, non-temporal stores), no
//          arithmetic: what the memory system allows for this frame
//
// For a small frame (C2, 1024^2: 2,048 octet waves, cache-resident) the gap
// between the forward and these floors is the part of its time the transform
// itself costs (bench.py extras c2_floor_us).
#include "hpdct_launch.hpp"

namespace hpdct {

namespace {

__global__ void floor_empty_kernel() {}

// lane i of the grid converts pixels [8i, 8i + 8) (+ k * stride): one 8-byte
// load, two 16-byte non-temporal stores per step
__global__ void floor_copy_kernel(const uint8_t* __restrict__ in, float* __restrict__ out, uint64_t n) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x * 8u;
    for (uint64_t i = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 8u; i < n; i += stride) {
        if (i + 8u <= n) {
            const uint2 w = *reinterpret_cast<const uint2*>(in + i);
            float4 a, b;
            a.x = byte_f32(w.x, 0), a.y = byte_f32(w.x, 1), a.z = byte_f32(w.x, 2), a.w = byte_f32(w.x, 3);
            b.x = byte_f32(w.y, 0), b.y = byte_f32(w.y, 1), b.z = byte_f32(w.y, 2), b.w = byte_f32(w.y, 3);
            st<true>(reinterpret_cast<float4*>(out + i), a);
            st<true>(reinterpret_cast<float4*>(out + i) + 1, b);
        } else {
            for (uint64_t j = i; j < n; ++j) out[j] = static_cast<float>(in[j]);
        }
    }
}

}  // namespace

// The (grid, workgroup) the uint8 -> fp32 forward launches for g
// (launch_fdct_impl -> fdct_octet_go / fdct_tile_go), without its residency cap.
void forward_u8_f32_shape(const TileGrid& g, dim3& grid, dim3& block) {
    if (pick_mapping(g, false) == Mapping::kOctet) {
        constexpr unsigned kV = kOctVar<float>;
        grid = octet_grid(g, kBlock<kV>), block = dim3(kBlock<kV>);
        return;
    }
    const uint32_t sets_per_cu = ((g.ntiles + 63u) / 64u + device_cus() - 1u) / device_cus();
    const uint32_t b = sets_per_cu <= kBigWgSetsPerCU ? 1024u : 64u;
    grid = grid_for(g, false, 0, b), block = dim3(b);
}

hipError_t launch_floor_probe(int kind, const uint8_t* in, float* out, const TileGrid& g, hipStream_t s) {
    dim3 grid, block;
    forward_u8_f32_shape(g, grid, block);
    if (kind == 0) {
        hipLaunchKernelGGL(floor_empty_kernel, grid, block, 0, s);
    } else {
        hipLaunchKernelGGL(floor_copy_kernel, grid, block, 0, s, in, out, static_cast<uint64_t>(g.ntiles) * 64u);
    }
    return hipGetLastError();
}

}  // namespace hpdct
