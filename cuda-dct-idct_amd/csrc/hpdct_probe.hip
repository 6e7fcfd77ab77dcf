// hpdct_probe.hip -- floor probes for hpdct_floor_probe and the copy ceilings
// of hpdct_copy_ceiling (include/hpdct_baseline.h): what a launch of the
// uint8 -> fp32 forward of a given frame costs with no transform in it, and
// what the memory system allows for the bytes each kernel of the path moves.
// Measurement only; the product path never calls them.
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

// The copy ceiling of a kernel that reads kIn bytes and writes kO0 (+ kO1)
// bytes per pixel (hpdct_copy_ceiling).  One wave per workgroup, 2,048 pixels
// per wave.  kA pixels per lane and instruction: 4 when a plane is fp32 (each
// fp32 instruction 1 KiB contiguous, as the kernels' re-staged row stores),
// else 8 (8 B per lane, as the int8 forward's row accesses).  All loads are
// issued before the first store.  The dynamic LDS argument only caps
// residency; the kernel does not touch it.
constexpr uint32_t kCeilPx = 2048;
__device__ __forceinline__ void st_nt(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ uint32_t pack4_trunc(const float4& f) {
    return (static_cast<uint32_t>(f.x) & 255u) | (static_cast<uint32_t>(f.y) & 255u) << 8 |
           (static_cast<uint32_t>(f.z) & 255u) << 16 | (static_cast<uint32_t>(f.w) & 255u) << 24;
}
// in and o1 may be one plane (an in-place write-back, as the drop-in
// kernels' X-128 and q*Q planes): each lane stores only what it loaded.
template <int kIn, int kO0, int kO1>
__global__ __launch_bounds__(64) void copy_ceiling_kernel(const void* in, void* __restrict__ o0, void* o1) {
    constexpr bool kWide = kIn == 4 || kO0 == 4 || kO1 == 4;
    constexpr uint32_t kA = kWide ? 4u : 8u, kG = kCeilPx / (64u * kA);
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kCeilPx + threadIdx.x * kA;
    if constexpr (!kWide) {
        uint2 r[kG];
        unroll<kG>([&](auto k) { r[k] = *reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(in) + base + k * 512u); });
        unroll<kG>([&](auto k) {
            st<true>(reinterpret_cast<uint2*>(static_cast<uint8_t*>(o0) + base + k * 512u), r[k]);
            if constexpr (kO1 != 0) st<true>(reinterpret_cast<uint2*>(static_cast<uint8_t*>(o1) + base + k * 512u), r[k]);
        });
    } else {
        float4 f[kG];
        unroll<kG>([&](auto k) {
            if constexpr (kIn == 4) {
                f[k] = *reinterpret_cast<const float4*>(static_cast<const float*>(in) + base + k * 256u);
            } else {
                const uint32_t w = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(in) + base + k * 256u);
                f[k] = make_float4(byte_f32(w, 0), byte_f32(w, 1), byte_f32(w, 2), byte_f32(w, 3));
            }
        });
        auto put = [&](void* o, auto bytes, auto k) {
            if constexpr (decltype(bytes)::value == 4) {
                st<true>(reinterpret_cast<float4*>(static_cast<float*>(o) + base + k * 256u), f[k]);
            } else {
                st_nt(reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(o) + base + k * 256u), pack4_trunc(f[k]));
            }
        };
        unroll<kG>([&](auto k) {
            put(o0, std::integral_constant<int, kO0>{}, k);
            if constexpr (kO1 != 0) put(o1, std::integral_constant<int, kO1>{}, k);
        });
    }
}

template <int kIn, int kO0, int kO1>
hipError_t copy_ceiling_go(const void* in, void* o0, void* o1, uint64_t n, uint32_t cap_waves, hipStream_t s) {
    const size_t dyn = residency_cap_lds(0, cap_waves);
    hipLaunchKernelGGL((copy_ceiling_kernel<kIn, kO0, kO1>), dim3(static_cast<uint32_t>(n / kCeilPx)), dim3(64), dyn,
                       s, in, o0, o1);
    return hipGetLastError();
}

template <int kIn, int kO0>
hipError_t copy_ceiling_o1(const void* in, void* o0, void* o1, int o1_bytes, uint64_t n, uint32_t cap,
                           hipStream_t s) {
    switch (o1_bytes) {
        case 0: return copy_ceiling_go<kIn, kO0, 0>(in, o0, nullptr, n, cap, s);
        case 1: return copy_ceiling_go<kIn, kO0, 1>(in, o0, o1, n, cap, s);
        default: return copy_ceiling_go<kIn, kO0, 4>(in, o0, o1, n, cap, s);
    }
}

}  // namespace

hipError_t launch_copy_ceiling(const void* in, int in_bytes, void* o0, int o0_bytes, void* o1, int o1_bytes,
                               uint64_t n, uint32_t cap_waves, hipStream_t s) {
    if (in_bytes == 1) {
        return o0_bytes == 1 ? copy_ceiling_o1<1, 1>(in, o0, o1, o1_bytes, n, cap_waves, s)
                             : copy_ceiling_o1<1, 4>(in, o0, o1, o1_bytes, n, cap_waves, s);
    }
    return o0_bytes == 1 ? copy_ceiling_o1<4, 1>(in, o0, o1, o1_bytes, n, cap_waves, s)
                         : copy_ceiling_o1<4, 4>(in, o0, o1, o1_bytes, n, cap_waves, s);
}

// The (grid, workgroup) the uint8 -> fp32 forward with the default table
// launches for g (launch_fdct_impl -> launch_fdct_duo_u8 / fdct_octet_go /
// fdct_tile_go), without its residency cap.
void forward_u8_f32_shape(const TileGrid& g, dim3& grid, dim3& block) {
    if (duo_fwd_u8_fits(g)) {
        const uint32_t waves = (g.ntiles + 31u) / 32u, per = kDuoFwdBlock / 64u;
        grid = dim3((waves + per - 1u) / per), block = dim3(kDuoFwdBlock);
        return;
    }
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
