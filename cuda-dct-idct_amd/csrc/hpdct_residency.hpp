// hpdct_residency.hpp -- residency caps by dynamic-LDS reservation (round 3):
// the device attributes the caps read and the reservation that leaves room for
// at most k workgroups per CU.  Shared by the launch choice (hpdct_launch.hpp)
// and the round-trip / duo-forward launchers (hpdct_rt_duo.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace hpdct {

// The cap is set by reserving dynamic LDS the kernel does not use: a
// workgroup that holds more than 1/(k+1) of the CU's LDS leaves room for at
// most k.  The LDS size is the device's own
// (hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 160 KiB on gfx950 per
// MI355X_MICROARCH.md), so the caps keep their meaning on a part with another
// LDS size.
constexpr size_t kLdsPerCUDefault = 160u * 1024u;

// A device attribute of the current device, cached per thread and device.
template <hipDeviceAttribute_t kAttr>
inline int device_attr(int fallback) {
    static thread_local int cached_dev = -1;
    static thread_local int cached = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fallback;
    if (dev != cached_dev) {
        int v = 0;
        cached = hipDeviceGetAttribute(&v, kAttr, dev) == hipSuccess && v > 0 ? v : fallback;
        cached_dev = dev;
    }
    return cached;
}
inline uint32_t device_cus() {
    return static_cast<uint32_t>(device_attr<hipDeviceAttributeMultiprocessorCount>(256));
}
inline size_t device_lds_per_cu() {
    return static_cast<size_t>(
        device_attr<hipDeviceAttributeMaxSharedMemoryPerMultiprocessor>(static_cast<int>(kLdsPerCUDefault)));
}

// dynamic LDS bytes for at most `wgs` resident workgroups per CU of a kernel
// that has `static_bytes` of its own (0 when no reservation is needed)
inline size_t residency_cap_lds(size_t static_bytes, uint32_t wgs) {
    if (wgs == 0) return 0;
    const size_t per = (device_lds_per_cu() / wgs) & ~static_cast<size_t>(511);
    return per > static_bytes ? per - static_bytes : 0;
}
template <typename K>
size_t static_lds_of(K kern) {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kern)) == hipSuccess ? a.sharedSizeBytes : 0;
}

}  // namespace hpdct
