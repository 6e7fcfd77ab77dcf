// hpdct_roundtrip.hip -- launcher of the one-pass round trip: which kernel
// (the two-lanes-per-tile kernel of hpdct_rt_duo.hpp, or the tile-per-lane
// kernel of hpdct_roundtrip.hpp) and where its quality sums go.
#include <map>
#include <mutex>
#include <vector>

#include "hpdct.h"
#include "hpdct_roundtrip.hpp"

namespace hpdct {
namespace {

// Spread slots for the sums (kRtSpread sub-slots, kRtSpreadBytes = 16 KiB
// each), one per (device, caller's sums pointer), handed out from zeroed
// chunks: the round trip adds into the slot and rt_spread_finish_kernel folds
// it into the caller's struct, leaving it zero for the next launch with that
// pointer.  Launches with one sums pointer share its slot; the fold is atomic,
// so accumulate launches on different streams lose nothing.  A
// slot stays with its pointer until hpdct_roundtrip_release_sums returns it
// to the device's free list.  nullptr when a new chunk would be needed inside
// a stream capture, or past kMaxSlots live pointers on a device (64 MiB of
// slots): the launch then takes the tile kernel with a memset of *sums
// (overwrite) or atomics into *sums (accumulate).
constexpr size_t kSlotChunk = 256;  // 256 x 16 KiB = 4 MiB per allocation
constexpr size_t kMaxSlots = size_t(1) << 12;

struct DeviceSlots {
    std::map<const void*, unsigned long long*> by_sums;
    std::vector<unsigned long long*> free;  // released slots (zero)
    unsigned char* chunk = nullptr;
    size_t used = kSlotChunk;
    hipStream_t zero_stream = nullptr;
};

std::mutex g_slot_mutex;
std::map<int, DeviceSlots> g_slots;

unsigned long long* slot_for(int dev, const void* sums, hipStream_t s) {
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    DeviceSlots& d = g_slots[dev];
    auto it = d.by_sums.find(sums);
    if (it != d.by_sums.end()) return it->second;
    if (!d.free.empty()) {
        unsigned long long* const slot = d.free.back();
        d.free.pop_back();
        d.by_sums.emplace(sums, slot);
        return slot;
    }
    if (d.by_sums.size() >= kMaxSlots) return nullptr;
    if (d.used == kSlotChunk) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        // relaxed capture mode for this thread while it allocates and
        // synchronises: a stream capture another thread runs in global mode
        // is then left intact
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        if (hipThreadExchangeStreamCaptureMode(&mode) != hipSuccess) return nullptr;
        struct Restore {
            hipStreamCaptureMode m;
            ~Restore() { (void)hipThreadExchangeStreamCaptureMode(&m); }
        } restore{mode};
        if (!d.zero_stream && hipStreamCreateWithFlags(&d.zero_stream, hipStreamNonBlocking) != hipSuccess) {
            d.zero_stream = nullptr;
            return nullptr;
        }
        void* p = nullptr;
        if (hipMalloc(&p, kSlotChunk * kRtSpreadBytes) != hipSuccess) return nullptr;
        // zero before any stream can launch with one of its slots
        if (hipMemsetAsync(p, 0, kSlotChunk * kRtSpreadBytes, d.zero_stream) != hipSuccess ||
            hipStreamSynchronize(d.zero_stream) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        d.chunk = static_cast<unsigned char*>(p);
        d.used = 0;
    }
    auto* const slot = reinterpret_cast<unsigned long long*>(d.chunk + d.used++ * kRtSpreadBytes);
    d.by_sums.emplace(sums, slot);
    return slot;
}

// A launch that failed after the round trip was queued may leave its slot
// non-zero.  The slot is zeroed behind it on the same stream, so the pointer
// keeps its slot (a graph captured earlier with that slot stays correct);
// only when even that fails does the pointer get a fresh slot next time.
void recover_slot(int dev, const void* sums, unsigned long long* slot, hipStream_t s) {
    if (hipMemsetAsync(slot, 0, kRtSpreadBytes, s) == hipSuccess) return;
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    g_slots[dev].by_sums.erase(sums);
}

}  // namespace

// hpdct_roundtrip_release_sums: the slot of `sums` (on whichever device holds
// one) back to that device's free list.  The caller guarantees no launch with
// that pointer is still in flight, so the slot is zero (each fold leaves it
// so).  Returns whether the pointer had a slot.
bool release_sums_slot(const void* sums) {
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    bool found = false;
    for (auto& kv : g_slots) {
        DeviceSlots& d = kv.second;
        auto it = d.by_sums.find(sums);
        if (it == d.by_sums.end()) continue;
        d.free.push_back(it->second);
        d.by_sums.erase(it);
        found = true;
    }
    return found;
}

namespace {

hipError_t tile(const uint8_t* img, float* coef, void* recon, int recon_kind, RtSums* sums, const TileGrid& g,
                const QParams& qp, int fast, hipStream_t s) {
    switch (recon_kind) {
        case kRtReconU8: return launch_rt_tile_u8(img, coef, recon, sums, g, qp, fast, s);
        case kRtReconF32: return launch_rt_tile_f32(img, coef, recon, sums, g, qp, fast, s);
        default: return launch_rt_tile_none(img, coef, nullptr, sums, g, qp, fast, s);
    }
}

}  // namespace

// The kernel: the two-lanes-per-tile round trip (hpdct_rt_duo.hpp) for the
// verified quotient (fast 1 or 2) with any reconstruction, when its sums (if
// any) have a spread slot, the width is a multiple of 256 pixels (whole
// 32-tile runs per wave) and the mapping is not forced to "tile"; 8192^2
// with sums and a uint8 reconstruction 74.3-74.8 us against 78.4 for the
// tile kernel with the same sums path, without sums 67.0 against 76.8
// (tools/kb_rt, profiles/r05/f/).  Otherwise the tile-per-lane kernel (IEEE
// division, ragged widths, forced tile mapping), with its sums in the spread
// slot's sub-slot 0 when it has one.  The duo kernel addresses a wave's rows
// with 32-bit byte offsets from the wave's base (DuoAddr, 2 k width + 4 lane
// fp32 words), which stay below 2^32 for widths below 2^22 pixels; wider
// frames take the tile kernel.
hipError_t launch_roundtrip(const uint8_t* img, float* coef, void* recon, int recon_kind, RtSums* sums,
                            const TileGrid& g, const QParams& qp, int fast, bool zero_sums, hipStream_t s) {
    int dev = -1;
    unsigned long long* slot = nullptr;
    if (sums && hipGetDevice(&dev) == hipSuccess) slot = slot_for(dev, sums, s);
    const bool duo = fast != 0 && (!sums || slot) && g.tiles_x % 32u == 0u && g.width < (uint64_t(1) << 22) &&
                     mapping_mode() != HPDCT_MAPPING_TILE;
    hipError_t e;
    if (duo) {
        e = launch_rt_duo(img, coef, recon_kind == kRtReconNone ? nullptr : recon, recon_kind, slot, g, qp, fast, s);
    } else if (slot) {
        e = tile(img, coef, recon, recon_kind, reinterpret_cast<RtSums*>(slot), g, qp, fast, s);
    } else {
        if (sums && zero_sums) {
            e = hipMemsetAsync(sums, 0, sizeof(RtSums), s);
            if (e != hipSuccess) return e;
        }
        return tile(img, coef, recon, recon_kind, sums, g, qp, fast, s);
    }
    if (e == hipSuccess && slot) e = launch_rt_finish(sums, slot, !zero_sums, s);
    if (e != hipSuccess && slot) recover_slot(dev, sums, slot, s);
    return e;
}

}  // namespace hpdct
