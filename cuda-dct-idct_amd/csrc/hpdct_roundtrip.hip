// hpdct_roundtrip.hip -- launcher of the one-pass round trip (hpdct_roundtrip.hpp).
#include <map>
#include <mutex>

#include "hpdct_roundtrip.hpp"

namespace hpdct {
namespace {

// Sums slots for hpdct_roundtrip_u8, one per (device, caller's sums pointer),
// handed out from zeroed chunks and never returned: the round trip adds into
// the slot and rt_finish_kernel moves it over the caller's struct, leaving it
// zero for the next launch with that pointer.  Launches with one sums pointer
// are ordered (one stream, or one graph) or race on the caller's struct
// anyway, so they may share its slot.  nullptr (the launch then zeroes the
// caller's struct with a memset) when a new chunk would be needed inside a
// stream capture, or past kMaxSlots pointers on a device.
constexpr size_t kSlotChunk = 1024;
constexpr size_t kMaxSlots = size_t(1) << 16;

struct DeviceSlots {
    std::map<const void*, RtSums*> by_sums;
    RtSums* chunk = nullptr;
    size_t used = kSlotChunk;
    hipStream_t zero_stream = nullptr;
};

std::mutex g_slot_mutex;
std::map<int, DeviceSlots> g_slots;

RtSums* slot_for(int dev, const void* sums, hipStream_t s) {
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    DeviceSlots& d = g_slots[dev];
    auto it = d.by_sums.find(sums);
    if (it != d.by_sums.end()) return it->second;
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
        if (hipMalloc(&p, kSlotChunk * sizeof(RtSums)) != hipSuccess) return nullptr;
        // zero before any stream can launch with one of its slots
        if (hipMemsetAsync(p, 0, kSlotChunk * sizeof(RtSums), d.zero_stream) != hipSuccess ||
            hipStreamSynchronize(d.zero_stream) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        d.chunk = static_cast<RtSums*>(p);
        d.used = 0;
    }
    RtSums* const slot = d.chunk + d.used++;
    d.by_sums.emplace(sums, slot);
    return slot;
}

// A launch that failed after the round trip was queued may leave its slot
// non-zero.  The slot is zeroed behind it on the same stream, so the pointer
// keeps its slot (a graph captured earlier with that slot stays correct);
// only when even that fails does the pointer get a fresh slot next time.
void recover_slot(int dev, const void* sums, RtSums* slot, hipStream_t s) {
    if (hipMemsetAsync(slot, 0, sizeof(RtSums), s) == hipSuccess) return;
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    g_slots[dev].by_sums.erase(sums);
}

}  // namespace

hipError_t launch_roundtrip(const uint8_t* img, float* coef, void* recon, int recon_kind, RtSums* sums,
                            const TileGrid& g, const QParams& qp, int fast, bool zero_sums, hipStream_t s) {
    int dev = -1;
    RtSums* slot = nullptr;
    if (sums && zero_sums && hipGetDevice(&dev) == hipSuccess) slot = slot_for(dev, sums, s);
    const hipError_t e = launch_roundtrip_impl(img, coef, recon, recon_kind, sums, g, qp, fast, s, zero_sums, slot);
    if (e != hipSuccess && slot) recover_slot(dev, sums, slot, s);
    return e;
}

}  // namespace hpdct
