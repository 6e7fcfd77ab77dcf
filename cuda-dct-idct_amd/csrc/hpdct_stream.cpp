// hpdct_stream.cpp -- host-resident frame batches through the forward pass
// with copy/compute overlap (BASELINE config C5: a batch of independent
// frames streamed H2D / D2H).  The reference has no equivalent: its drivers
// do one blocking cudaMemcpy each way per image (benchmark_newAppr.cu:88,97).
//
// Pipeline: frame f goes to stream f % nstreams, which owns one device input
// and one device output buffer; on that stream: H2D copy -> fused forward
// kernel -> D2H copy.  Streams run concurrently, so the H2D DMA of one frame,
// the kernel of another and the D2H DMA of a third overlap; a stream's own
// operations are ordered, which makes its buffer reuse safe.  Host buffers
// should be pinned (hipHostMalloc / torch pin_memory) for the copies to be
// asynchronous and overlap.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "hpdct.h"

namespace {
struct DeviceRing {
    std::vector<hipStream_t> streams;
    std::vector<void*> in, out;
    ~DeviceRing() {
        for (void* p : in) (void)hipFree(p);
        for (void* p : out) (void)hipFree(p);
        for (hipStream_t s : streams) (void)hipStreamDestroy(s);
    }
};
}  // namespace

extern "C" hpdct_status hpdct_stream_forward(const uint8_t* const* h_frames, void* const* h_coef, int64_t n_frames,
                                             int64_t height, int64_t width, hpdct_dtype out_type, int nstreams,
                                             float* elapsed_ms) {
    if (!h_frames || !h_coef || n_frames < 0 || nstreams < 1 || nstreams > 16) return HPDCT_ERROR_INVALID_VALUE;
    if (out_type != HPDCT_F32 && out_type != HPDCT_I8) return HPDCT_ERROR_UNSUPPORTED;
    if (height <= 0 || width <= 0 || height % 8 || width % 8) return HPDCT_ERROR_INVALID_VALUE;
    for (int64_t f = 0; f < n_frames; ++f)
        if (!h_frames[f] || !h_coef[f]) return HPDCT_ERROR_INVALID_VALUE;
    if (n_frames == 0) {
        if (elapsed_ms) *elapsed_ms = 0.0f;
        return HPDCT_SUCCESS;
    }
    const size_t px = static_cast<size_t>(height) * static_cast<size_t>(width);
    const size_t out_bytes = px * (out_type == HPDCT_F32 ? 4 : 1);
    DeviceRing ring;
    for (int s = 0; s < nstreams; ++s) {
        hipStream_t st;
        void *di = nullptr, *dout = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return HPDCT_ERROR_DEVICE;
        ring.streams.push_back(st);
        if (hipMalloc(&di, px) != hipSuccess) return HPDCT_ERROR_DEVICE;
        ring.in.push_back(di);
        if (hipMalloc(&dout, out_bytes) != hipSuccess) return HPDCT_ERROR_DEVICE;
        ring.out.push_back(dout);
    }
    hipEvent_t t0, t1;
    if (hipEventCreate(&t0) != hipSuccess || hipEventCreate(&t1) != hipSuccess) return HPDCT_ERROR_DEVICE;
    // start marker: every stream waits for it, so the timed region holds the whole batch
    hipError_t e = hipEventRecord(t0, ring.streams[0]);
    for (int s = 1; s < nstreams && e == hipSuccess; ++s) e = hipStreamWaitEvent(ring.streams[s], t0, 0);
    for (int64_t f = 0; f < n_frames && e == hipSuccess; ++f) {
        const int s = static_cast<int>(f % nstreams);
        hipStream_t st = ring.streams[s];
        e = hipMemcpyAsync(ring.in[s], h_frames[f], px, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) break;
        const hpdct_status hs = hpdct_forward(ring.in[s], HPDCT_U8, ring.out[s], out_type, height, width, nullptr,
                                              0u, st);
        if (hs != HPDCT_SUCCESS) {
            (void)hipEventDestroy(t0);
            (void)hipEventDestroy(t1);
            (void)hipDeviceSynchronize();
            return hs;
        }
        e = hipMemcpyAsync(h_coef[f], ring.out[s], out_bytes, hipMemcpyDeviceToHost, st);
    }
    // end marker after every stream's last operation
    for (int s = 1; s < nstreams && e == hipSuccess; ++s) {
        hipEvent_t done;
        e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
        if (e != hipSuccess) break;
        e = hipEventRecord(done, ring.streams[s]);
        if (e == hipSuccess) e = hipStreamWaitEvent(ring.streams[0], done, 0);
        (void)hipEventDestroy(done);
    }
    if (e == hipSuccess) e = hipEventRecord(t1, ring.streams[0]);
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    for (hipStream_t st : ring.streams) (void)hipStreamSynchronize(st);
    if (e != hipSuccess) return HPDCT_ERROR_DEVICE;
    if (elapsed_ms) *elapsed_ms = ms;
    return HPDCT_SUCCESS;
}
