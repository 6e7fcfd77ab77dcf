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
#include "hpdct_kernels.h"

namespace {
hpdct_status fail(hpdct_status st, const std::string& msg) {
    return static_cast<hpdct_status>(hpdct::set_last_error(st, msg.c_str()));
}
hpdct_status device_fail(hipError_t e, const char* what) {
    return fail(HPDCT_ERROR_DEVICE, std::string("hpdct_stream_forward: ") + what + ": " + hipGetErrorString(e));
}

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
    if (!h_frames || !h_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: null frame list");
    if (n_frames < 0) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: negative frame count");
    if (nstreams < 1 || nstreams > 16)
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: nstreams must be in 1..16");
    if (out_type != HPDCT_F32 && out_type != HPDCT_I8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "hpdct_stream_forward: output must be HPDCT_F32 or HPDCT_I8");
    if (height <= 0 || width <= 0 || height % 8 || width % 8)
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: height and width must be positive multiples of 8");
    for (int64_t f = 0; f < n_frames; ++f)
        if (!h_frames[f] || !h_coef[f])
            return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: null frame or output pointer at index " +
                                                       std::to_string(f));
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
        hipError_t he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (he != hipSuccess) return device_fail(he, "hipStreamCreateWithFlags");
        ring.streams.push_back(st);
        if ((he = hipMalloc(&di, px)) != hipSuccess) return device_fail(he, "hipMalloc (frames)");
        ring.in.push_back(di);
        if ((he = hipMalloc(&dout, out_bytes)) != hipSuccess) return device_fail(he, "hipMalloc (coefficients)");
        ring.out.push_back(dout);
    }
    hipEvent_t t0, t1;
    if (hipError_t he = hipEventCreate(&t0); he != hipSuccess) return device_fail(he, "hipEventCreate");
    if (hipError_t he = hipEventCreate(&t1); he != hipSuccess) {
        (void)hipEventDestroy(t0);
        return device_fail(he, "hipEventCreate");
    }
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
    if (e != hipSuccess) return device_fail(e, "copy/compute pipeline");
    if (elapsed_ms) *elapsed_ms = ms;
    return HPDCT_SUCCESS;
}
