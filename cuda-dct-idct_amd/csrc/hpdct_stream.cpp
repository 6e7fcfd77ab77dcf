// hpdct_stream.cpp -- host-resident frame batches through the forward pass
// with copy/compute overlap (BASELINE config C5: a batch of independent
// frames streamed H2D / D2H).  The reference has no equivalent: its drivers
// do one blocking cudaMemcpy each way per image (benchmark_newAppr.cu:88,97).
//
// Pipeline ("streams", the product): frame f goes to stream f % nstreams,
// which owns one device input and one device output buffer; on that stream:
// H2D copy -> fused forward kernel -> D2H copy.  Streams run concurrently, so
// the H2D DMA of one frame, the kernel of another and the D2H DMA of a third
// overlap; a stream's own operations are ordered, which makes its buffer reuse
// safe.  With 2 streams each DMA direction stays busy in steady state (a
// stream's H2D of frame f + 2 follows its own D2H of frame f, which follows the
// other stream's D2H): 0.97 (fp32) / 0.90 (int8) of the copy-only duplex
// ceiling of the same bytes (profiles/r04/a/bench.json.log, extras.c5).
//
// HPDCT_STREAM_PIPELINE=engines selects an A/B layout measured in round 4 and
// rejected: one in-order stream per engine (H2D copies, kernels, D2H copies)
// over a ring of nstreams device slots, ordered by per-slot events (H2D(f)
// after kernel(f - slots), kernel(f) after H2D(f) and D2H(f - slots), D2H(f)
// after kernel(f)).  It is bit-exact but ran at 213-440 fp32 / 1,580-1,630
// int8 frames/s against 784 / 2,542 for the product: on this ROCm the
// cross-stream event waits in front of every copy serialise the pipeline.
// Host buffers should be pinned (hipHostMalloc / torch pin_memory) for the
// copies to be asynchronous and overlap.
//
// The streams, device ring and timing events live in an hpdct_stream_ctx
// (hpdct_stream_create / _run / _destroy), so a caller that streams many
// batches pays their creation once; hpdct_stream_forward is the one-shot
// form (create, run, destroy).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "hpdct.h"
#include "hpdct_kernels.h"

struct hpdct_stream_ctx_s {
    int64_t height = 0, width = 0;
    hpdct_dtype out_type = HPDCT_F32;
    int device = -1;
    bool engines = false;             // A/B: one stream per engine over a slot ring (else one per slot)
    std::vector<hipStream_t> streams;  // engines: {H2D, kernels, D2H}; else one per slot
    std::vector<void*> in, out;        // the device ring, one pair per slot
    std::vector<hipEvent_t> done;      // streams layout: per stream, its last operation of a batch
    std::vector<hipEvent_t> loaded, computed, drained;  // engines layout: per slot
    hipEvent_t t0 = nullptr, t1 = nullptr;

    ~hpdct_stream_ctx_s() {
        for (void* p : in) (void)hipFree(p);
        for (void* p : out) (void)hipFree(p);
        for (hipEvent_t e : done) (void)hipEventDestroy(e);
        for (hipEvent_t e : loaded) (void)hipEventDestroy(e);
        for (hipEvent_t e : computed) (void)hipEventDestroy(e);
        for (hipEvent_t e : drained) (void)hipEventDestroy(e);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
        for (hipStream_t s : streams) (void)hipStreamDestroy(s);
    }
};

namespace {
hpdct_status fail(hpdct_status st, const std::string& msg) {
    return static_cast<hpdct_status>(hpdct::set_last_error(st, msg.c_str()));
}
hpdct_status device_fail(hipError_t e, const char* what) {
    return fail(HPDCT_ERROR_DEVICE, std::string("hpdct stream: ") + what + ": " + hipGetErrorString(e));
}

hpdct_status validate(int64_t height, int64_t width, hpdct_dtype out_type, int nstreams) {
    if (nstreams < 1 || nstreams > 16)
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct stream: nstreams must be in 1..16");
    if (out_type != HPDCT_F32 && out_type != HPDCT_I8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "hpdct stream: output must be HPDCT_F32 or HPDCT_I8");
    if (height <= 0 || width <= 0 || height % 8 || width % 8)
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct stream: height and width must be positive multiples of 8");
    return HPDCT_SUCCESS;
}

hpdct_status create(hpdct_stream_ctx* out_ctx, int64_t height, int64_t width, hpdct_dtype out_type, int nstreams) {
    if (!out_ctx) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_create: null handle pointer");
    *out_ctx = nullptr;
    if (hpdct_status st = validate(height, width, out_type, nstreams)) return st;
    hpdct_stream_ctx c = new (std::nothrow) hpdct_stream_ctx_s;
    if (!c) return fail(HPDCT_ERROR_DEVICE, "hpdct stream: out of host memory");
    c->height = height;
    c->width = width;
    c->out_type = out_type;
    const size_t px = static_cast<size_t>(height) * static_cast<size_t>(width);
    const size_t out_bytes = px * (out_type == HPDCT_F32 ? 4 : 1);
    const char* layout = getenv("HPDCT_STREAM_PIPELINE");
    c->engines = layout && strcmp(layout, "engines") == 0;
    hipError_t he = hipGetDevice(&c->device);
    if (c->engines) {
        for (int k = 0; k < 3 && he == hipSuccess; ++k) {
            hipStream_t st;
            if ((he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) == hipSuccess) c->streams.push_back(st);
        }
        for (int s = 0; s < nstreams && he == hipSuccess; ++s) {
            void *di = nullptr, *dout = nullptr;
            if ((he = hipMalloc(&di, px)) != hipSuccess) break;
            c->in.push_back(di);
            if ((he = hipMalloc(&dout, out_bytes)) != hipSuccess) break;
            c->out.push_back(dout);
            for (auto* v : {&c->loaded, &c->computed, &c->drained}) {
                hipEvent_t ev;
                if ((he = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) break;
                v->push_back(ev);
            }
        }
    }
    for (int s = 0; s < nstreams && he == hipSuccess && !c->engines; ++s) {
        hipStream_t st;
        void *di = nullptr, *dout = nullptr;
        hipEvent_t ev;
        if ((he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) break;
        c->streams.push_back(st);
        if ((he = hipMalloc(&di, px)) != hipSuccess) break;
        c->in.push_back(di);
        if ((he = hipMalloc(&dout, out_bytes)) != hipSuccess) break;
        c->out.push_back(dout);
        if ((he = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) break;
        c->done.push_back(ev);
    }
    if (he == hipSuccess) he = hipEventCreate(&c->t0);
    if (he == hipSuccess) he = hipEventCreate(&c->t1);
    if (he != hipSuccess) {
        delete c;
        return device_fail(he, "creating the streams / device ring");
    }
    *out_ctx = c;
    return HPDCT_SUCCESS;
}

// the engines layout (see the file comment)
hpdct_status run_engines(hpdct_stream_ctx c, const uint8_t* const* h_frames, void* const* h_coef, int64_t n_frames,
                         float* elapsed_ms, size_t px, size_t out_bytes) {
    hipStream_t h2d = c->streams[0], comp = c->streams[1], d2h = c->streams[2];
    const int64_t slots = static_cast<int64_t>(c->in.size());
    hipError_t e = hipEventRecord(c->t0, h2d);
    if (e == hipSuccess) e = hipStreamWaitEvent(comp, c->t0, 0);
    if (e == hipSuccess) e = hipStreamWaitEvent(d2h, c->t0, 0);
    for (int64_t f = 0; f < n_frames && e == hipSuccess; ++f) {
        const int64_t s = f % slots;
        const bool reuse = f >= slots;  // the slot held frame f - slots
        if (reuse) e = hipStreamWaitEvent(h2d, c->computed[s], 0);  // its input consumed
        if (e == hipSuccess) e = hipMemcpyAsync(c->in[s], h_frames[f], px, hipMemcpyHostToDevice, h2d);
        if (e == hipSuccess) e = hipEventRecord(c->loaded[s], h2d);
        if (e == hipSuccess) e = hipStreamWaitEvent(comp, c->loaded[s], 0);
        if (e == hipSuccess && reuse) e = hipStreamWaitEvent(comp, c->drained[s], 0);  // its output drained
        if (e != hipSuccess) break;
        const hpdct_status hs =
            hpdct_forward(c->in[s], HPDCT_U8, c->out[s], c->out_type, c->height, c->width, nullptr, 0u, comp);
        if (hs != HPDCT_SUCCESS) {
            for (hipStream_t x : c->streams) (void)hipStreamSynchronize(x);
            return hs;
        }
        e = hipEventRecord(c->computed[s], comp);
        if (e == hipSuccess) e = hipStreamWaitEvent(d2h, c->computed[s], 0);
        if (e == hipSuccess) e = hipMemcpyAsync(h_coef[f], c->out[s], out_bytes, hipMemcpyDeviceToHost, d2h);
        if (e == hipSuccess) e = hipEventRecord(c->drained[s], d2h);
    }
    // the last D2H is the batch's last operation (D2H copies are in frame order)
    if (e == hipSuccess) e = hipEventRecord(c->t1, d2h);
    if (e == hipSuccess) e = hipEventSynchronize(c->t1);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->t0, c->t1);
    for (hipStream_t st : c->streams) (void)hipStreamSynchronize(st);
    if (e != hipSuccess) return device_fail(e, "copy/compute pipeline");
    if (elapsed_ms) *elapsed_ms = ms;
    return HPDCT_SUCCESS;
}

hpdct_status run(hpdct_stream_ctx c, const uint8_t* const* h_frames, void* const* h_coef, int64_t n_frames,
                 float* elapsed_ms) {
    if (!c) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_run: null context");
    if (!h_frames || !h_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct stream: null frame list");
    if (n_frames < 0) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct stream: negative frame count");
    for (int64_t f = 0; f < n_frames; ++f)
        if (!h_frames[f] || !h_coef[f])
            return fail(HPDCT_ERROR_INVALID_VALUE,
                        "hpdct stream: null frame or output pointer at index " + std::to_string(f));
    if (n_frames == 0) {
        if (elapsed_ms) *elapsed_ms = 0.0f;
        return HPDCT_SUCCESS;
    }
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != c->device)
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_run: the context belongs to device " +
                                                   std::to_string(c->device) + ", the current device is " +
                                                   std::to_string(cur));
    const int64_t height = c->height, width = c->width;
    const size_t px = static_cast<size_t>(height) * static_cast<size_t>(width);
    const size_t out_bytes = px * (c->out_type == HPDCT_F32 ? 4 : 1);
    if (c->engines) return run_engines(c, h_frames, h_coef, n_frames, elapsed_ms, px, out_bytes);
    const int nstreams = static_cast<int>(c->streams.size());
    // start marker: every stream waits for it, so the timed region holds the whole batch
    hipError_t e = hipEventRecord(c->t0, c->streams[0]);
    for (int s = 1; s < nstreams && e == hipSuccess; ++s) e = hipStreamWaitEvent(c->streams[s], c->t0, 0);
    for (int64_t f = 0; f < n_frames && e == hipSuccess; ++f) {
        const int s = static_cast<int>(f % nstreams);
        hipStream_t st = c->streams[s];
        // staggered start (round 6): stream s's first upload waits for stream
        // s-1's, so the streams run out of phase and one stream's D2H copy
        // overlaps the next one's H2D copy from the first frame on.  Started
        // together they ran in step (all uploads, then all downloads) unless
        // they happened to drift apart: int8 C5 0.70-0.91 of the copy-only
        // duplex ceiling from box to box (BENCH_r05 extras.c5, profiles/r06/)
        if (f > 0 && f < nstreams) e = hipStreamWaitEvent(st, c->done[s - 1], 0);
        if (e == hipSuccess) e = hipMemcpyAsync(c->in[s], h_frames[f], px, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && f + 1 < nstreams && f + 1 < n_frames) e = hipEventRecord(c->done[s], st);
        if (e != hipSuccess) break;
        const hpdct_status hs =
            hpdct_forward(c->in[s], HPDCT_U8, c->out[s], c->out_type, height, width, nullptr, 0u, st);
        if (hs != HPDCT_SUCCESS) {
            for (hipStream_t x : c->streams) (void)hipStreamSynchronize(x);
            return hs;
        }
        e = hipMemcpyAsync(h_coef[f], c->out[s], out_bytes, hipMemcpyDeviceToHost, st);
    }
    // end marker after every stream's last operation
    for (int s = 1; s < nstreams && e == hipSuccess; ++s) {
        e = hipEventRecord(c->done[s], c->streams[s]);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->streams[0], c->done[s], 0);
    }
    if (e == hipSuccess) e = hipEventRecord(c->t1, c->streams[0]);
    if (e == hipSuccess) e = hipEventSynchronize(c->t1);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->t0, c->t1);
    for (hipStream_t st : c->streams) (void)hipStreamSynchronize(st);
    if (e != hipSuccess) return device_fail(e, "copy/compute pipeline");
    if (elapsed_ms) *elapsed_ms = ms;
    return HPDCT_SUCCESS;
}

// no C++ exception may cross the C ABI
template <typename F>
hpdct_status guarded(const char* what, F&& f) {
    try {
        return f();
    } catch (const std::exception& ex) {
        return fail(HPDCT_ERROR_DEVICE, std::string(what) + ": " + ex.what());
    } catch (...) {
        return fail(HPDCT_ERROR_DEVICE, std::string(what) + ": host exception");
    }
}
}  // namespace

extern "C" {

hpdct_status hpdct_stream_create(hpdct_stream_ctx* ctx, int64_t height, int64_t width, hpdct_dtype out_type,
                                 int nstreams) {
    return guarded("hpdct_stream_create", [&] { return create(ctx, height, width, out_type, nstreams); });
}

hpdct_status hpdct_stream_run(hpdct_stream_ctx ctx, const uint8_t* const* h_frames, void* const* h_coef,
                              int64_t n_frames, float* elapsed_ms) {
    return guarded("hpdct_stream_run", [&] { return run(ctx, h_frames, h_coef, n_frames, elapsed_ms); });
}

hpdct_status hpdct_stream_destroy(hpdct_stream_ctx ctx) {
    delete ctx;  // run() leaves every stream idle, so the ring is free to go
    return HPDCT_SUCCESS;
}

hpdct_status hpdct_stream_forward(const uint8_t* const* h_frames, void* const* h_coef, int64_t n_frames,
                                  int64_t height, int64_t width, hpdct_dtype out_type, int nstreams,
                                  float* elapsed_ms) {
    if (!h_frames || !h_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: null frame list");
    if (n_frames < 0) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_stream_forward: negative frame count");
    if (hpdct_status st = validate(height, width, out_type, nstreams)) return st;
    for (int64_t f = 0; f < n_frames; ++f)
        if (!h_frames[f] || !h_coef[f])
            return fail(HPDCT_ERROR_INVALID_VALUE,
                        "hpdct_stream_forward: null frame or output pointer at index " + std::to_string(f));
    if (n_frames == 0) {  // nothing to stream: no device resources either
        if (elapsed_ms) *elapsed_ms = 0.0f;
        return HPDCT_SUCCESS;
    }
    hpdct_stream_ctx c = nullptr;
    if (hpdct_status st = hpdct_stream_create(&c, height, width, out_type, nstreams)) return st;
    const hpdct_status st = hpdct_stream_run(c, h_frames, h_coef, n_frames, elapsed_ms);
    hpdct_stream_destroy(c);
    return st;
}

}  // extern "C"
