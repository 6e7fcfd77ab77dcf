// hpdct_api.cpp -- the extern "C" boundary (include/hpdct.h): validation,
// library-owned quantisation table, dispatch to the gfx950 kernels.
// No torch types, no CPU fallback: every compute entry point launches a HIP
// kernel or returns an error.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

#include "hpdct.h"
#include "hpdct_kernels.h"
#include "hpdct_tables.h"

#define HPDCT_VERSION_STRING "hpdct 0.1.0 (gfx950)"

namespace {

using hpdct::Mat64;
using hpdct::QParams;
using hpdct::TileGrid;
using hpdct::FrameTable;
using hpdct::kMaxFramesPerLaunch;
using hpdct::launch_fdct_frames;

// JPEG luminance table and the HpApprDCT matrix (main_newAppr.cu:60-81): the
// same constexpr arrays the kernels compile into immediates (hpdct_tables.h).
constexpr const float (&kDefaultQ)[64] = hpdct::tables::kQ;
constexpr const float (&kDefaultT)[64] = hpdct::tables::kT;

// hpdct_mapping in force: -1 = not yet read from HPDCT_MAPPING.
std::atomic<int> g_mapping{-1};

int mapping_from_env() {
    const char* e = getenv("HPDCT_MAPPING");
    if (!e || !*e || strcmp(e, "auto") == 0) return HPDCT_MAPPING_AUTO;
    if (strcmp(e, "tile") == 0) return HPDCT_MAPPING_TILE;
    if (strcmp(e, "octet") == 0) return HPDCT_MAPPING_OCTET;
    if (strcmp(e, "duo") == 0) return HPDCT_MAPPING_DUO;
    fprintf(stderr, "hpdct: ignoring HPDCT_MAPPING=%s (expected auto, tile, octet or duo)\n", e);
    return HPDCT_MAPPING_AUTO;
}


thread_local std::string g_last_error;

hpdct_status fail(hpdct_status st, const std::string& msg) {
    g_last_error = msg;
    return st;
}

}  // namespace

int hpdct::set_last_error(int st, const char* msg) {
    g_last_error = msg ? msg : "";
    return st;
}

namespace {

hpdct_status device_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return HPDCT_SUCCESS;
    return fail(HPDCT_ERROR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// max |q| the forward quantiser can produce for uint8 input with the built-in T:
// |C[v][u]| <= 128 * ||T_v||_1 * ||T_u||_1 (plus fp rounding), q = round(C/Q).
bool int8_safe(const Mat64& q) {
    double n1[8];
    for (int r = 0; r < 8; ++r) {
        n1[r] = 0.0;
        for (int i = 0; i < 8; ++i) n1[r] += std::fabs((double)kDefaultT[r * 8 + i]);
    }
    for (int v = 0; v < 8; ++v)
        for (int u = 0; u < 8; ++u) {
            const double cmax = 128.0 * n1[v] * n1[u] * (1.0 + 1e-5);
            if (std::floor(cmax / std::fabs((double)q.v[v * 8 + u]) + 0.5) > 127.0) return false;
        }
    return true;
}

hpdct_status make_grid(int64_t height, int64_t width, TileGrid& g) {
    if (height <= 0 || width <= 0 || (height % 8) != 0 || (width % 8) != 0)
        return fail(HPDCT_ERROR_INVALID_VALUE, "height and width must be positive multiples of 8 (got " +
                                                   std::to_string(height) + "x" + std::to_string(width) + ")");
    const int64_t tiles = (height / 8) * (width / 8);
    if (tiles >= (int64_t(1) << 32) || (width / 8) >= (int64_t(1) << 32))
        return fail(HPDCT_ERROR_INVALID_VALUE, "image too large: tile count must be < 2^32");
    g.ntiles = static_cast<uint32_t>(tiles);
    g.tiles_x = static_cast<uint32_t>(width / 8);
    g.width = static_cast<uint64_t>(width);
    return HPDCT_SUCCESS;
}

// The 3-operation quotient of the kernels gives the same roundf() as IEEE
// C/Q for every |C| <= 4096 when Q is an integer in 1..255 (exhaustive on the
// GPU: tests/tools/verify_fastdiv.hip, log in tests/tools/verify_fastdiv.gpu.log;
// CPU cross-check for the JPEG table: tests/tools/verify_fastdiv.c).
bool fastdiv_table(const Mat64& q) {
    for (float v : q.v)
        if (!(v >= 1.0f && v <= 255.0f) || v != std::floor(v)) return false;
    return true;
}

QParams make_qparams(const Mat64& q) {
    QParams p;
    p.q = q;
    for (int i = 0; i < 64; ++i) p.r.v[i] = 1.0f / q.v[i];  // RN(1/Q), as the verification tools compute it
    return p;
}

// The library-owned quantiser: the table, its reciprocals and the two
// properties the launches need, computed once per hpdct_set_quant_table
// (not per call) and copied out under the mutex.
struct QState {
    QParams qp;
    bool fastdiv_ok;  // integers in 1..255: the verified 3-op quotient is exact
    bool int8_ok;     // |q| <= 127 for uint8 input with the built-in T
};

QState make_qstate(const Mat64& q) { return QState{make_qparams(q), fastdiv_table(q), int8_safe(q)}; }

std::mutex g_q_mutex;
QState g_qs = [] {
    Mat64 m;
    memcpy(m.v, kDefaultQ, sizeof(m.v));
    return make_qstate(m);
}();

QState current_qstate() {
    std::lock_guard<std::mutex> lk(g_q_mutex);
    return g_qs;
}

bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }
uintptr_t row_align(hpdct_dtype t) { return t == HPDCT_F32 ? 16 : 8; }
size_t elem_size(hpdct_dtype t) { return t == HPDCT_F32 ? 4 : 1; }

}  // namespace

extern "C" {

const char* hpdct_version(void) { return HPDCT_VERSION_STRING; }

const char* hpdct_status_string(hpdct_status s) {
    switch (s) {
        case HPDCT_SUCCESS: return "success";
        case HPDCT_ERROR_INVALID_VALUE: return "invalid value";
        case HPDCT_ERROR_UNSUPPORTED: return "unsupported dtype/flag combination";
        case HPDCT_ERROR_RANGE: return "quantised values can overflow int8 with this table";
        case HPDCT_ERROR_DEVICE: return "HIP runtime error";
    }
    return "unknown status";
}

const char* hpdct_last_error_string(void) { return g_last_error.c_str(); }

hpdct_status hpdct_set_mapping(hpdct_mapping mapping) {
    if (mapping != HPDCT_MAPPING_AUTO && mapping != HPDCT_MAPPING_TILE && mapping != HPDCT_MAPPING_OCTET &&
        mapping != HPDCT_MAPPING_DUO)
        return HPDCT_ERROR_INVALID_VALUE;
    g_mapping.store(static_cast<int>(mapping));
    return HPDCT_SUCCESS;
}

hpdct_mapping hpdct_get_mapping(void) { return static_cast<hpdct_mapping>(hpdct::mapping_mode()); }

void hpdct_default_quant_table(float* q64) {
    if (q64) memcpy(q64, kDefaultQ, sizeof(kDefaultQ));
}
void hpdct_default_transform(float* t64) {
    if (t64) memcpy(t64, kDefaultT, sizeof(kDefaultT));
}

hpdct_status hpdct_set_quant_table(const float* q64) {
    Mat64 m;
    if (!q64) {
        memcpy(m.v, kDefaultQ, sizeof(m.v));
    } else {
        for (int i = 0; i < 64; ++i)
            if (!std::isfinite(q64[i]) || q64[i] == 0.0f)
                return fail(HPDCT_ERROR_INVALID_VALUE, "quant table entries must be finite and non-zero");
        memcpy(m.v, q64, sizeof(m.v));
    }
    const QState qs = make_qstate(m);
    std::lock_guard<std::mutex> lk(g_q_mutex);
    g_qs = qs;
    return HPDCT_SUCCESS;
}

hpdct_status hpdct_get_quant_table(float* q64) {
    if (!q64) return fail(HPDCT_ERROR_INVALID_VALUE, "null output pointer");
    const QState qs = current_qstate();
    memcpy(q64, qs.qp.q.v, sizeof(qs.qp.q.v));
    return HPDCT_SUCCESS;
}

hpdct_status hpdct_forward(const void* d_image, hpdct_dtype in_type, void* d_coef, hpdct_dtype out_type,
                           int64_t height, int64_t width, const float* d_transform, unsigned flags, void* stream) {
    TileGrid g;
    if (hpdct_status st = make_grid(height, width, g)) return st;
    if (!d_image || !d_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "null image or coefficient pointer");
    if (flags & ~(HPDCT_FLAG_NO_QUANT | HPDCT_FLAG_WRITEBACK_SHIFT | HPDCT_FLAG_NO_SHIFT | HPDCT_FLAG_ROW_FIRST))
        return fail(HPDCT_ERROR_UNSUPPORTED, "unknown or inverse-only flag bits");
    if (in_type != HPDCT_U8 && in_type != HPDCT_F32)
        return fail(HPDCT_ERROR_UNSUPPORTED, "forward input must be HPDCT_U8 or HPDCT_F32");
    if (out_type != HPDCT_F32 && out_type != HPDCT_I8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "forward output must be HPDCT_F32 or HPDCT_I8");
    const bool quant = !(flags & HPDCT_FLAG_NO_QUANT);
    const bool wb = (flags & HPDCT_FLAG_WRITEBACK_SHIFT) != 0;
    const float shift = (flags & HPDCT_FLAG_NO_SHIFT) ? 0.0f : 128.0f;
    if (wb && in_type != HPDCT_F32)
        return fail(HPDCT_ERROR_UNSUPPORTED, "HPDCT_FLAG_WRITEBACK_SHIFT needs an fp32 input");
    const bool row_first = (flags & HPDCT_FLAG_ROW_FIRST) != 0;
    if (row_first && (in_type != HPDCT_F32 || out_type != HPDCT_F32))
        return fail(HPDCT_ERROR_UNSUPPORTED, "HPDCT_FLAG_ROW_FIRST is the fp32 -> fp32 (cublasDCTv2) path");
    if (out_type == HPDCT_I8) {
        if (!quant) return fail(HPDCT_ERROR_UNSUPPORTED, "int8 output needs quantisation");
        if (in_type != HPDCT_U8 || d_transform || shift != 128.0f)
            return fail(HPDCT_ERROR_UNSUPPORTED, "int8 output needs uint8 input, the built-in T and the level shift");
    }
    if (!aligned(d_image, row_align(in_type)) || !aligned(d_coef, row_align(out_type)))
        return fail(HPDCT_ERROR_INVALID_VALUE, "device pointers must be 16-byte (fp32) / 8-byte (8-bit) aligned");
    const size_t in_bytes = static_cast<size_t>(height) * width * elem_size(in_type);
    const char* ib = static_cast<const char*>(d_image);
    const char* ob = static_cast<const char*>(d_coef);
    const size_t out_bytes = static_cast<size_t>(height) * width * elem_size(out_type);
    if (ib < ob + out_bytes && ob < ib + in_bytes)
        return fail(HPDCT_ERROR_INVALID_VALUE, "image and coefficient buffers overlap");
    const QState qs = current_qstate();
    if (out_type == HPDCT_I8 && !qs.int8_ok)
        return fail(HPDCT_ERROR_RANGE, "current quant table can produce |q| > 127: use fp32 output");
    const QParams& qp = qs.qp;
    // |C| <= 8*255 for uint8 input with the built-in T, well inside the verified |C| <= 4096;
    // fp32 input (any T) takes it row by row behind a range test (kVarFastDivChecked, duo kernels)
    const bool fastdiv = quant && qs.fastdiv_ok && ((in_type == HPDCT_U8 && d_transform == nullptr) || in_type == HPDCT_F32);

    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool bt = d_transform == nullptr;
    hipError_t e = hipSuccess;
    using namespace hpdct;
#define FWD(TI, TO, QN, WB)                                                                                        \
    e = bt ? launch_fdct<TI, TO, QN, true, WB>(static_cast<const TI*>(d_image), static_cast<TO*>(d_coef),         \
                                               static_cast<float*>(const_cast<void*>(d_image)), g, d_transform,    \
                                               qp, shift, fastdiv, row_first, s)                                   \
           : launch_fdct<TI, TO, QN, false, WB>(static_cast<const TI*>(d_image), static_cast<TO*>(d_coef),        \
                                                static_cast<float*>(const_cast<void*>(d_image)), g, d_transform,   \
                                                qp, shift, fastdiv, row_first, s)
    if (in_type == HPDCT_U8) {
        if (out_type == HPDCT_I8) {
            FWD(uint8_t, int8_t, true, false);
        } else if (quant) {
            FWD(uint8_t, float, true, false);
        } else {
            FWD(uint8_t, float, false, false);
        }
    } else {
        if (quant && wb) {
            FWD(float, float, true, true);
        } else if (quant) {
            FWD(float, float, true, false);
        } else if (wb) {
            FWD(float, float, false, true);
        } else {
            FWD(float, float, false, false);
        }
    }
#undef FWD
    return device_status(e, "forward kernel launch");
}

}  // extern "C"

namespace {
hpdct_status forward_frames(const uint8_t* const* d_images, void* const* d_coefs, hpdct_dtype out_type,
                            int64_t n_frames, int64_t height, int64_t width, void* stream) {
    TileGrid g;
    if (hpdct_status st = make_grid(height, width, g)) return st;
    if (n_frames < 0) return fail(HPDCT_ERROR_INVALID_VALUE, "negative frame count");
    if (n_frames == 0) return HPDCT_SUCCESS;
    if (!d_images || !d_coefs) return fail(HPDCT_ERROR_INVALID_VALUE, "null frame or coefficient pointer table");
    if (out_type != HPDCT_F32 && out_type != HPDCT_I8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "frame-list output must be HPDCT_F32 or HPDCT_I8");
    const size_t in_bytes = static_cast<size_t>(height) * width;
    const size_t out_bytes = in_bytes * elem_size(out_type);
    // every plane as a byte interval; a coefficient plane may overlap nothing
    struct Span {
        uintptr_t a, b;
        bool write;
    };
    std::vector<Span> spans;
    spans.reserve(static_cast<size_t>(n_frames) * 2);
    for (int64_t f = 0; f < n_frames; ++f) {
        if (!d_images[f] || !d_coefs[f])
            return fail(HPDCT_ERROR_INVALID_VALUE, "null device pointer for frame " + std::to_string(f));
        if (!aligned(d_images[f], 8) || !aligned(d_coefs[f], row_align(out_type)))
            return fail(HPDCT_ERROR_INVALID_VALUE, "frame " + std::to_string(f) +
                                                       ": device pointers must be 8-byte (uint8 / int8) / "
                                                       "16-byte (fp32) aligned");
        const uintptr_t i = reinterpret_cast<uintptr_t>(d_images[f]), o = reinterpret_cast<uintptr_t>(d_coefs[f]);
        spans.push_back({i, i + in_bytes, false});
        spans.push_back({o, o + out_bytes, true});
    }
    // one sweep in start order (O(n log n); input planes may repeat, so a
    // pairwise scan would be quadratic): a span conflicts if a write span
    // seen before ends after its start, or if it writes and any span seen
    // before ends after its start
    std::sort(spans.begin(), spans.end(), [](const Span& x, const Span& y) { return x.a < y.a; });
    uintptr_t end_all = 0, end_write = 0;
    for (const Span& sp : spans) {
        if (sp.a < end_write || (sp.write && sp.a < end_all))
            return fail(HPDCT_ERROR_INVALID_VALUE, "a coefficient plane overlaps another frame's plane");
        end_all = std::max(end_all, sp.b);
        if (sp.write) end_write = std::max(end_write, sp.b);
    }
    const QState qs = current_qstate();
    if (out_type == HPDCT_I8 && !qs.int8_ok)
        return fail(HPDCT_ERROR_RANGE, "current quant table can produce |q| > 127: use fp32 output");
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int64_t f0 = 0; f0 < n_frames; f0 += kMaxFramesPerLaunch) {
        const int n = static_cast<int>(std::min<int64_t>(kMaxFramesPerLaunch, n_frames - f0));
        hipError_t e;
        if (out_type == HPDCT_F32) {
            FrameTable<float> ft{};
            for (int k = 0; k < n; ++k) {
                ft.in[k] = d_images[f0 + k];
                ft.out[k] = static_cast<float*>(d_coefs[f0 + k]);
            }
            e = launch_fdct_frames<float>(ft, n, g, qs.qp, qs.fastdiv_ok, s);
        } else {
            FrameTable<int8_t> ft{};
            for (int k = 0; k < n; ++k) {
                ft.in[k] = d_images[f0 + k];
                ft.out[k] = static_cast<int8_t*>(d_coefs[f0 + k]);
            }
            e = launch_fdct_frames<int8_t>(ft, n, g, qs.qp, qs.fastdiv_ok, s);
        }
        if (e != hipSuccess) return device_status(e, "frame-list forward launch");
    }
    return HPDCT_SUCCESS;
}
}  // namespace

extern "C" {

// no C++ exception may cross the C ABI: a garbage n_frames makes the span
// table's allocation throw, which becomes a status here
hpdct_status hpdct_forward_frames(const uint8_t* const* d_images, void* const* d_coefs, hpdct_dtype out_type,
                                  int64_t n_frames, int64_t height, int64_t width, void* stream) {
    try {
        return forward_frames(d_images, d_coefs, out_type, n_frames, height, width, stream);
    } catch (const std::exception& e) {
        return fail(HPDCT_ERROR_INVALID_VALUE, std::string("hpdct_forward_frames: ") + e.what());
    } catch (...) {
        return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_forward_frames: host exception");
    }
}

hpdct_status hpdct_inverse(const void* d_coef, hpdct_dtype in_type, void* d_image, hpdct_dtype out_type,
                           int64_t height, int64_t width, const float* d_transform, unsigned flags, void* stream) {
    TileGrid g;
    if (hpdct_status st = make_grid(height, width, g)) return st;
    if (!d_image || !d_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "null image or coefficient pointer");
    if (flags & ~(HPDCT_FLAG_NO_QUANT | HPDCT_FLAG_NO_SHIFT | HPDCT_FLAG_ROW_FIRST | HPDCT_FLAG_WRITEBACK_DEQUANT))
        return fail(HPDCT_ERROR_UNSUPPORTED, "unknown or forward-only flag bits");
    if (in_type != HPDCT_F32 && in_type != HPDCT_I8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "inverse input must be HPDCT_F32 or HPDCT_I8");
    if (out_type != HPDCT_F32 && out_type != HPDCT_U8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "inverse output must be HPDCT_F32 or HPDCT_U8");
    if (!aligned(d_image, row_align(out_type)) || !aligned(d_coef, row_align(in_type)))
        return fail(HPDCT_ERROR_INVALID_VALUE, "device pointers must be 16-byte (fp32) / 8-byte (8-bit) aligned");
    const size_t in_bytes = static_cast<size_t>(height) * width * elem_size(in_type);
    const size_t out_bytes = static_cast<size_t>(height) * width * elem_size(out_type);
    const char* ib = static_cast<const char*>(d_coef);
    const char* ob = static_cast<const char*>(d_image);
    if (ib < ob + out_bytes && ob < ib + in_bytes)
        return fail(HPDCT_ERROR_INVALID_VALUE, "coefficient and image buffers overlap");
    const bool deq = !(flags & HPDCT_FLAG_NO_QUANT);
    const float shift = (flags & HPDCT_FLAG_NO_SHIFT) ? 0.0f : 128.0f;
    const bool row_first = (flags & HPDCT_FLAG_ROW_FIRST) != 0;
    const bool wb = (flags & HPDCT_FLAG_WRITEBACK_DEQUANT) != 0;
    if ((row_first || wb) && (in_type != HPDCT_F32 || out_type != HPDCT_F32))
        return fail(HPDCT_ERROR_UNSUPPORTED, "ROW_FIRST / WRITEBACK_DEQUANT are fp32 -> fp32 (cublasDCTv2) options");
    if (wb && !deq) return fail(HPDCT_ERROR_UNSUPPORTED, "HPDCT_FLAG_WRITEBACK_DEQUANT needs dequantisation");
    float* dq_out = wb ? static_cast<float*>(const_cast<void*>(d_coef)) : nullptr;
    const Mat64 q = current_qstate().qp.q;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool bt = d_transform == nullptr;
    hipError_t e = hipSuccess;
    using namespace hpdct;
#define INV(TI, TO, DQ)                                                                                           \
    e = bt ? launch_idct<TI, TO, DQ, true>(static_cast<const TI*>(d_coef), static_cast<TO*>(d_image), dq_out, g, \
                                           d_transform, q, shift, row_first, s)                                  \
           : launch_idct<TI, TO, DQ, false>(static_cast<const TI*>(d_coef), static_cast<TO*>(d_image), dq_out, g,\
                                            d_transform, q, shift, row_first, s)
#define INV_Q(TI, TO)          \
    if (deq) {                 \
        INV(TI, TO, true);     \
    } else {                   \
        INV(TI, TO, false);    \
    }
    if (in_type == HPDCT_F32) {
        if (out_type == HPDCT_F32) {
            INV_Q(float, float)
        } else {
            INV_Q(float, uint8_t)
        }
    } else {
        if (out_type == HPDCT_F32) {
            INV_Q(int8_t, float)
        } else {
            INV_Q(int8_t, uint8_t)
        }
    }
#undef INV_Q
#undef INV
    return device_status(e, "inverse kernel launch");
}

namespace {
hpdct_status roundtrip(const uint8_t* d_image, float* d_coef, void* d_recon, hpdct_dtype recon_type,
                       hpdct_roundtrip_sums* d_sums, int64_t height, int64_t width, void* stream, bool zero_sums) {
    static_assert(sizeof(hpdct_roundtrip_sums) == sizeof(hpdct::RtSums), "hpdct_roundtrip_sums layout");
    TileGrid g;
    if (hpdct_status st = make_grid(height, width, g)) return st;
    if (!d_image || !d_coef) return fail(HPDCT_ERROR_INVALID_VALUE, "null image or coefficient pointer");
    if (d_recon && recon_type != HPDCT_U8 && recon_type != HPDCT_F32)
        return fail(HPDCT_ERROR_UNSUPPORTED, "reconstruction must be HPDCT_U8 or HPDCT_F32");
    if (!aligned(d_image, 8) || !aligned(d_coef, 16) || (d_recon && !aligned(d_recon, row_align(recon_type))) ||
        (d_sums && !aligned(d_sums, 8)))
        return fail(HPDCT_ERROR_INVALID_VALUE,
                    "device pointers must be 16-byte (fp32) / 8-byte (8-bit planes, sums) aligned");
    const size_t px = static_cast<size_t>(height) * width;
    struct Span {
        const char* p;
        size_t n;
    };
    const Span spans[4] = {{static_cast<const char*>(static_cast<const void*>(d_image)), px},
                           {reinterpret_cast<const char*>(d_coef), px * 4},
                           {static_cast<const char*>(d_recon), d_recon ? px * elem_size(recon_type) : 0},
                           {reinterpret_cast<const char*>(d_sums), d_sums ? sizeof(hpdct_roundtrip_sums) : 0}};
    for (int a = 0; a < 4; ++a)
        for (int b = a + 1; b < 4; ++b)
            if (spans[a].n && spans[b].n && spans[a].p < spans[b].p + spans[b].n &&
                spans[b].p < spans[a].p + spans[a].n)
                return fail(HPDCT_ERROR_INVALID_VALUE, "image, coefficient, reconstruction and sums buffers overlap");
    const QState qs = current_qstate();
    // packed int8 rows + the verified quotient when both properties hold, else
    // IEEE division with the rows kept in fp32 (any finite non-zero table)
    const bool fast = qs.fastdiv_ok && qs.int8_ok;
    const int kind = !d_recon ? hpdct::kRtReconNone : recon_type == HPDCT_U8 ? hpdct::kRtReconU8 : hpdct::kRtReconF32;
    return device_status(hpdct::launch_roundtrip(d_image, d_coef, d_recon, kind,
                                                 reinterpret_cast<hpdct::RtSums*>(d_sums), g, qs.qp, fast, zero_sums,
                                                 static_cast<hipStream_t>(stream)),
                         "round-trip kernel launch");
}
}  // namespace

hpdct_status hpdct_roundtrip_u8(const uint8_t* d_image, float* d_coef, void* d_recon, hpdct_dtype recon_type,
                                hpdct_roundtrip_sums* d_sums, int64_t height, int64_t width, void* stream) {
    return roundtrip(d_image, d_coef, d_recon, recon_type, d_sums, height, width, stream, true);
}

hpdct_status hpdct_roundtrip_u8_accumulate(const uint8_t* d_image, float* d_coef, void* d_recon,
                                           hpdct_dtype recon_type, hpdct_roundtrip_sums* d_sums, int64_t height,
                                           int64_t width, void* stream) {
    if (!d_sums) return fail(HPDCT_ERROR_INVALID_VALUE, "hpdct_roundtrip_u8_accumulate needs the sums struct");
    return roundtrip(d_image, d_coef, d_recon, recon_type, d_sums, height, width, stream, false);
}

hpdct_status hpdct_forward_u8_f32(const uint8_t* d_image, float* d_coef, int64_t height, int64_t width,
                                  void* stream) {
    return hpdct_forward(d_image, HPDCT_U8, d_coef, HPDCT_F32, height, width, nullptr, 0u, stream);
}
hpdct_status hpdct_forward_u8_i8(const uint8_t* d_image, int8_t* d_coef, int64_t height, int64_t width,
                                 void* stream) {
    return hpdct_forward(d_image, HPDCT_U8, d_coef, HPDCT_I8, height, width, nullptr, 0u, stream);
}
hpdct_status hpdct_inverse_f32_f32(const float* d_coef, float* d_image, int64_t height, int64_t width,
                                   void* stream) {
    return hpdct_inverse(d_coef, HPDCT_F32, d_image, HPDCT_F32, height, width, nullptr, 0u, stream);
}

hpdct_status hpdct_fill_hash_u8(uint8_t* d_out, int64_t n, uint64_t seed, int64_t first_index, void* stream) {
    if (!d_out || n < 0 || first_index < 0) return fail(HPDCT_ERROR_INVALID_VALUE, "bad fill arguments");
    if (!aligned(d_out, 16)) return fail(HPDCT_ERROR_INVALID_VALUE, "fill target must be 16-byte aligned");
    if (n == 0) return HPDCT_SUCCESS;
    return device_status(hpdct::launch_fill_hash(d_out, static_cast<uint64_t>(n), seed,
                                                 static_cast<uint64_t>(first_index), static_cast<hipStream_t>(stream)),
                         "fill kernel launch");
}

// glibc rand() after srand(seed) (benchmark_newAppr.cu:46-51), via the
// reentrant random_r family so the caller's rand() state is untouched.
void hpdct_fill_rand_u8(uint8_t* h_out, int64_t n, uint32_t seed) {
    struct random_data rd;
    char statebuf[128];
    memset(&rd, 0, sizeof(rd));
    initstate_r(seed, statebuf, sizeof(statebuf), &rd);
    srandom_r(seed, &rd);
    for (int64_t i = 0; i < n; ++i) {
        int32_t r;
        random_r(&rd, &r);
        h_out[i] = static_cast<uint8_t>(r % 256);
    }
}

// convertToFloat (utils.cu:10-15)
void hpdct_u8_to_f32(const uint8_t* h_in, float* h_out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) h_out[i] = static_cast<float>(h_in[i]);
}
// convertToUnsignedChar (utils.cu:18-24): clamp then truncate
void hpdct_f32_to_u8(const float* h_in, uint8_t* h_out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) h_out[i] = static_cast<uint8_t>(fminf(fmaxf(h_in[i], 0.0f), 255.0f));
}

}  // extern "C"

int hpdct::mapping_mode() {
    int m = g_mapping.load(std::memory_order_relaxed);
    if (m < 0) {
        int expected = -1;
        g_mapping.compare_exchange_strong(expected, mapping_from_env());
        m = g_mapping.load();
    }
    return m;
}
