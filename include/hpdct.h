/*
 * hpdct.h -- native C-ABI of the MI355X (gfx950) 8x8 block DCT/IDCT +
 * quantisation path (HpApprDCT arithmetic).  Library: libhpdct.so
 * (cuda-dct-idct_amd/lib/).
 *
 * Every entry point takes plain device pointers, 64-bit sizes and an optional
 * HIP stream (hipStream_t passed as void*; NULL = the null stream), returns a
 * status code and never exits the process.  The reference's own C++ entry
 * points (dct_all_blocks_cuda / idct_all_blocks_cuda, with their
 * print-and-exit semantics) are in hpdct_compat.h and are implemented on top
 * of these.
 *
 * Reference interface each function replaces (file:line into the reference,
 * GerryDps/CUDA-DCT-IDCT):
 *   hpdct_forward          dct_all_blocks_cuda      main_newAppr.cu:252-291
 *                          (sub_matrix_scalar -> cuda_matrix_dct ->
 *                          divide_matrices fused into one pass)
 *   hpdct_inverse          idct_all_blocks_cuda     main_newAppr.cu:293-332
 *                          (multiply_matrices -> cuda_matrix_idct ->
 *                          add_matrix_scalar fused into one pass)
 *   hpdct_roundtrip_u8     dct_all_blocks_cuda then idct_all_blocks_cuda
 *                          (main_newAppr.cu:99,120) and the host-side
 *                          PEEN/MSE of README.md:62-69, in one pass
 *   hpdct_forward(..., HPDCT_FLAG_ROW_FIRST)  dct_all_blocks  main_cublass_2.cu:197-252
 *   hpdct_inverse(..., HPDCT_FLAG_ROW_FIRST)  idct_all_blocks main_cublass_2.cu:257-311
 *   hpdct_set_quant_table  cudaMemcpyToSymbol(const_quant_matrix, ...)
 *                          main_newAppr.cu:19,70 (Q is library-owned here)
 *   hpdct_default_*        the Q and T tables of main_newAppr.cu:60-81
 *   hpdct_fill_rand_u8     not a device op in the reference: the synthetic
 *   (host)                 input of benchmark_newAppr.cu:46-51
 *                          (srand(42); rand()%256), restated
 *   hpdct_u8_from_f32 ... host conversions utils.cu:10-24
 *
 * Layout: an image is `height` rows of `width` elements, row-major, densely
 * packed (row pitch == width elements).  Coefficients are written in the
 * reference's spatial layout: coefficient (v,u) of tile (by,bx) sits at
 * [(8*by + v) * width + 8*bx + u].  A batch of F frames of HxW stacked in
 * memory is the single image (F*H) x W: tiles never cross a frame boundary
 * when H is a multiple of 8.  height and width must be positive multiples of
 * 8 (the reference silently produces garbage otherwise; we refuse).
 */
#ifndef HPDCT_H
#define HPDCT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum hpdct_status {
    HPDCT_SUCCESS = 0,
    HPDCT_ERROR_INVALID_VALUE = 1, /* NULL pointer, size not a positive multiple of 8, too many tiles */
    HPDCT_ERROR_UNSUPPORTED = 2,   /* dtype / flag combination not provided */
    HPDCT_ERROR_RANGE = 3,         /* int8 coefficients requested but the quant table can overflow int8 */
    HPDCT_ERROR_DEVICE = 4         /* a HIP runtime call failed: see hpdct_last_error_string() */
} hpdct_status;

typedef enum hpdct_dtype {
    HPDCT_U8 = 0,  /* uint8 pixels (0..255)                                   */
    HPDCT_I8 = 1,  /* int8 quantised coefficients (wire format, |q| <= 127)   */
    HPDCT_F32 = 2  /* fp32 pixels or coefficients (the reference's only type) */
} hpdct_dtype;

/* Flags for hpdct_forward / hpdct_inverse. */
#define HPDCT_FLAG_NO_QUANT 0x1u       /* forward: skip /Q+round; inverse: skip xQ (raw coefficients) */
#define HPDCT_FLAG_WRITEBACK_SHIFT 0x2u /* forward, f32 input only: also store X-128 back into the
                                           input buffer, as the reference's in-place sub_matrix_scalar
                                           does (main_newAppr.cu:273) */
#define HPDCT_FLAG_NO_SHIFT 0x4u       /* skip the -128 / +128 level shift (diagnostics, round trips) */
#define HPDCT_FLAG_ROW_FIRST 0x8u      /* fp32 -> fp32 only: cublasDCTv2 pass order (main_cublass_2.cu:228-235,
                                          288-295): the row pass X.T^T (D.T) before the column pass */
#define HPDCT_FLAG_WRITEBACK_DEQUANT 0x10u /* inverse, fp32 -> fp32 with dequantisation: also store q*Q back
                                              into the coefficient buffer, as the cublasDCTv2 inverse's in-place
                                              multiply_matrices does (main_cublass_2.cu:285) */

/* Library / error information. */
const char* hpdct_version(void);
/* Build provenance: "src=<sha256 of csrc/ + include/> git=<rev> arch=gfx950"
 * (cuda-dct-idct_amd/src_digest.py defines the digest; bench.py recomputes it
 * from the tree it runs in).  No reference counterpart. */
const char* hpdct_build_info(void);
const char* hpdct_status_string(hpdct_status status);
const char* hpdct_last_error_string(void); /* thread-local, last failing call */

/* Built-in tables (main_newAppr.cu:60-68 Q, :73-81 T), copied into caller memory. */
void hpdct_default_quant_table(float* q64);
void hpdct_default_transform(float* t64);

/* Library-owned quantisation table used by every subsequent forward/inverse
 * call (process-wide).  q64: HOST pointer to 64 floats, row-major [v][u];
 * NULL restores the default JPEG luminance table.  Entries must be finite and
 * non-zero. */
hpdct_status hpdct_set_quant_table(const float* q64);
hpdct_status hpdct_get_quant_table(float* q64);

/* Forward 8x8 block transform.
 *   d_image    : device, height*width elements of in_type (HPDCT_U8 or HPDCT_F32)
 *   d_coef     : device, height*width elements of out_type (HPDCT_F32, or
 *                HPDCT_I8 with quantisation on)
 *   d_transform: device pointer to 64 floats T[v][i], or NULL for the
 *                built-in HpApprDCT matrix
 *   flags      : HPDCT_FLAG_*
 *   stream     : hipStream_t or NULL
 * Computes, per tile, q = round((T . (X-128) . T^T) / Q) with the reference's
 * fp32 fused-multiply-add order and IEEE division.  Asynchronous w.r.t. the
 * host.  d_image and d_coef must not overlap (except that d_image is written
 * with X-128 under HPDCT_FLAG_WRITEBACK_SHIFT). */
hpdct_status hpdct_forward(const void* d_image, hpdct_dtype in_type, void* d_coef, hpdct_dtype out_type,
                           int64_t height, int64_t width, const float* d_transform, unsigned flags,
                           void* stream);

/* Inverse 8x8 block transform.
 *   d_coef : device, height*width elements of in_type (HPDCT_F32 or HPDCT_I8)
 *   d_image: device, height*width elements of out_type: HPDCT_F32 (R+128, no
 *            clamp, as the reference) or HPDCT_U8 (then clamped to [0,255] and
 *            truncated, as convertToUnsignedChar, utils.cu:18-24)
 * Computes R = T^T . (q*Q) . T + 128 per tile. */
hpdct_status hpdct_inverse(const void* d_coef, hpdct_dtype in_type, void* d_image, hpdct_dtype out_type,
                           int64_t height, int64_t width, const float* d_transform, unsigned flags,
                           void* stream);

/* Typed shorthands for the common cases (built-in T, library Q). */
hpdct_status hpdct_forward_u8_f32(const uint8_t* d_image, float* d_coef, int64_t height, int64_t width,
                                  void* stream);
hpdct_status hpdct_forward_u8_i8(const uint8_t* d_image, int8_t* d_coef, int64_t height, int64_t width,
                                 void* stream);
hpdct_status hpdct_inverse_f32_f32(const float* d_coef, float* d_image, int64_t height, int64_t width,
                                   void* stream);

/* One-pass round trip (BASELINE config C3: forward DCT + IDCT with the
 * PEEN/MSE check).  The reference runs dct_all_blocks_cuda then
 * idct_all_blocks_cuda (main_newAppr.cu:99,120; benchmark_newAppr.cu:93,105)
 * and measures quality on the host (README.md:62-69).  Here one kernel reads
 * the uint8 frame once and writes
 *   d_coef   fp32 quantised coefficients (required; as hpdct_forward U8 -> F32)
 *   d_recon  the reconstruction R+128 as recon_type HPDCT_U8 (clamp +
 *            truncate) or HPDCT_F32 (no clamp), or NULL for none (as
 *            hpdct_inverse F32 -> recon_type on d_coef)
 *   d_sums   device struct, or NULL: the quality sums below (overwritten).  The
 *            kernel adds into a 16 KiB library "spread slot" kept per d_sums
 *            pointer (64 sub-slots on separate 256-B lines, so the atomics of
 *            many waves do not queue on one line; allocated zeroed on first
 *            use, 256 = 4 MiB at a time) and a one-wave kernel then folds it
 *            into *d_sums and zeroes it: no memset before the kernel.  A slot
 *            stays with its pointer until hpdct_roundtrip_release_sums.
 *            Without a slot (an allocation would be needed inside a stream
 *            capture, or 4096 pointers = 64 MiB of slots are live on the
 *            device) the launch memsets *d_sums and takes the tile-per-lane
 *            kernel.  Two overwriting launches in flight at once with the
 *            same d_sums on different streams race, as they would on the
 *            struct itself (accumulating ones do not: see below).
 * Built-in T, the library Q, level shift 128; coefficients and reconstruction
 * are bit-identical to the two separate calls.  HBM traffic per pixel: 1 B
 * read, 4 B (+1 or 4 B) written, against 10 B for the two calls.
 * PEEN = 100 sqrt(sse / sum_x2) %, MSE = sse / (height*width) (the
 * definitions of the README table). */
typedef struct hpdct_roundtrip_sums {
    uint64_t sse_f32_fx; /* sum (x - (R+128))^2 in units of 2^-16 (HPDCT_SSE_F32_UNIT): per tile four
                            fp32 partial sums, one per (row parity, column parity) class of its
                            pixels (an fma chain over the class's 16 pixels in row-major order, so
                            NOT the exact sum: relative error ~1e-10 on a 8192^2 frame), each
                            rounded to the unit, then all added exactly in any order.  Bit 63
                            (HPDCT_SSE_F32_INVALID) is set, sticky, when some partial sum is
                            non-finite or >= 2^24 (an extreme caller table on the IEEE path): the
                            field then holds no sum */
    uint64_t sse_u8;     /* sum (x - u8(R+128))^2, exact */
    uint64_t sum_x2;     /* sum x^2, exact */
} hpdct_roundtrip_sums;
#define HPDCT_SSE_F32_UNIT (1.0 / 65536.0)
#define HPDCT_SSE_F32_INVALID (1ull << 63)
hpdct_status hpdct_roundtrip_u8(const uint8_t* d_image, float* d_coef, void* d_recon, hpdct_dtype recon_type,
                                hpdct_roundtrip_sums* d_sums, int64_t height, int64_t width, void* stream);

/* The same round trip, but the frame's quality sums are ADDED to *d_sums,
 * which the caller has zeroed (d_sums required; the same spread slot and fold
 * kernel, which adds instead of overwriting).  A pipeline that owns a ring of
 * per-frame sums slots zeroes the ring once, with one memset for many frames,
 * and gets the same per-frame sums (or a batch total, if frames share a
 * slot).  The fold takes the slot with atomic exchanges and adds with atomic
 * adds, so frames that share d_sums may run on different streams at once. */
hpdct_status hpdct_roundtrip_u8_accumulate(const uint8_t* d_image, float* d_coef, void* d_recon,
                                           hpdct_dtype recon_type, hpdct_roundtrip_sums* d_sums, int64_t height,
                                           int64_t width, void* stream);

/* Return the spread slot kept for d_sums (16 KiB of device memory) to the
 * library, e.g. before freeing a ring of per-frame sums structs.  Call it when
 * no round trip with d_sums is in flight and no captured HIP graph that uses
 * d_sums will be replayed (the slot may go to another pointer); a later round
 * trip with the same pointer takes a slot again.  A pointer without a slot (or
 * NULL) is a no-op.  No reference counterpart. */
hpdct_status hpdct_roundtrip_release_sums(const hpdct_roundtrip_sums* d_sums);

/* A list of independent device frames in as few launches as possible (config
 * C2's small frames: one 1024^2 frame per launch is dispatch-bound, ~3.6 us for
 * ~0.9 us of work).  d_images / d_coefs: HOST arrays of n_frames DEVICE
 * pointers; frame f is height x width uint8 at d_images[f] (8-byte aligned),
 * its coefficients go to d_coefs[f] as out_type HPDCT_F32 (16-byte aligned) or
 * HPDCT_I8 (8-byte aligned).  Frames need not be contiguous or distinct inputs
 * (a pool may repeat), but no coefficient plane may overlap another plane or
 * any input.  Built-in T, the library Q, level shift 128: the result is
 * bit-identical to n_frames calls of hpdct_forward.  One kernel launch per 64
 * frames (the pointer table travels in the kernel arguments); asynchronous on
 * `stream`; n_frames == 0 is a no-op.  The reference has no batch entry
 * (dct_all_blocks_cuda takes one image, main_newAppr.cu:252). */
hpdct_status hpdct_forward_frames(const uint8_t* const* d_images, void* const* d_coefs, hpdct_dtype out_type,
                                  int64_t n_frames, int64_t height, int64_t width, void* stream);

/* Host-resident batch (BASELINE config C5): frame f (height x width uint8 at
 * h_frames[f]) -> coefficients at h_coef[f] (out_type HPDCT_F32 or HPDCT_I8),
 * pipelined over nstreams (1..16) HIP streams, each with one device input and
 * one output buffer: H2D copy, fused forward kernel and D2H copy of different
 * frames overlap (2 streams keep both DMA directions busy: 0.90-0.97 of the
 * copy-only duplex ceiling on MI355X).  HPDCT_STREAM_PIPELINE=engines selects
 * a rejected A/B layout (one stream per engine over nstreams device slots).
 * Pointers may repeat (a pool cycled over the batch).  Host
 * buffers should be pinned for the copies to overlap.  Synchronous: returns
 * when every coefficient plane is in host memory; *elapsed_ms (may be NULL)
 * receives the device-timed span of the batch.  Replaces the reference's
 * one-image blocking H2D/compute/D2H sequence (benchmark_newAppr.cu:88-109). */
hpdct_status hpdct_stream_forward(const uint8_t* const* h_frames, void* const* h_coef, int64_t n_frames,
                                  int64_t height, int64_t width, hpdct_dtype out_type, int nstreams,
                                  float* elapsed_ms);

/* The same pipeline with its resources kept across calls: hpdct_stream_create
 * makes the nstreams HIP streams, their device input/output buffers (one
 * height x width frame each) and the timing events on the current device;
 * hpdct_stream_run streams one batch through them (semantics and timing as
 * hpdct_stream_forward, on the context's device); hpdct_stream_destroy frees
 * them.  hpdct_stream_forward is create + run + destroy.  A context is not
 * thread-safe: one run at a time. */
typedef struct hpdct_stream_ctx_s* hpdct_stream_ctx;
hpdct_status hpdct_stream_create(hpdct_stream_ctx* ctx, int64_t height, int64_t width, hpdct_dtype out_type,
                                 int nstreams);
hpdct_status hpdct_stream_run(hpdct_stream_ctx ctx, const uint8_t* const* h_frames, void* const* h_coef,
                              int64_t n_frames, float* elapsed_ms);
hpdct_status hpdct_stream_destroy(hpdct_stream_ctx ctx);

/* Synthetic frames generated on the device (BASELINE config C4): pixel
 * i of the frame = splitmix64(seed, first_index + i) & 255 (the oracle's
 * oracle_fill_hash_u8 restates it). */
hpdct_status hpdct_fill_hash_u8(uint8_t* d_out, int64_t n, uint64_t seed, int64_t first_index, void* stream);

/* Decode n int8 wire coefficients (hpdct_forward's HPDCT_I8 output, e.g. a
 * root's gathered C4 frame) into the fp32 coefficient plane
 * dct_all_blocks_cuda produces (main_newAppr.cu:252-291): out[i] = (float)q[i].
 * Equal in value to the fp32 forward's output; a -0.0 of that output decodes
 * as +0.0.  Device pointers: d_q 4-byte, d_out 16-byte aligned.  Async on
 * `stream`.  No reference counterpart (the reference has no int8 format). */
hpdct_status hpdct_decode_i8_f32(const int8_t* d_q, float* d_out, int64_t n, void* stream);

/* Work mapping of the kernels (new; the reference has one fixed decomposition
 * per program).  Output is bit-identical in every mapping; only speed differs.
 *   AUTO   per frame: eight lanes per 8x8 tile ("octet") for frames below
 *          8 x 64-tile sets per CU; above that two lanes per tile ("duo") for
 *          fp32 -> fp32 and the fp32 -> uint8 inverse, one lane per tile for
 *          the rest (DESIGN.md "Kernels").
 *   TILE   one lane per tile always.     OCTET  eight lanes per tile always.
 *   DUO    two lanes per tile for every fp32 -> fp32 kernel and the fp32 -> uint8
 *          inverse, AUTO otherwise.
 * The cublasDCTv2 pass order (HPDCT_FLAG_ROW_FIRST) runs two lanes per tile
 * (rows first) except under TILE.  Process-wide; the initial value comes from the environment variable
 * HPDCT_MAPPING ("auto", "tile", "octet", "duo"), else AUTO.  For A/B
 * measurement and tests; set it while no call is in flight. */
typedef enum hpdct_mapping {
    HPDCT_MAPPING_AUTO = 0,
    HPDCT_MAPPING_TILE = 1,
    HPDCT_MAPPING_OCTET = 2,
    HPDCT_MAPPING_DUO = 3
} hpdct_mapping;
hpdct_status hpdct_set_mapping(hpdct_mapping mapping);
hpdct_mapping hpdct_get_mapping(void);

/* Host-side helpers (no device work). */
void hpdct_fill_rand_u8(uint8_t* h_out, int64_t n, uint32_t seed); /* srand(seed); rand()%256 (glibc TYPE_3) */
void hpdct_u8_to_f32(const uint8_t* h_in, float* h_out, int64_t n); /* convertToFloat, utils.cu:10-15 */
void hpdct_f32_to_u8(const float* h_in, uint8_t* h_out, int64_t n); /* convertToUnsignedChar, utils.cu:18-24 */

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* HPDCT_H */
