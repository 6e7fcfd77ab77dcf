/*
 * hpdct_dist.h -- native row-shard layer of the MI355X DCT path over RCCL
 * (BASELINE config C4: one large frame row-sharded across the GPUs of a node,
 * RCCL over xGMI only for the final gather).  Library: libhpdct_dist.so
 * (cuda-dct-idct_amd/lib/), linked against libhpdct.so and librccl.so, so a
 * caller of the single-GPU path does not pull RCCL in.
 *
 * The reference has no multi-GPU code: its callers are
 * single-process C/C++ host programs (main_newAppr.cu:88-120,
 * benchmark_newAppr.cu:82-109) calling dct_all_blocks_cuda once per image.
 * This layer gives such a caller the north_star's sharded form:
 *
 *   hpdct_shard_rows      which rows a rank owns (whole 8-row tile rows,
 *                         sizes differing by at most one tile row)
 *   hpdct_comm_*          RCCL communicators: one per GPU of this process
 *                         (ncclCommInitAll) or one per process (unique id +
 *                         ncclCommInitRank, the id shared by the caller)
 *   hpdct_forward_slab    the fused forward kernel on this rank's slab
 *   hpdct_gather_rows     the only collective: every rank's coefficient slab
 *                         to the root's full frame (ncclSend / ncclRecv in one
 *                         group; slabs may differ by a tile row)
 *   hpdct_forward_sharded forward_slab + gather_rows in one call
 *
 * Tiles are independent, so a slab's coefficients are bit-identical to the
 * same rows of a one-GPU hpdct_forward of the whole frame.
 *
 * A process that drives several GPUs from one thread calls the gathers (or
 * hpdct_forward_sharded) of all its communicators between
 * hpdct_group_start() and hpdct_group_end() (ncclGroupStart/End), exactly
 * as RCCL requires for single-thread multi-device use.
 *
 * Agreement (a gather whose ranks disagree on its size would post sends and
 * receives that never complete):
 *   - communicators of one hpdct_comm_init_all: the gathers of a group are
 *     queued and compared at hpdct_group_end; they are posted only when every
 *     communicator asked for the same gathers in the same order and none of
 *     the calls failed its checks, otherwise nothing is posted and
 *     hpdct_group_end returns the error;
 *   - per-process communicators (hpdct_comm_init_rank): one 64-byte max
 *     all-reduce before the first gather of a (height, width, type, root) the
 *     communicator has not agreed on yet.  It catches ranks that disagree on
 *     that first gather of a new geometry; ranks that later mix an agreed
 *     geometry with a new one on the same call are not caught (the caller
 *     keeps the ranks' call sequences alike, as for any collective).
 */
#ifndef HPDCT_DIST_H
#define HPDCT_DIST_H

#include <stdint.h>

#include "hpdct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hpdct_comm_s* hpdct_comm;

#define HPDCT_UNIQUE_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES (rccl.h:40) */
typedef struct hpdct_unique_id {
    char internal[HPDCT_UNIQUE_ID_BYTES];
} hpdct_unique_id;

/* Rows [*first_row, *first_row + *rows) of a height-row frame owned by rank
 * (0 <= rank < world): contiguous slabs of whole tile rows, earlier ranks get
 * the extra tile row.  Host-only (no device work). */
hpdct_status hpdct_shard_rows(int64_t height, int world, int rank, int64_t* first_row, int64_t* rows);

/* Communicators.  init_all: one communicator per listed device, all in this
 * process (comms[i] drives devices[i], rank i).  unique_id + init_rank: one
 * communicator per process; rank 0 creates the id and the caller delivers it
 * to every rank (e.g. through its launcher's store); `device` is the HIP
 * device the communicator and every call on it use. */
hpdct_status hpdct_comm_init_all(hpdct_comm* comms, int ndev, const int* devices);
hpdct_status hpdct_comm_unique_id(hpdct_unique_id* id);
hpdct_status hpdct_comm_init_rank(hpdct_comm* comm, int nranks, const hpdct_unique_id* id, int rank, int device);
hpdct_status hpdct_comm_destroy(hpdct_comm comm);
int hpdct_comm_rank(hpdct_comm comm);   /* -1 for NULL */
int hpdct_comm_size(hpdct_comm comm);   /* -1 for NULL */
int hpdct_comm_device(hpdct_comm comm); /* -1 for NULL */

/* ncclGroupStart / ncclGroupEnd (one thread driving several communicators). */
hpdct_status hpdct_group_start(void);
hpdct_status hpdct_group_end(void);

/* The forward kernel on this rank's slab of an height x width frame:
 * d_slab = the slab's pixels (rows x width uint8, rows from hpdct_shard_rows),
 * d_coef_slab = its coefficients (rows x width of out_type HPDCT_F32 or
 * HPDCT_I8).  Built-in T, library Q, level shift 128; runs on the
 * communicator's device, on `stream` (NULL = that device's null stream). */
hpdct_status hpdct_forward_slab(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                int64_t height, int64_t width, void* stream);

/* Gather: every rank passes its slab (rows x width elements of `type`,
 * HPDCT_F32 / HPDCT_I8 / HPDCT_U8); the root receives the full
 * height x width frame in d_frame (ignored elsewhere, may be NULL).  The
 * root's own slab is copied device to device unless it already sits at its
 * place in d_frame.  Asynchronous on `stream`. */
hpdct_status hpdct_gather_rows(hpdct_comm comm, const void* d_slab, void* d_frame, hpdct_dtype type, int64_t height,
                               int64_t width, int root, void* stream);

/* The int8 wire format's gather: every rank but the
 * root passes its int8 coefficient slab (d_slab, from hpdct_forward_slab with
 * HPDCT_I8); the root has already written its own slab as fp32 at its rows of
 * d_frame_f32 (hpdct_forward of its slab into d_frame_f32 + first_row * width)
 * and passes d_slab = NULL.  The root receives the peers' slabs into
 * d_frame_i8 (a height x width int8 scratch frame; the root's rows are not
 * touched) and decodes them into d_frame_f32 (hpdct_decode_i8_f32: at most two
 * launches, the rows before and after its own slab), so d_frame_f32 ends as
 * the fp32 frame of a one-GPU hpdct_forward, bit for bit.  Asynchronous on
 * `stream`; inside hpdct_group_start/end the decodes are issued at the
 * outermost hpdct_group_end, behind the receives. */
hpdct_status hpdct_gather_decode_i8(hpdct_comm comm, const int8_t* d_slab, int8_t* d_frame_i8, float* d_frame_f32,
                                    int64_t height, int64_t width, int root, void* stream);

/* hpdct_forward_slab then hpdct_gather_rows of the coefficient slab. */
hpdct_status hpdct_forward_sharded(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                   void* d_frame, int64_t height, int64_t width, int root, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* HPDCT_DIST_H */
