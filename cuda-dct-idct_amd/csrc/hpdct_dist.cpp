// hpdct_dist.cpp -- the row-shard layer of include/hpdct_dist.h on RCCL
// (libhpdct_dist.so).  The slab kernel is libhpdct's hpdct_forward; the only
// collective is the gather of the coefficient slabs to the root, as
// ncclSend / ncclRecv pairs inside one group (rccl.h:700,722), which also
// covers slabs that differ by a tile row (ncclGather, rccl.h:745, needs equal
// counts).  Bytes travel as ncclUint8: the element type does not matter to a
// gather.  Before the first gather of a geometry, the ranks check that they
// agree on it (hpdct_dist_geometry.hpp): a disagreement is an error on every
// rank instead of sends and receives of different sizes that never complete.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>

#include "hpdct.h"
#include "hpdct_dist.h"
#include "hpdct_dist_geometry.hpp"
#include "hpdct_kernels.h"

static_assert(HPDCT_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "hpdct_unique_id size");

namespace {
// Communicators of one hpdct_comm_init_all call live in this process: each
// round of gathers (one per communicator, normally inside one
// hpdct_group_start/end) is compared on the host, no collective needed.
struct Clique {
    std::mutex m;
    int reported = 0;  // gathers of the current round so far
    hpdct::dist::Geometry g{};
};
thread_local int t_group_depth = 0;
}  // namespace

struct hpdct_comm_s {
    ncclComm_t nccl;
    int rank, size, device;
    std::shared_ptr<Clique> clique;   // init_all communicators only
    hpdct::dist::AgreedSet agreed;    // init_rank: geometries the ranks agreed on
    int64_t* d_check = nullptr;       // init_rank: 64 B for the agreement all-reduce
};

namespace {

hpdct_status fail(hpdct_status st, const std::string& msg) {
    return static_cast<hpdct_status>(hpdct::set_last_error(st, msg.c_str()));
}
hpdct_status nccl_status(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return HPDCT_SUCCESS;
    return fail(HPDCT_ERROR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
hpdct_status hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return HPDCT_SUCCESS;
    return fail(HPDCT_ERROR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
size_t elem_size(hpdct_dtype t) { return t == HPDCT_F32 ? 4 : 1; }

// The caller's current device is restored on scope exit (calls on a
// communicator run on its device).
struct DeviceScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int dev) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// (first_row, rows) of every rank, as hpdct_shard_rows
void shard(int64_t height, int world, int rank, int64_t& first, int64_t& rows) {
    const int64_t tile_rows = height / 8, base = tile_rows / world, extra = tile_rows % world;
    first = (rank * base + (rank < extra ? rank : extra)) * 8;
    rows = (base + (rank < extra ? 1 : 0)) * 8;
}

hpdct_status check_geometry(hpdct_comm comm, int64_t height, int64_t width) {
    if (!comm) return fail(HPDCT_ERROR_INVALID_VALUE, "null communicator");
    if (height <= 0 || width <= 0 || height % 8 || width % 8)
        return fail(HPDCT_ERROR_INVALID_VALUE, "height and width must be positive multiples of 8");
    if (height / 8 < comm->size)
        return fail(HPDCT_ERROR_INVALID_VALUE, "fewer tile rows (" + std::to_string(height / 8) + ") than ranks (" +
                                                   std::to_string(comm->size) + ")");
    return HPDCT_SUCCESS;
}

// The ranks agree on this gather's geometry (see the file comment).
// (A one-rank per-process communicator runs the check too: it is once per
// geometry, and it keeps the all-reduce path exercised on a one-GPU box.)
hpdct_status check_agreement(hpdct_comm comm, const hpdct::dist::Geometry& g, hipStream_t s) {
    if (comm->clique) {
        Clique& c = *comm->clique;
        std::lock_guard<std::mutex> lock(c.m);
        if (c.reported == 0) c.g = g;  // the round's first gather sets the geometry
        const bool same = c.g == g;
        if (++c.reported == comm->size) c.reported = 0;  // round complete
        if (same) return HPDCT_SUCCESS;
        return fail(HPDCT_ERROR_INVALID_VALUE,
                    "gathers of one round disagree on (height, width, type, root) across the communicators");
    }
    if (comm->agreed.contains(g)) return HPDCT_SUCCESS;
    if (t_group_depth > 0)
        return fail(HPDCT_ERROR_INVALID_VALUE,
                    "the first gather of a new geometry on a per-process communicator must be outside "
                    "hpdct_group_start/end (its agreement check synchronises the stream)");
    if (!comm->d_check) {
        void* p = nullptr;
        if (hpdct_status st = hip_status(hipMalloc(&p, sizeof(int64_t) * hpdct::dist::kCheckWords), "hipMalloc"))
            return st;
        comm->d_check = static_cast<int64_t*>(p);
    }
    int64_t v[hpdct::dist::kCheckWords];
    hpdct::dist::pack_for_max(g, v);
    if (hpdct_status st = hip_status(hipMemcpyAsync(comm->d_check, v, sizeof(v), hipMemcpyHostToDevice, s),
                                     "hipMemcpyAsync"))
        return st;
    if (hpdct_status st = nccl_status(ncclAllReduce(comm->d_check, comm->d_check, hpdct::dist::kCheckWords,
                                                    ncclInt64, ncclMax, comm->nccl, s),
                                      "ncclAllReduce (geometry check)"))
        return st;
    if (hpdct_status st = hip_status(hipMemcpyAsync(v, comm->d_check, sizeof(v), hipMemcpyDeviceToHost, s),
                                     "hipMemcpyAsync"))
        return st;
    if (hpdct_status st = hip_status(hipStreamSynchronize(s), "hipStreamSynchronize")) return st;
    if (!hpdct::dist::agree_after_max(v))
        return fail(HPDCT_ERROR_INVALID_VALUE,
                    "ranks disagree on the gather's (height, width, type, root): max (" + std::to_string(v[0]) +
                        ", " + std::to_string(v[1]) + ", " + std::to_string(v[2]) + ", " + std::to_string(v[3]) +
                        ") vs min (" + std::to_string(-v[4]) + ", " + std::to_string(-v[5]) + ", " +
                        std::to_string(-v[6]) + ", " + std::to_string(-v[7]) + ")");
    comm->agreed.add(g);
    return HPDCT_SUCCESS;
}

}  // namespace

extern "C" {

hpdct_status hpdct_shard_rows(int64_t height, int world, int rank, int64_t* first_row, int64_t* rows) {
    if (!first_row || !rows) return fail(HPDCT_ERROR_INVALID_VALUE, "null output pointer");
    if (height <= 0 || height % 8) return fail(HPDCT_ERROR_INVALID_VALUE, "height must be a positive multiple of 8");
    if (world < 1 || rank < 0 || rank >= world) return fail(HPDCT_ERROR_INVALID_VALUE, "rank out of range");
    shard(height, world, rank, *first_row, *rows);
    return HPDCT_SUCCESS;
}

hpdct_status hpdct_comm_init_all(hpdct_comm* comms, int ndev, const int* devices) {
    if (!comms || !devices || ndev < 1) return fail(HPDCT_ERROR_INVALID_VALUE, "bad communicator list");
    for (int i = 0; i < ndev; ++i) comms[i] = nullptr;
    ncclComm_t* raw = new (std::nothrow) ncclComm_t[ndev];
    if (!raw) return fail(HPDCT_ERROR_DEVICE, "out of host memory");
    const hpdct_status st = nccl_status(ncclCommInitAll(raw, ndev, devices), "ncclCommInitAll");
    if (st != HPDCT_SUCCESS) {
        delete[] raw;
        return st;
    }
    bool ok = true;
    std::shared_ptr<Clique> clique(new (std::nothrow) Clique());
    ok = clique != nullptr;
    for (int i = 0; i < ndev && ok; ++i) {
        comms[i] = new (std::nothrow) hpdct_comm_s{raw[i], i, ndev, devices[i], clique, {}, nullptr};
        ok = ok && comms[i];
    }
    if (!ok) {  // all or nothing: no communicator survives a failed call
        for (int i = 0; i < ndev; ++i) {
            (void)ncclCommDestroy(raw[i]);
            delete comms[i];
            comms[i] = nullptr;
        }
    }
    delete[] raw;
    return ok ? HPDCT_SUCCESS : fail(HPDCT_ERROR_DEVICE, "out of host memory");
}

hpdct_status hpdct_comm_unique_id(hpdct_unique_id* id) {
    if (!id) return fail(HPDCT_ERROR_INVALID_VALUE, "null id");
    ncclUniqueId u;
    const hpdct_status st = nccl_status(ncclGetUniqueId(&u), "ncclGetUniqueId");
    if (st == HPDCT_SUCCESS) memcpy(id->internal, u.internal, sizeof(u.internal));
    return st;
}

hpdct_status hpdct_comm_init_rank(hpdct_comm* comm, int nranks, const hpdct_unique_id* id, int rank, int device) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
        return fail(HPDCT_ERROR_INVALID_VALUE, "bad communicator arguments");
    *comm = nullptr;
    DeviceScope ds(device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    ncclUniqueId u;
    memcpy(u.internal, id->internal, sizeof(u.internal));
    ncclComm_t c;
    if (hpdct_status st = nccl_status(ncclCommInitRank(&c, nranks, u, rank), "ncclCommInitRank")) return st;
    *comm = new (std::nothrow) hpdct_comm_s{c, rank, nranks, device, nullptr, {}, nullptr};
    if (!*comm) {
        (void)ncclCommDestroy(c);
        return fail(HPDCT_ERROR_DEVICE, "out of host memory");
    }
    return HPDCT_SUCCESS;
}

hpdct_status hpdct_comm_destroy(hpdct_comm comm) {
    if (!comm) return HPDCT_SUCCESS;
    if (comm->d_check) {
        DeviceScope ds(comm->device);
        (void)hipFree(comm->d_check);
    }
    const hpdct_status st = nccl_status(ncclCommDestroy(comm->nccl), "ncclCommDestroy");
    delete comm;
    return st;
}

int hpdct_comm_rank(hpdct_comm comm) { return comm ? comm->rank : -1; }
int hpdct_comm_size(hpdct_comm comm) { return comm ? comm->size : -1; }
int hpdct_comm_device(hpdct_comm comm) { return comm ? comm->device : -1; }

hpdct_status hpdct_group_start(void) {
    const hpdct_status st = nccl_status(ncclGroupStart(), "ncclGroupStart");
    if (st == HPDCT_SUCCESS) ++t_group_depth;
    return st;
}
hpdct_status hpdct_group_end(void) {
    if (t_group_depth > 0) --t_group_depth;
    return nccl_status(ncclGroupEnd(), "ncclGroupEnd");
}

hpdct_status hpdct_forward_slab(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                int64_t height, int64_t width, void* stream) {
    if (hpdct_status st = check_geometry(comm, height, width)) return st;
    int64_t first, rows;
    shard(height, comm->size, comm->rank, first, rows);
    DeviceScope ds(comm->device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    return hpdct_forward(d_slab, HPDCT_U8, d_coef_slab, out_type, rows, width, nullptr, 0u, stream);
}

hpdct_status hpdct_gather_rows(hpdct_comm comm, const void* d_slab, void* d_frame, hpdct_dtype type, int64_t height,
                               int64_t width, int root, void* stream) {
    if (hpdct_status st = check_geometry(comm, height, width)) return st;
    if (type != HPDCT_F32 && type != HPDCT_I8 && type != HPDCT_U8)
        return fail(HPDCT_ERROR_UNSUPPORTED, "gather type must be HPDCT_F32, HPDCT_I8 or HPDCT_U8");
    if (root < 0 || root >= comm->size) return fail(HPDCT_ERROR_INVALID_VALUE, "root out of range");
    if (!d_slab) return fail(HPDCT_ERROR_INVALID_VALUE, "null slab pointer");
    if (comm->rank == root && !d_frame) return fail(HPDCT_ERROR_INVALID_VALUE, "null frame pointer on the root");
    const size_t row_bytes = static_cast<size_t>(width) * elem_size(type);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DeviceScope ds(comm->device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    const hpdct::dist::Geometry geo{{height, width, static_cast<int64_t>(type), root}};
    if (hpdct_status st = check_agreement(comm, geo, s)) return st;
    // one rank whose slab already sits in the frame: nothing moves
    if (comm->size == 1 && d_frame == d_slab) return HPDCT_SUCCESS;
    int64_t first, rows;
    if (comm->rank != root) {
        shard(height, comm->size, comm->rank, first, rows);
        return nccl_status(ncclSend(d_slab, static_cast<size_t>(rows) * row_bytes, ncclUint8, root, comm->nccl, s),
                           "ncclSend");
    }
    char* frame = static_cast<char*>(d_frame);
    if (hpdct_status st = nccl_status(ncclGroupStart(), "ncclGroupStart")) return st;
    hpdct_status st = HPDCT_SUCCESS;
    for (int r = 0; r < comm->size && st == HPDCT_SUCCESS; ++r) {
        shard(height, comm->size, r, first, rows);
        char* dst = frame + static_cast<size_t>(first) * row_bytes;
        const size_t bytes = static_cast<size_t>(rows) * row_bytes;
        if (r == root) {
            if (dst != d_slab)
                st = hip_status(hipMemcpyAsync(dst, d_slab, bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
        } else {
            st = nccl_status(ncclRecv(dst, bytes, ncclUint8, r, comm->nccl, s), "ncclRecv");
        }
    }
    const hpdct_status end = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    return st != HPDCT_SUCCESS ? st : end;
}

hpdct_status hpdct_forward_sharded(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                   void* d_frame, int64_t height, int64_t width, int root, void* stream) {
    if (hpdct_status st = hpdct_forward_slab(comm, d_slab, d_coef_slab, out_type, height, width, stream)) return st;
    return hpdct_gather_rows(comm, d_coef_slab, d_frame, out_type, height, width, root, stream);
}

}  // extern "C"
