// hpdct_dist.cpp -- the row-shard layer of include/hpdct_dist.h on RCCL
// (libhpdct_dist.so).  The slab kernel is libhpdct's hpdct_forward; the only
// collective is the gather of the coefficient slabs to the root, as
// ncclSend / ncclRecv pairs inside one group (rccl.h:700,722), which also
// covers slabs that differ by a tile row (ncclGather, rccl.h:745, needs equal
// counts).  Bytes travel as ncclUint8: the element type does not matter to a
// gather.  The ranks check that they agree on a gather before anything is
// posted (hpdct_dist_geometry.hpp), so a disagreement is an error instead of
// sends and receives of different sizes that never complete:
//   - communicators of one hpdct_comm_init_all (one thread, one group): their
//     gathers are queued, compared on the host at hpdct_group_end and posted
//     there only if every communicator asked for the same gathers;
//   - a per-process communicator: one 64-byte max all-reduce before the first
//     gather of a geometry it has not agreed on yet (see hpdct_dist.h for what
//     that covers).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "hpdct.h"
#include "hpdct_dist.h"
#include "hpdct_dist_geometry.hpp"
#include "hpdct_kernels.h"

static_assert(HPDCT_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "hpdct_unique_id size");

namespace {
using hpdct::dist::Post;
using hpdct::dist::RootSlab;

// The root's int8 -> fp32 decode of the peer rows of a gather-decode: launched
// after the receives are enqueued, i.e. after the outermost ncclGroupEnd.
struct DecodeJob {
    int device;
    hipStream_t s;
    const int8_t* src;
    float* dst;
    int64_t n;
};

// One gather call, ready to post.
struct Pending {
    struct hpdct_comm_s* comm;
    std::vector<Post> plan;
    const char* slab;
    char* frame;
    hipStream_t s;
    std::vector<DecodeJob> decodes;
};

// Communicators of one hpdct_comm_init_all call live in this process: the
// gathers of a group are queued per communicator and compared on the host
// at hpdct_group_end (hpdct::dist::clique_round_agrees), no collective needed.
struct Clique {
    std::mutex m;
    std::vector<std::vector<hpdct::dist::Geometry>> asked;  // per communicator rank, in call order
    std::vector<bool> failed;                               // a call of that communicator failed validation
    std::vector<Pending> queued;
    explicit Clique(int n) : asked(n), failed(n, false) {}
    void clear() {
        for (auto& a : asked) a.clear();
        std::fill(failed.begin(), failed.end(), false);
        queued.clear();
    }
};
thread_local int t_group_depth = 0;
thread_local std::vector<std::shared_ptr<Clique>> t_cliques;  // cliques with gathers in the open group
thread_local std::vector<DecodeJob> t_decodes;                // decodes waiting for the outermost group end
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

hpdct_status check_geometry(hpdct_comm comm, int64_t height, int64_t width) {
    if (!comm) return fail(HPDCT_ERROR_INVALID_VALUE, "null communicator");
    if (height <= 0 || width <= 0 || height % 8 || width % 8)
        return fail(HPDCT_ERROR_INVALID_VALUE, "height and width must be positive multiples of 8");
    if (height / 8 < comm->size)
        return fail(HPDCT_ERROR_INVALID_VALUE, "fewer tile rows (" + std::to_string(height / 8) + ") than ranks (" +
                                                   std::to_string(comm->size) + ")");
    return HPDCT_SUCCESS;
}

// A per-process communicator: the ranks agree on this gather's geometry (see
// the file comment).  A one-rank communicator runs the check too: it is once
// per geometry, and it keeps the all-reduce path exercised on a one-GPU box.
hpdct_status check_agreement(hpdct_comm comm, const hpdct::dist::Geometry& g, hipStream_t s) {
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

// Posts one gather's operations (inside the caller's ncclGroupStart/End).
hpdct_status post_plan(const Pending& p) {
    DeviceScope ds(p.comm->device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    for (const Post& o : p.plan) {
        hpdct_status st = HPDCT_SUCCESS;
        switch (o.kind) {
            case Post::kSend:
                st = nccl_status(ncclSend(p.slab, o.bytes, ncclUint8, o.peer, p.comm->nccl, p.s), "ncclSend");
                break;
            case Post::kRecv:
                st = nccl_status(ncclRecv(p.frame + o.offset, o.bytes, ncclUint8, o.peer, p.comm->nccl, p.s),
                                 "ncclRecv");
                break;
            case Post::kCopy:
                if (p.frame + o.offset != p.slab)
                    st = hip_status(hipMemcpyAsync(p.frame + o.offset, p.slab, o.bytes, hipMemcpyDeviceToDevice, p.s),
                                    "hipMemcpyAsync");
                break;
        }
        if (st != HPDCT_SUCCESS) return st;
    }
    return HPDCT_SUCCESS;
}

hpdct_status run_decodes(std::vector<DecodeJob>& jobs) {
    hpdct_status first = HPDCT_SUCCESS;
    for (const DecodeJob& j : jobs) {
        DeviceScope ds(j.device);
        hpdct_status st = ds.err != hipSuccess ? hip_status(ds.err, "hipSetDevice")
                                               : hpdct_decode_i8_f32(j.src, j.dst, j.n, j.s);
        if (first == HPDCT_SUCCESS) first = st;
    }
    jobs.clear();
    return first;
}

// The shared part of the gathers: validation, agreement, then the posts now
// (per-process communicator, or a lone init_all communicator outside a group)
// or queued for hpdct_group_end (init_all communicators inside a group).
hpdct_status gather(hpdct_comm comm, const void* d_slab, void* d_frame, hpdct_dtype type, int64_t height,
                    int64_t width, int root, void* stream, RootSlab own, float* d_frame_f32) {
    hpdct_status st = check_geometry(comm, height, width);
    const bool defer = st == HPDCT_SUCCESS && comm->clique && t_group_depth > 0;
    auto note_failure = [&](hpdct_status e) {
        if (comm && comm->clique && t_group_depth > 0) {
            // the round fails as a whole: nothing of it is posted at group end
            std::lock_guard<std::mutex> lock(comm->clique->m);
            comm->clique->failed[comm->rank] = true;
            if (std::find(t_cliques.begin(), t_cliques.end(), comm->clique) == t_cliques.end())
                t_cliques.push_back(comm->clique);
        }
        return e;
    };
    if (st != HPDCT_SUCCESS) return note_failure(st);
    if (type != HPDCT_F32 && type != HPDCT_I8 && type != HPDCT_U8)
        return note_failure(fail(HPDCT_ERROR_UNSUPPORTED, "gather type must be HPDCT_F32, HPDCT_I8 or HPDCT_U8"));
    if (root < 0 || root >= comm->size) return note_failure(fail(HPDCT_ERROR_INVALID_VALUE, "root out of range"));
    if (comm->rank != root && !d_slab) return note_failure(fail(HPDCT_ERROR_INVALID_VALUE, "null slab pointer"));
    if (comm->rank == root && own != RootSlab::kSkip && !d_slab)
        return note_failure(fail(HPDCT_ERROR_INVALID_VALUE, "null slab pointer"));
    if (comm->rank == root && !d_frame) return note_failure(fail(HPDCT_ERROR_INVALID_VALUE, "null frame pointer on the root"));
    if (comm->rank == root && own == RootSlab::kSkip && !d_frame_f32)
        return note_failure(fail(HPDCT_ERROR_INVALID_VALUE, "null fp32 frame pointer on the root"));
    if (comm->clique && comm->size > 1 && t_group_depth == 0)
        return fail(HPDCT_ERROR_INVALID_VALUE,
                    "gathers on communicators of hpdct_comm_init_all go between hpdct_group_start and "
                    "hpdct_group_end (one thread drives every device)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const hpdct::dist::Geometry geo{{height, width, static_cast<int64_t>(type), root}};

    Pending p{comm, {}, static_cast<const char*>(d_slab), static_cast<char*>(d_frame), s, {}};
    // the root's slab is in place only when it sits at ITS rows of the frame
    // (frame + first * row bytes); a slab at the start of the frame of a root
    // whose rows start further down is copied
    p.plan = hpdct::dist::gather_plan(height, width, elem_size(type), comm->size, root, comm->rank,
                                      hpdct::dist::root_slab_mode(own, d_slab, d_frame, height, width,
                                                                  elem_size(type), comm->size, root, comm->rank));
    if (comm->rank == root && own == RootSlab::kSkip) {
        // decode the peer rows: the slabs before the root's and after it are contiguous
        int64_t first, rows;
        hpdct::dist::shard_rows(height, comm->size, root, first, rows);
        const int8_t* q = static_cast<const int8_t*>(d_frame);
        if (first > 0) p.decodes.push_back({comm->device, s, q, d_frame_f32, first * width});
        if (first + rows < height)
            p.decodes.push_back({comm->device, s, q + (first + rows) * width, d_frame_f32 + (first + rows) * width,
                                 (height - first - rows) * width});
    }

    if (defer) {
        Clique& c = *comm->clique;
        std::lock_guard<std::mutex> lock(c.m);
        c.asked[comm->rank].push_back(geo);
        c.queued.push_back(std::move(p));
        if (std::find(t_cliques.begin(), t_cliques.end(), comm->clique) == t_cliques.end())
            t_cliques.push_back(comm->clique);
        return HPDCT_SUCCESS;
    }
    DeviceScope ds(comm->device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    if (!comm->clique) {
        if (hpdct_status e = check_agreement(comm, geo, s)) return e;
    }
    if (p.plan.empty() && p.decodes.empty()) return HPDCT_SUCCESS;
    if (hpdct_status e = nccl_status(ncclGroupStart(), "ncclGroupStart")) return e;
    st = post_plan(p);
    const hpdct_status end = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    if (st == HPDCT_SUCCESS) st = end;
    if (st != HPDCT_SUCCESS) return st;
    if (t_group_depth > 0) {  // the receives are enqueued at the outermost group end
        t_decodes.insert(t_decodes.end(), p.decodes.begin(), p.decodes.end());
        return HPDCT_SUCCESS;
    }
    return run_decodes(p.decodes);
}

}  // namespace

extern "C" {

hpdct_status hpdct_shard_rows(int64_t height, int world, int rank, int64_t* first_row, int64_t* rows) {
    if (!first_row || !rows) return fail(HPDCT_ERROR_INVALID_VALUE, "null output pointer");
    if (height <= 0 || height % 8) return fail(HPDCT_ERROR_INVALID_VALUE, "height must be a positive multiple of 8");
    if (world < 1 || rank < 0 || rank >= world) return fail(HPDCT_ERROR_INVALID_VALUE, "rank out of range");
    hpdct::dist::shard_rows(height, world, rank, *first_row, *rows);
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
    std::shared_ptr<Clique> clique(new (std::nothrow) Clique(ndev));
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
    if (t_group_depth == 0) {  // a new group: no round of an earlier (abandoned) group survives
        for (auto& c : t_cliques) {
            std::lock_guard<std::mutex> lock(c->m);
            c->clear();
        }
        t_cliques.clear();
        t_decodes.clear();
    }
    const hpdct_status st = nccl_status(ncclGroupStart(), "ncclGroupStart");
    if (st == HPDCT_SUCCESS) ++t_group_depth;
    return st;
}

hpdct_status hpdct_group_end(void) {
    if (t_group_depth > 0) --t_group_depth;
    hpdct_status st = HPDCT_SUCCESS;
    if (t_group_depth == 0) {
        // each clique's round: posted whole if its communicators agree, else not at all
        for (auto& cp : t_cliques) {
            Clique& c = *cp;
            std::lock_guard<std::mutex> lock(c.m);
            if (!hpdct::dist::clique_round_agrees(c.asked, c.failed)) {
                if (st == HPDCT_SUCCESS)
                    st = fail(HPDCT_ERROR_INVALID_VALUE,
                              "the gathers of this group disagree across the communicators (or one failed its "
                              "checks): nothing was posted");
            } else {
                for (const Pending& p : c.queued) {
                    const hpdct_status e = post_plan(p);
                    if (st == HPDCT_SUCCESS) st = e;
                    t_decodes.insert(t_decodes.end(), p.decodes.begin(), p.decodes.end());
                }
            }
            c.clear();
        }
        t_cliques.clear();
    }
    const hpdct_status end = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    if (st == HPDCT_SUCCESS) st = end;
    if (t_group_depth == 0) {
        // the receives are enqueued now: the decodes go behind them on their streams
        const hpdct_status d = st == HPDCT_SUCCESS ? run_decodes(t_decodes) : (t_decodes.clear(), HPDCT_SUCCESS);
        if (st == HPDCT_SUCCESS) st = d;
    }
    return st;
}

hpdct_status hpdct_forward_slab(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                int64_t height, int64_t width, void* stream) {
    if (hpdct_status st = check_geometry(comm, height, width)) return st;
    int64_t first, rows;
    hpdct::dist::shard_rows(height, comm->size, comm->rank, first, rows);
    DeviceScope ds(comm->device);
    if (ds.err != hipSuccess) return hip_status(ds.err, "hipSetDevice");
    return hpdct_forward(d_slab, HPDCT_U8, d_coef_slab, out_type, rows, width, nullptr, 0u, stream);
}

hpdct_status hpdct_gather_rows(hpdct_comm comm, const void* d_slab, void* d_frame, hpdct_dtype type, int64_t height,
                               int64_t width, int root, void* stream) {
    return gather(comm, d_slab, d_frame, type, height, width, root, stream, RootSlab::kCopy, nullptr);
}

hpdct_status hpdct_gather_decode_i8(hpdct_comm comm, const int8_t* d_slab, int8_t* d_frame_i8, float* d_frame_f32,
                                    int64_t height, int64_t width, int root, void* stream) {
    return gather(comm, d_slab, d_frame_i8, HPDCT_I8, height, width, root, stream, RootSlab::kSkip, d_frame_f32);
}

hpdct_status hpdct_forward_sharded(hpdct_comm comm, const uint8_t* d_slab, void* d_coef_slab, hpdct_dtype out_type,
                                   void* d_frame, int64_t height, int64_t width, int root, void* stream) {
    if (hpdct_status st = hpdct_forward_slab(comm, d_slab, d_coef_slab, out_type, height, width, stream)) return st;
    return hpdct_gather_rows(comm, d_coef_slab, d_frame, out_type, height, width, root, stream);
}

}  // extern "C"
