// hpdct_dist_geometry.hpp -- the host-side arithmetic of hpdct_dist.cpp:
// the row shards, the sends / receives / copies one gather posts on a rank,
// and the checks that the ranks agree on a gather.  Host-only C++ so the CPU
// tests can drive it without RCCL (tests/test_dist_geometry.py).
//
// A gather whose ranks disagree on (height, width, type, root) posts sends and
// receives of different sizes and RCCL waits forever.  Before the first
// gather of a geometry a communicator has not seen, every rank contributes
// g = (height, width, type, root) and -g to one max all-reduce of 8 int64;
// the ranks agree exactly when max(g) == -max(-g), i.e. max == min, in every
// field.  Every rank sees the same reduced vector, so either all proceed or
// all refuse: nobody is left waiting in the payload exchange.  Later gathers
// of an agreed geometry run without the check (payload only).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace hpdct {
namespace dist {

struct Geometry {
    int64_t v[4];  // height, width, element type, root
    bool operator==(const Geometry& o) const {
        return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2] && v[3] == o.v[3];
    }
};

constexpr int kCheckWords = 8;

inline void pack_for_max(const Geometry& g, int64_t (&out)[kCheckWords]) {
    for (int i = 0; i < 4; ++i) {
        out[i] = g.v[i];
        out[4 + i] = -g.v[i];
    }
}

// true when the max-reduced vector says every rank packed the same geometry
inline bool agree_after_max(const int64_t (&red)[kCheckWords]) {
    for (int i = 0; i < 4; ++i)
        if (red[i] != -red[4 + i]) return false;
    return true;
}

// element-wise max of one rank's packed vector into an accumulator (what
// ncclAllReduce(ncclMax) computes; used by the host tests)
inline void max_into(int64_t (&acc)[kCheckWords], const int64_t (&x)[kCheckWords]) {
    for (int i = 0; i < kCheckWords; ++i) acc[i] = x[i] > acc[i] ? x[i] : acc[i];
}

// Geometries one communicator has already agreed on (a handful at most:
// e.g. the fp32 and the int8 gather of one frame size).
struct AgreedSet {
    std::vector<Geometry> seen;
    bool contains(const Geometry& g) const {
        for (const Geometry& s : seen)
            if (s == g) return true;
        return false;
    }
    void add(const Geometry& g) {
        if (!contains(g)) seen.push_back(g);
    }
};

// (first_row, rows) of `rank` in a height-row frame: contiguous slabs of whole
// 8-row tile rows, earlier ranks take the extra tile row (hpdct_shard_rows)
inline void shard_rows(int64_t height, int world, int rank, int64_t& first, int64_t& rows) {
    const int64_t tile_rows = height / 8, base = tile_rows / world, extra = tile_rows % world;
    first = (rank * base + (rank < extra ? rank : extra)) * 8;
    rows = (base + (rank < extra ? 1 : 0)) * 8;
}

// One operation a rank posts for a gather.  kSend: the rank's slab to the
// root; kRecv (root): peer's slab into the frame at `offset` bytes; kCopy
// (root): its own slab into the frame at `offset`, device to device.
struct Post {
    enum Kind : int { kSend = 0, kRecv = 1, kCopy = 2 };
    Kind kind;
    int peer;
    int64_t first_row, rows;
    uint64_t offset, bytes;
};

// Root's own slab in a gather: copied into the frame, already there (no
// copy), or not part of this gather (the int8 gather-decode: the root wrote
// its slab as fp32 into the fp32 frame itself).
enum class RootSlab : int { kCopy = 0, kInPlace = 1, kSkip = 2 };

// The operations `rank` posts for a gather of a height x width frame of
// `elem`-byte elements to `root`, in posting order (the root: ranks 0..N-1).
inline std::vector<Post> gather_plan(int64_t height, int64_t width, size_t elem, int world, int root, int rank,
                                     RootSlab own) {
    std::vector<Post> plan;
    const uint64_t row_bytes = static_cast<uint64_t>(width) * elem;
    int64_t first, rows;
    if (rank != root) {
        shard_rows(height, world, rank, first, rows);
        plan.push_back({Post::kSend, root, first, rows, 0, static_cast<uint64_t>(rows) * row_bytes});
        return plan;
    }
    for (int r = 0; r < world; ++r) {
        shard_rows(height, world, r, first, rows);
        const uint64_t off = static_cast<uint64_t>(first) * row_bytes, bytes = static_cast<uint64_t>(rows) * row_bytes;
        if (r != root) {
            plan.push_back({Post::kRecv, r, first, rows, off, bytes});
        } else if (own == RootSlab::kCopy) {
            plan.push_back({Post::kCopy, r, first, rows, off, bytes});
        }
    }
    return plan;
}

// The mode gather_plan is called with on `rank`: a kCopy root whose slab
// already sits at its own rows of the frame (slab == frame + first * row
// bytes) needs no copy and posts nothing for itself, so a world-1 gather
// posts nothing at all; a slab anywhere else, e.g. at the start of the frame
// of a root whose first row is not 0, is copied.  Other ranks and modes pass
// through.
inline RootSlab root_slab_mode(RootSlab own, const void* slab, const void* frame, int64_t height, int64_t width,
                               size_t elem, int world, int root, int rank) {
    if (own != RootSlab::kCopy || rank != root || !slab || !frame) return own;
    int64_t first, rows;
    shard_rows(height, world, root, first, rows);
    const char* at = static_cast<const char*>(frame) + static_cast<uint64_t>(first) * static_cast<uint64_t>(width) * elem;
    return at == static_cast<const char*>(slab) ? RootSlab::kInPlace : RootSlab::kCopy;
}

// Communicators of one ncclCommInitAll (one thread, one group): the gathers
// each of them was asked for in the group, in call order.  The round may be
// posted only when every communicator was asked for the same sequence of
// geometries (gather i of every communicator alike) and none of the calls
// failed its own validation; otherwise nothing is posted anywhere.
inline bool clique_round_agrees(const std::vector<std::vector<Geometry>>& per_comm,
                                const std::vector<bool>& comm_failed) {
    if (per_comm.empty()) return true;
    for (size_t c = 0; c < per_comm.size(); ++c) {
        if (c < comm_failed.size() && comm_failed[c]) return false;
        if (per_comm[c].size() != per_comm[0].size()) return false;
        for (size_t i = 0; i < per_comm[c].size(); ++i)
            if (!(per_comm[c][i] == per_comm[0][i])) return false;
    }
    return true;
}

}  // namespace dist
}  // namespace hpdct
