// hpdct_dist_geometry.hpp -- the gather geometry agreement test of
// hpdct_dist.cpp, host-only C++ so the CPU tests can drive it without RCCL
// (tests/test_dist_geometry.py).
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

}  // namespace dist
}  // namespace hpdct
