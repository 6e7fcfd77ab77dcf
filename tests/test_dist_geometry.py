"""The gather geometry agreement of the RCCL row-shard layer
(csrc/hpdct_dist_geometry.hpp, used by hpdct_gather_rows before the first
gather of a geometry), on the CPU: a small C++ driver
packs each simulated rank's (height, width, type, root), reduces with the
element-wise max that ncclAllReduce(ncclMax) computes, and asks the same
decision function the library asks.  Every rank sees the same reduced vector,
so all ranks proceed or all refuse.  The integrated path (the all-reduce on a
real communicator) runs at world 1 on the GPU (tests/test_gpu_dist.py)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cuda-dct-idct_amd", "csrc")

DRIVER = r"""
#include <stdio.h>
#include <stdlib.h>
#include "hpdct_dist_geometry.hpp"
using namespace hpdct::dist;
// argv: groups of 4 numbers, one group per rank
int main(int argc, char** argv) {
    int ranks = (argc - 1) / 4;
    int64_t acc[kCheckWords];
    for (int i = 0; i < kCheckWords; ++i) acc[i] = INT64_MIN;
    for (int r = 0; r < ranks; ++r) {
        Geometry g{{atoll(argv[1 + 4 * r]), atoll(argv[2 + 4 * r]), atoll(argv[3 + 4 * r]), atoll(argv[4 + 4 * r])}};
        int64_t v[kCheckWords];
        pack_for_max(g, v);
        max_into(acc, v);
    }
    AgreedSet s;
    Geometry a{{16384, 16384, 2, 0}}, b{{16384, 16384, 1, 0}};
    s.add(a); s.add(a); s.add(b);
    if (!s.contains(a) || !s.contains(b) || s.seen.size() != 2) return 3;
    printf("%s\n", agree_after_max(acc) ? "agree" : "disagree");
    return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("geo")
    src = d / "geo.cpp"
    src.write_text(DRIVER)
    exe = d / "geo"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I", CSRC, str(src), "-o", str(exe)], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


def run(driver, *ranks):
    args = [str(v) for g in ranks for v in g]
    r = subprocess.run([driver] + args, capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_agreeing_ranks_proceed(driver):
    g = (16384, 16384, 2, 0)
    assert run(driver, g) == "agree"
    assert run(driver, *[g] * 8) == "agree"


@pytest.mark.parametrize("field", range(4))
def test_any_disagreeing_field_refuses(driver, field):
    g = [16384, 16384, 2, 0]
    bad = list(g)
    bad[field] += 8 if field < 2 else 1
    ranks = [tuple(g)] * 7 + [tuple(bad)]
    assert run(driver, *ranks) == "disagree"
    # the odd rank out in the middle, and a smaller value, too
    bad2 = list(g)
    bad2[field] -= 8 if field < 2 else 1
    ranks = [tuple(g)] * 3 + [tuple(bad2)] + [tuple(g)] * 4
    assert run(driver, *ranks) == "disagree"


def test_ragged_but_equal_geometry_agrees(driver):
    # ranks owning different row counts still pass the same frame geometry
    g = (16392, 520, 1, 0)
    assert run(driver, *[g] * 3) == "agree"


def test_library_uses_the_check():
    src = open(os.path.join(CSRC, "hpdct_dist.cpp")).read()
    assert '#include "hpdct_dist_geometry.hpp"' in src
    assert "check_agreement(comm, geo, s)" in src
    assert "ncclAllReduce(comm->d_check, comm->d_check, hpdct::dist::kCheckWords" in src
