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


# ---- the posts of one gather (hpdct::dist::gather_plan, hpdct_dist.cpp's
# gather) and the init_all group check (clique_round_agrees) -----------------
PLAN_DRIVER = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "hpdct_dist_geometry.hpp"
using namespace hpdct::dist;
// plan <height> <width> <elem> <world> <root> <rank> <own: 0 copy, 1 in place, 2 skip>
// round <n_comms> then per comm: <failed> <count> <count x (h w type root)>
int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "plan")) {
        const auto plan = gather_plan(atoll(argv[2]), atoll(argv[3]), (size_t)atoll(argv[4]), atoi(argv[5]),
                                      atoi(argv[6]), atoi(argv[7]), (RootSlab)atoi(argv[8]));
        for (const Post& p : plan)
            printf("%d %d %lld %lld %llu %llu\n", (int)p.kind, p.peer, (long long)p.first_row, (long long)p.rows,
                   (unsigned long long)p.offset, (unsigned long long)p.bytes);
        return 0;
    }
    if (argc > 1 && !strcmp(argv[1], "round")) {
        int a = 2;
        const int n = atoi(argv[a++]);
        std::vector<std::vector<Geometry>> asked(n);
        std::vector<bool> failed(n);
        for (int c = 0; c < n; ++c) {
            failed[c] = atoi(argv[a++]) != 0;
            const int cnt = atoi(argv[a++]);
            for (int i = 0; i < cnt; ++i, a += 4)
                asked[c].push_back(Geometry{{atoll(argv[a]), atoll(argv[a + 1]), atoll(argv[a + 2]), atoll(argv[a + 3])}});
        }
        printf("%s\n", clique_round_agrees(asked, failed) ? "post" : "refuse");
        return 0;
    }
    if (argc > 1 && !strcmp(argv[1], "mode")) {
        // mode <height> <width> <elem> <world> <root> <rank> <own> <slab byte offset into the frame>
        static char frame[1];
        const char* slab = frame + atoll(argv[9]);
        printf("%d\n", (int)root_slab_mode((RootSlab)atoi(argv[8]), slab, frame, atoll(argv[2]), atoll(argv[3]),
                                           (size_t)atoll(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7])));
        return 0;
    }
    return 2;
}
"""


@pytest.fixture(scope="module")
def plan_driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("plan")
    src = d / "plan.cpp"
    src.write_text(PLAN_DRIVER)
    exe = d / "plan"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I", CSRC, str(src), "-o", str(exe)], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


def _plan(exe, height, width, elem, world, root, rank, own):
    r = subprocess.run([exe, "plan"] + [str(v) for v in (height, width, elem, world, root, rank, own)],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return [tuple(int(x) for x in line.split()) for line in r.stdout.split("\n") if line.strip()]


def _shard(height, world, rank):
    import importlib.util
    spec = importlib.util.spec_from_file_location("hpdct_dist_py", os.path.join(ROOT, "cuda-dct-idct_amd",
                                                                                 "hpdct_dist.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.shard_rows(height, world, rank)


SEND, RECV, COPY = 0, 1, 2


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("height", [16384, 16384 + 8 * 3, 8 * 8 + 8 * 5, 8 * 11])
@pytest.mark.parametrize("elem", [4, 1])
def test_gather_plan_every_post(plan_driver, world, height, elem):
    """Every (rank, first, rows, bytes) each rank posts, for equal and ragged
    slabs, every root, the root's own slab copied, in place or skipped (the
    int8 gather-decode): sends carry exactly the slab, the root receives every
    peer's rows at their offset, and the frame is tiled without gap or overlap."""
    if height // 8 < world:
        pytest.skip("fewer tile rows than ranks is refused by check_geometry")
    width = 8 * 7
    row_bytes = width * elem
    for root in range(world):
        for own in (0, 1, 2):
            covered = []
            for rank in range(world):
                plan = _plan(plan_driver, height, width, elem, world, root, rank, own)
                first, rows = _shard(height, world, rank)
                if rank != root:
                    assert plan == [(SEND, root, first, rows, 0, rows * row_bytes)]
                    continue
                expect = []
                for r in range(world):
                    f, n = _shard(height, world, r)
                    if r != root:
                        expect.append((RECV, r, f, n, f * row_bytes, n * row_bytes))
                    elif own == 0:
                        expect.append((COPY, r, f, n, f * row_bytes, n * row_bytes))
                assert plan == expect
                covered = [(p[4], p[4] + p[5]) for p in plan]
            if own != 0:  # the root's own rows are the one hole
                f, n = _shard(height, world, root)
                covered.append((f * row_bytes, (f + n) * row_bytes))
            covered.sort()
            assert covered[0][0] == 0 and covered[-1][1] == height * row_bytes
            assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


def _round(exe, comms):
    args = ["round", str(len(comms))]
    for failed, geos in comms:
        args += [str(int(failed)), str(len(geos))]
        for g in geos:
            args += [str(v) for v in g]
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_clique_round_posts_only_when_all_agree(plan_driver):
    """an init_all group is posted only when every communicator was
    asked for the same gathers in the same order and none failed its checks;
    interleaved rounds (fp32 then int8 on every communicator) are fine."""
    f32, i8 = (16384, 16384, 2, 0), (16384, 16384, 1, 0)
    assert _round(plan_driver, [(False, [f32])] * 8) == "post"
    assert _round(plan_driver, [(False, [f32, i8])] * 4) == "post"
    assert _round(plan_driver, [(False, [f32, i8])] * 3 + [(False, [i8, f32])]) == "refuse"
    assert _round(plan_driver, [(False, [f32])] * 3 + [(False, [])]) == "refuse"  # one communicator missing
    assert _round(plan_driver, [(False, [f32])] * 3 + [(True, [])]) == "refuse"   # one call failed its checks
    assert _round(plan_driver, [(False, [f32])] * 2 + [(False, [(16384, 16384, 2, 1)])]) == "refuse"


R_COPY, R_IN_PLACE, R_SKIP = 0, 1, 2  # hpdct::dist::RootSlab


def _mode(exe, height, width, elem, world, root, rank, own, slab_off):
    r = subprocess.run([exe, "mode"] + [str(v) for v in (height, width, elem, world, root, rank, own, slab_off)],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return int(r.stdout.strip())


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("elem", [4, 1])
def test_root_slab_in_place_only_at_its_own_rows(plan_driver, world, elem):
    """hpdct_gather_rows treats the root's slab as already
    in place only when it sits at the root's OWN rows of the frame.  A root
    other than 0 whose slab is the start of the frame (slab == frame) must
    copy it to its rows, or rank 0's receive overwrites it and the root's rows
    stay unwritten.  Every root, slab at the frame start and at its rows."""
    height, width = 8 * 13, 8 * 5
    for root in range(world):
        first, _ = _shard(height, world, root)
        at_rows = first * width * elem
        assert _mode(plan_driver, height, width, elem, world, root, root, R_COPY, at_rows) == R_IN_PLACE  # in place
        want_start = R_IN_PLACE if at_rows == 0 else R_COPY  # root 0: its rows ARE the frame start
        assert _mode(plan_driver, height, width, elem, world, root, root, R_COPY, 0) == want_start
        # the plan of a root > 0 with slab == frame copies its own rows
        if at_rows:
            plan = _plan(plan_driver, height, width, elem, world, root, root, R_COPY)
            assert (COPY, root, first, _shard(height, world, root)[1], at_rows,
                    _shard(height, world, root)[1] * width * elem) in plan
        # skip (the int8 gather-decode) and non-root ranks pass through
        assert _mode(plan_driver, height, width, elem, world, root, root, R_SKIP, 0) == R_SKIP
        for rank in range(world):
            if rank != root:
                assert _mode(plan_driver, height, width, elem, world, root, rank, R_COPY, at_rows) == R_COPY


def test_library_uses_root_slab_mode():
    src = open(os.path.join(CSRC, "hpdct_dist.cpp")).read()
    assert "hpdct::dist::root_slab_mode(own, d_slab, d_frame" in src
    assert "d_frame == d_slab ?" not in src
