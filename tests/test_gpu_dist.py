"""The native row-shard layer over RCCL (include/hpdct_dist.h,
libhpdct_dist.so) on the GPU, at world size 1 (the GPU box has one MI355X):

  - a communicator from ncclCommInitAll and one from a unique id +
    ncclCommInitRank;
  - hpdct_forward_slab + hpdct_gather_rows of fp32 and int8 coefficients and
    of uint8 pixels, bit-exact against hpdct_forward of the whole frame (at
    world 1 the root's slab is the frame: the gather copies it device to
    device into the root's frame buffer);
  - the single-process multi-device driver `benchmark_hpdct <n> --gpus 1`
    (ncclCommInitAll, slab forward, RCCL gather, byte compare);
  - bench.py's process-group path at WORLD_SIZE=1 (init_process_group("nccl"),
    device-tensor all_reduce) with its C4 leg on the native gather.

The world-size >= 2 flow of the same partition runs over gloo on the CPU
(tests/test_distributed.py) and with the HIP kernel in two processes on one
GPU (tests/test_gpu_configs.py); RCCL ranks need a GPU each.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def comm1(hp, dev):
    c = hp.Comm.init_all([dev.index])[0]
    assert (c.rank, c.size, c.device) == (0, 1, dev.index)
    yield c
    c.destroy()


@pytest.mark.parametrize("out_dtype", ["float32", "int8"])
@pytest.mark.parametrize("h,w", [(2048, 4096), (1032, 520)])
def test_world1_slab_forward_and_gather_equal_forward(hp, dev, comm1, out_dtype, h, w):
    import torch
    x = torch.empty((h, w), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=11)
    dt = getattr(torch, out_dtype)
    slab = torch.empty((h, w), dtype=dt, device=dev)
    frame = torch.full((h, w), 3, dtype=dt, device=dev)
    hp.forward_slab(comm1, x, slab, h, w)
    hp.gather_rows(comm1, slab, frame, h, w, root=0)
    ref = hp.forward(x, out_dtype=dt)
    torch.cuda.synchronize()
    if dt == torch.float32:
        assert torch.equal(slab.view(torch.int32), ref.view(torch.int32))
        assert torch.equal(frame.view(torch.int32), ref.view(torch.int32))
    else:
        assert torch.equal(slab, ref) and torch.equal(frame, ref)


def test_world1_gather_uint8_pixels(hp, dev, comm1):
    import torch
    x = torch.randint(0, 256, (64, 128), dtype=torch.uint8, device=dev)
    frame = torch.zeros_like(x)
    hp.gather_rows(comm1, x, frame, 64, 128, root=0)
    torch.cuda.synchronize()
    assert torch.equal(frame, x)


def test_world1_comm_from_unique_id(hp, dev):
    import torch
    uid = hp.comm_unique_id()
    assert len(uid) == hp.UNIQUE_ID_BYTES
    c = hp.Comm.init_rank(1, uid, 0, dev.index)
    try:
        x = torch.empty((512, 1024), dtype=torch.uint8, device=dev)
        hp.fill_hash_u8(x, seed=3)
        slab = torch.empty((512, 1024), dtype=torch.float32, device=dev)
        frame = torch.empty_like(slab)
        hp.forward_slab(c, x, slab, 512, 1024)
        hp.gather_rows(c, slab, frame, 512, 1024, root=0)
        torch.cuda.synchronize()
        assert torch.equal(frame.view(torch.int32), hp.forward(x).view(torch.int32))
    finally:
        c.destroy()


def test_world1_unique_id_comm_checks_each_new_geometry(hp, dev):
    """A per-process communicator runs the geometry agreement all-reduce
    (hpdct_dist_geometry.hpp) before the first gather of every new
    (height, width, type, root), then gathers payload only: fp32, int8 and
    again fp32 at one size, then a second size, all correct."""
    import torch
    c = hp.Comm.init_rank(1, hp.comm_unique_id(), 0, dev.index)
    try:
        for (h, w) in ((256, 512), (256, 512), (64, 1024)):
            x = torch.empty((h, w), dtype=torch.uint8, device=dev)
            hp.fill_hash_u8(x, seed=h + w)
            for dt in (torch.float32, torch.int8, torch.float32):
                slab = hp.forward(x, out_dtype=dt)
                frame = torch.zeros_like(slab)
                hp.gather_rows(c, slab, frame, h, w, root=0)
                torch.cuda.synchronize()
                assert torch.equal(frame, slab)
    finally:
        c.destroy()


def test_world1_root_slab_in_place_is_a_no_op(hp, dev, comm1):
    """The root's slab computed in place in the frame (bench C4 leg): at world
    1 the gather moves nothing and leaves the frame as computed."""
    import torch
    x = torch.empty((512, 1024), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=9)
    frame = torch.empty((512, 1024), dtype=torch.float32, device=dev)
    hp.forward_slab(comm1, x, frame, 512, 1024)
    hp.gather_rows(comm1, frame, frame, 512, 1024, root=0)
    torch.cuda.synchronize()
    assert torch.equal(frame.view(torch.int32), hp.forward(x).view(torch.int32))


@pytest.mark.parametrize("n", [1024 * 1024, 4096 * 4096 + 8, 1000, 0])
def test_decode_int8_to_fp32(hp, dev, n):
    """The root-side decode of the int8 wire format (hpdct_decode_i8_f32):
    out = (float)q for every int8 value, whole 1 KiB wave blocks and a
    ragged tail."""
    import torch
    q = torch.randint(-128, 128, (n,), dtype=torch.int8, device=dev)
    out = torch.full((n,), 7.0, dtype=torch.float32, device=dev)
    hp.decode_i8_f32(q, out)
    torch.cuda.synchronize()
    assert torch.equal(out, q.float())


def test_decode_equals_fp32_forward_by_value(hp, dev):
    import torch
    x = torch.empty((2048, 4096), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=21)
    q8 = hp.forward(x, out_dtype=torch.int8)
    f = hp.forward(x)
    d = hp.decode_i8_f32(q8)
    torch.cuda.synchronize()
    assert torch.equal(d, f)  # value equality: -0.0 in f decodes as +0.0


def test_world1_gather_rejects_bad_root(hp, dev, comm1):
    import torch
    s = torch.empty((64, 64), dtype=torch.float32, device=dev)
    with pytest.raises(hp.HpdctError):
        hp.gather_rows(comm1, s, s.clone(), 64, 64, root=1)


def test_world1_gather_decode_int8_root_slab_fp32_in_place(hp, dev, comm1):
    """The int8 wire's gather (hpdct_gather_decode_i8): the
    root computes its own slab as fp32 in place in the fp32 frame and passes no
    int8 slab; at world 1 there are no peers, so nothing is received or
    decoded and the int8 scratch frame is left untouched."""
    import torch
    h, w = 1032, 520
    x = torch.empty((h, w), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=5)
    frame = torch.empty((h, w), dtype=torch.float32, device=dev)
    frame8 = torch.full((h, w), 7, dtype=torch.int8, device=dev)
    hp.forward_slab(comm1, x, frame, h, w)
    hp.gather_decode_i8(comm1, None, frame8, frame, h, w, root=0)
    torch.cuda.synchronize()
    assert torch.equal(frame.view(torch.int32), hp.forward(x).view(torch.int32))
    assert bool((frame8 == 7).all())
    # the same through a per-process communicator (its agreement all-reduce first)
    c = hp.Comm.init_rank(1, hp.comm_unique_id(), 0, dev.index)
    try:
        hp.gather_decode_i8(c, None, frame8, frame, h, w, root=0)
        torch.cuda.synchronize()
        assert torch.equal(frame.view(torch.int32), hp.forward(x).view(torch.int32))
    finally:
        c.destroy()


def test_world1_group_posts_queued_gathers_at_group_end(hp, dev, comm1):
    """init_all communicators inside hpdct_group_start/end: the gathers are
    queued and posted at hpdct_group_end once the round agrees:
    two gathers (fp32, then int8) in one group land after the group end."""
    import torch
    x = torch.empty((256, 512), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=17)
    f32, i8 = hp.forward(x), hp.forward(x, out_dtype=torch.int8)
    fr32, fr8 = torch.zeros_like(f32), torch.zeros_like(i8)
    torch.cuda.synchronize()
    hp.group_start()
    hp.gather_rows(comm1, f32, fr32, 256, 512, root=0)
    hp.gather_rows(comm1, i8, fr8, 256, 512, root=0)
    hp.group_end()
    torch.cuda.synchronize()
    assert torch.equal(fr32.view(torch.int32), f32.view(torch.int32)) and torch.equal(fr8, i8)


def test_world1_group_with_a_failed_gather_posts_nothing(hp, dev, comm1):
    """A gather that fails its own checks inside a group fails the whole
    round: hpdct_group_end posts none of the group's gathers and reports the
    error (nothing is left waiting on a peer)."""
    import torch
    good = torch.full((64, 64), 5.0, dtype=torch.float32, device=dev)
    frame = torch.zeros_like(good)
    hp.group_start()
    hp.gather_rows(comm1, good, frame, 64, 64, root=0)
    with pytest.raises(hp.HpdctError):
        hp.gather_rows(comm1, good, frame, 64, 64, root=1)
    with pytest.raises(hp.HpdctError):
        hp.group_end()
    torch.cuda.synchronize()
    assert bool((frame == 0).all())
    # the next group starts clean
    hp.group_start()
    hp.gather_rows(comm1, good, frame, 64, 64, root=0)
    hp.group_end()
    torch.cuda.synchronize()
    assert torch.equal(frame, good)


def test_driver_sharded_mode_one_gpu():
    exe = os.path.join(ROOT, "cuda-dct-idct_amd", "bin", "benchmark_hpdct")
    r = subprocess.run([exe, "4096", "3", "--gpus", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-exact yes" in r.stdout, r.stdout
    r = subprocess.run([exe, "2048", "--gpus", "1", "--int8"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "int8" in r.stdout and "bit-exact yes" in r.stdout, r.stdout + r.stderr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_nccl_process_group_at_world_size_1(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5", "--warmup", "2",
           "--size", "2048", "--sets", "4", "--no-cpu-baseline", "--sustain-s", "0", "--c4-size", "2048",
           "--c5-size", "512", "--c5-frames", "8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c4 = line["extras"]["c4"]
    assert c4["gather_path"].startswith("native RCCL"), c4
    assert c4["sharded_equals_unsharded"] is True
    assert c4["int8_wire_equals_fp32"] is True
    for k in (2, 4, 8):
        assert c4[f"predicted_compute_speedup_{k}"] > 0 and line[f"c4_predicted_compute_speedup_{k}"] > 0
    assert c4["gather_bytes_to_root"] == 0 and c4["gather_ms"] < 1.0
    assert c4["end_to_end_ms"] > 0 and c4["end_to_end_int8_ms"] > 0 and c4["decode_int8_ms"] > 0
    # world 1: the root's slab is fp32 in place for the int8 wire too, nothing is decoded
    assert c4["decoded_rows_on_root"] == 0 and c4["gather_int8_bytes_to_root"] == 0
    assert c4["decode_int8_sets"] >= 2
    assert line["parity_spot_check"] is True
    assert line["provenance"]["lib_matches_sources"] is True
    # the line says who took part in the gather
    assert c4["rccl_nranks"] == 1 and c4["pg_world"] == 1 and c4["gather_bytes_expected"] == 0
    assert line["c4_rccl_nranks"] == 1 and line["c4_pg_world"] == 1
    # every kernel beside its copy ceiling, at the end of the line
    ks = line["kernel_status"]
    assert list(line)[-1] == "kernel_status"
    for key in ("headline_fwd_u8_f32", "fwd_u8_i8", "inv_f32_f32", "dropin.dct_all_blocks_cuda", "c3.one_pass"):
        us, ceil, frac, status = ks[key]
        assert us > 0 and ceil > 0 and frac == round(ceil / us, 3) and status in ("done", "open")


def test_bench_watchdog_exits_nonzero_after_the_headline_line(tmp_path):
    """when the extras watchdog fires (a hung C4 gather, say), rank 0
    still prints the headline line, with extras.error set, and the process
    exits 3, not 0, so a caller that checks the exit code sees the hang."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5", "--warmup", "2",
           "--size", "2048", "--sets", "4", "--no-cpu-baseline", "--sustain-s", "0", "--extras-timeout-s", "0.5"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 3, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert "watchdog" in line["extras"]["error"] and line["value"] > 0
