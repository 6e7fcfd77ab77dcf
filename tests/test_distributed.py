"""Row-sharded multi-rank path (hpdct_dist) on CPU with the gloo backend.

The N>1 bench path shards a frame into 8-row-aligned slabs, runs the forward
kernel per slab on each GPU and gathers the coefficient slabs to rank 0 (RCCL
on the GPU node).  Here the same shard/gather code runs over gloo with
world_size 2 and 3; each rank computes its slab with the CPU oracle (the
checker: there is no GPU in this container) and rank 0 checks that the
gathered frame equals the oracle's unsharded result bit for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from hpdct_dist import all_shards, shard_rows  # noqa: E402


@pytest.mark.parametrize("height,world", [(8, 1), (64, 2), (72, 2), (16384, 8), (8192, 3), (40, 8), (800, 7)])
def test_shard_rows_partition(height, world):
    shards = all_shards(height, world)
    assert shards[0][0] == 0
    for (r0, rows), (n0, _) in zip(shards, shards[1:]):
        assert n0 == r0 + rows
    assert shards[-1][0] + shards[-1][1] == height
    assert all(r0 % 8 == 0 and rows % 8 == 0 for r0, rows in shards)
    sizes = [rows for _, rows in shards]
    assert max(sizes) - min(sizes) <= 8


def test_shard_rows_rejects_bad_input():
    with pytest.raises(ValueError):
        shard_rows(12, 2, 0)
    with pytest.raises(ValueError):
        shard_rows(16, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, height, width, result_path, wire_int8=False):
    import torch
    import torch.distributed as dist
    import oracle
    from hpdct_dist import gather_slabs, shard_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r0, rows = shard_rows(height, world, rank)
        # same stateless generator the bench uses on the device (C4)
        slab = oracle.hash_u8(rows * width, seed=42, first_index=r0 * width).reshape(rows, width)
        coef = torch.from_numpy(oracle.fdct(slab))
        if wire_int8:  # the C4 int8 wire format: |q| <= 98, decoded to fp32 on the root
            coef = coef.to(torch.int8)
        full = gather_slabs(coef, height, width, root=0)
        if rank == 0:
            ref = oracle.fdct(oracle.hash_u8(height * width, seed=42).reshape(height, width))
            if wire_int8:
                ok = np.array_equal(full.float().numpy(), ref)  # by value: the wire drops the sign of -0.0
            else:
                ok = np.array_equal(full.numpy().view(np.uint32), ref.view(np.uint32))
            with open(result_path, "w") as fh:
                fh.write("ok" if ok else "mismatch")
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,height,width,wire", [(2, 64, 96, False), (2, 72, 40, False), (3, 80, 64, False),
                                                     (2, 64, 96, True), (3, 72, 16, True),
                                                     # the node size of the C4 run: uniform slabs (gather) and
                                                     # ragged slabs (send/recv fan-in)
                                                     (8, 128, 64, False), (8, 136, 32, True)])
def test_sharded_gather_equals_unsharded(tmp_path, world, height, width, wire):
    import torch.multiprocessing as mp
    result = tmp_path / "result.txt"
    mp.spawn(_worker, args=(world, _free_port(), height, width, str(result), wire), nprocs=world, join=True)
    assert result.read_text() == "ok"


# ---- the native row-shard layer (include/hpdct_dist.h, libhpdct_dist.so) ----
# Host-only parts run here: the library loads (with librccl) and exports
# every declared symbol, its partition equals hpdct_dist.shard_rows, and bad
# arguments are rejected before any device work.  The RCCL gather itself
# runs in tests/test_gpu_dist.py.




@pytest.mark.parametrize("height,world", [(8, 1), (64, 2), (72, 2), (16384, 8), (8192, 3), (40, 8), (800, 7)])
def test_native_shard_rows_equals_python(height, world):
    import hpdct
    for r in range(world):
        assert hpdct.shard_rows_native(height, world, r) == shard_rows(height, world, r)


def test_native_dist_rejects_bad_arguments():
    import hpdct
    for h, w, r in ((12, 2, 0), (0, 1, 0), (16, 2, 2), (16, 0, 0), (16, 2, -1)):
        with pytest.raises(hpdct.HpdctError):
            hpdct.shard_rows_native(h, w, r)
    lib = hpdct.load_dist_library()
    # null communicator: refused with a status, no device touched
    assert lib.hpdct_gather_rows(None, None, None, 2, 64, 64, 0, None) == 1
    assert lib.hpdct_forward_slab(None, None, None, 2, 64, 64, None) == 1
    assert lib.hpdct_comm_rank(None) == -1 and lib.hpdct_comm_size(None) == -1
    assert lib.hpdct_comm_destroy(None) == 0
    with pytest.raises(hpdct.HpdctError):
        hpdct.Comm.init_rank(1, b"x" * 10, 0, 0)


# ---- the C4 leg's self-check of who took part (bench.c4_identity) -----------
def _identity_worker(rank, world, port, result_path):
    import json
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 16384
        _, rows = shard_rows(n, world, rank)
        # what the native RCCL leg records (communicator size == world) and
        # the gloo rehearsal (no communicator)
        native = bench.c4_identity(world, dist.get_world_size(), world, rank, n, rows)
        rehearsal = bench.c4_identity(world, dist.get_world_size(), None, rank, n, rows)
        refused = []
        for bad in ((world + 1, dist.get_world_size(), world), (world, dist.get_world_size(), world - 1)):
            try:
                bench.c4_identity(bad[0], bad[1], bad[2], rank, n, rows)
            except RuntimeError as e:
                refused.append(str(e))
        out = [None] * world
        dist.all_gather_object(out, {"native": native, "rehearsal": rehearsal, "refused": len(refused)})
        if rank == 0:
            with open(result_path, "w") as fh:
                json.dump(out, fh)
    finally:
        dist.destroy_process_group()


def test_c4_line_carries_the_rank_count_world2(tmp_path):
    """the C4 leg records rccl_nranks (hpdct_comm_size) and
    pg_world (dist.get_world_size()), fails loudly when either differs from
    --gpus, and on the root records gather_bytes_to_root = (N-1)/N of the
    fp32 frame: a two-rank gloo group assembles the fields the line carries."""
    import json
    import torch.multiprocessing as mp
    result = tmp_path / "identity.json"
    mp.spawn(_identity_worker, args=(2, _free_port(), str(result)), nprocs=2, join=True)
    got = json.loads(result.read_text())
    n = 16384
    for rank, r in enumerate(got):
        assert r["native"]["pg_world"] == 2 and r["native"]["rccl_nranks"] == 2
        assert r["rehearsal"]["rccl_nranks"] is None and r["rehearsal"]["pg_world"] == 2
        assert r["refused"] == 2
        if rank == 0:
            assert r["native"]["gather_bytes_to_root"] == n * n * 4 // 2 == r["native"]["gather_bytes_expected"]
        else:
            assert r["native"]["gather_bytes_to_root"] is None


@pytest.mark.parametrize("world", [1, 4, 8])
def test_c4_identity_root_bytes(world):
    sys.path.insert(0, ROOT)
    import bench
    n = 16384
    _, rows = shard_rows(n, world, 0)
    ident = bench.c4_identity(world, world, world, 0, n, rows)
    assert ident["gather_bytes_to_root"] == n * n * 4 * (world - 1) // world == ident["gather_bytes_expected"]
