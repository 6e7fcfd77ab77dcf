"""Row-sharding of one large frame across the GPUs of a node (BASELINE config
C4, north_star "row-sharded across the 8 GPUs ... RCCL only for the final
gather").  The reference has no multi-GPU code; this is
the build's own layer.

8x8 tiles are independent, so a frame shards into horizontal slabs of whole
tile rows with no halo and no exchange during compute.  The only collective is
the final gather of the coefficient slabs to the root rank
(torch.distributed.gather: RCCL over xGMI with the "nccl" backend, gloo on
CPU for the tests).
"""
from __future__ import annotations

from typing import List, Tuple


def shard_rows(height: int, world: int, rank: int) -> Tuple[int, int]:
    """(first_row, rows) owned by `rank`: contiguous slabs of whole 8-row tile
    rows, sizes differing by at most one tile row (earlier ranks get the extra)."""
    if height % 8:
        raise ValueError("height must be a multiple of 8")
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    tile_rows = height // 8
    base, extra = divmod(tile_rows, world)
    first = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return first * 8, count * 8


def all_shards(height: int, world: int) -> List[Tuple[int, int]]:
    return [shard_rows(height, world, r) for r in range(world)]


def gather_slabs(local, height: int, width: int, root: int = 0, group=None):
    """Gather every rank's coefficient slab (rows x width, same dtype) into a
    full (height x width) tensor on `root`; returns it there, None elsewhere.

    Uses torch.distributed.gather when all slabs have the same size (the
    common case: height divisible by 8*world), else a send/recv fan-in.
    With the gloo backend, device tensors are staged through host memory
    (gloo's gather and point-to-point take host tensors); RCCL moves them
    device to device over xGMI."""
    import torch
    import torch.distributed as dist

    if local.device.type != "cpu" and dist.get_backend(group) == "gloo":
        full = gather_slabs(local.cpu(), height, width, root, group)
        return None if full is None else full.to(local.device)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    shards = all_shards(height, world)
    uniform = len({rows for _, rows in shards}) == 1
    full = None
    if rank == root:
        full = torch.empty((height, width), dtype=local.dtype, device=local.device)
    if uniform:
        parts = None
        if rank == root:
            parts = [full[r0:r0 + rows] for r0, rows in shards]
        dist.gather(local.contiguous(), gather_list=parts, dst=root, group=group)
        return full
    if rank == root:
        for r, (r0, rows) in enumerate(shards):
            if r == root:
                full[r0:r0 + rows].copy_(local)
            else:
                buf = torch.empty((rows, width), dtype=local.dtype, device=local.device)
                dist.recv(buf, src=r, group=group)
                full[r0:r0 + rows].copy_(buf)
        return full
    dist.send(local.contiguous(), dst=root, group=group)
    return None
