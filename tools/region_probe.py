"""Timed-region probe (development tool, not the product): how the bench's
20-launch headline region compares with the same kernel in steady state.
The bench times exactly K launches right after a host sync (the contract's
barrier + synchronize), so the GPU is idle for a moment before the first timed
launch.  Variants, each repeated and interleaved, 16 rotating sets as in the
bench:
  A  the bench's lead-in (>= 20 ms of launches, a sync every 16), sync, region
  B  lead-in without intermediate syncs, sync, region
  C  B, then P untimed launches after the sync, then the region (start event
     recorded behind them: the GPU is busy when the region starts)
and per-launch durations after an idle gap (an event after every launch).
Usage: python tools/region_probe.py [K=20] [reps=8]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402

LEAD_S = 0.02


def lead_in(calls, sync_every):
    t0, i = time.perf_counter(), 0
    while time.perf_counter() - t0 < LEAD_S:
        calls[i % len(calls)]()
        i += 1
        if sync_every and i % sync_every == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return i


def region(calls, k, prime=0):
    for i in range(prime):
        calls[i % len(calls)]()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(k):
        calls[i % len(calls)]()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k * 1e3


def per_launch(calls, n, idle_s):
    torch.cuda.synchronize()
    time.sleep(idle_s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record()
    for i in range(n):
        calls[i % len(calls)]()
        ev[i + 1].record()
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)]


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    hpdct.load_library()
    n, sets = 8192, 16
    imgs = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(sets)]
    for s, t in enumerate(imgs):
        hpdct.fill_hash_u8(t, seed=s)
    calls = [hpdct.bind("fwd", imgs[s], outs[s]) for s in range(sets)]
    variants = {
        "A bench lead-in (sync/16), sync, region": lambda: (lead_in(calls, 16), region(calls, k))[1],
        "B lead-in back to back, sync, region": lambda: (lead_in(calls, 0), region(calls, k))[1],
        "C B + 16 untimed launches after the sync": lambda: (lead_in(calls, 0), region(calls, k, 16))[1],
        "C B + 64 untimed launches after the sync": lambda: (lead_in(calls, 0), region(calls, k, 64))[1],
        "D A + 64 untimed launches after the sync": lambda: (lead_in(calls, 16), region(calls, k, 64))[1],
    }
    res = {name: [] for name in variants}
    for _ in range(reps):
        for name, fn in variants.items():
            res[name].append(fn())
    print(f"K = {k}, {reps} repetitions, us per launch (mean / median / min / max)")
    for name, v in res.items():
        print(f"  {name:44s} {statistics.fmean(v):7.2f} {statistics.median(v):7.2f} {min(v):7.2f} {max(v):7.2f}",
              flush=True)
    lead_in(calls, 0)
    sustained = region(calls, 2000)
    print(f"  steady state, 2000 launches back to back: {sustained:.2f} us")
    for idle in (0.0001, 0.001, 0.01):
        lead_in(calls, 0)
        d = per_launch(calls, 64, idle)
        print(f"  after {idle * 1e3:g} ms idle, per launch: first 8 " + " ".join(f"{x:.1f}" for x in d[:8]) +
              f" | 9-20 mean {statistics.fmean(d[8:20]):.2f} | 21-64 mean {statistics.fmean(d[20:]):.2f}",
              flush=True)


if __name__ == "__main__":
    main()
