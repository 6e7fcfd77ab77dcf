"""Sequence probe (development tool, not the product): the bench's order --
the headline loop, then the fp32 runtime-T forward loop repeated -- with
per-repeat timing, to see whether the first VALU-heavy loop after the
memory-bound headline runs slow (a transient) or every loop does.
Usage: python tools/seq_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402


def us_per_launch(calls, steps=100, warmup=5):
    for i in range(warmup):
        calls[i % len(calls)]()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(steps):
        calls[i % len(calls)]()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps * 1e3


def main():
    dev = torch.device("cuda:0")
    hpdct.load_library()
    n, sets = 8192, 4
    imgs = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(sets)]
    for s, t in enumerate(imgs):
        hpdct.fill_hash_u8(t, seed=s)
    print(f"headline {us_per_launch([hpdct.bind('fwd', imgs[s], outs[s]) for s in range(sets)], 200, 20):.2f} us",
          flush=True)
    T = torch.from_numpy(hpdct.default_transform()).to(dev)
    f32_in = [imgs[s].float() for s in range(sets)]
    calls = [hpdct.bind("fwd", f32_in[s], outs[s], transform=T) for s in range(sets)]
    for rep in range(4):
        print(f"fwd f32 runtime-T rep {rep}: {us_per_launch(calls):.2f} us", flush=True)
    time.sleep(1.0)
    print(f"fwd f32 runtime-T after 1 s idle: {us_per_launch(calls):.2f} us", flush=True)
    i8 = [torch.empty((n, n), dtype=torch.int8, device=dev) for _ in range(sets)]
    for rep in range(2):
        print(f"fwd u8->i8 rep {rep}: {us_per_launch([hpdct.bind('fwd', imgs[s], i8[s]) for s in range(sets)]):.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
