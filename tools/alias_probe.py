"""Buffer-placement probe (development tool, not the product): kernels at
8192^2 with the output plane placed at a controlled byte distance from the
input plane (inside one pool per set), to see whether the relative HBM
placement of the streams a kernel reads and writes changes its time.
Usage: python tools/alias_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402

MiB = 1 << 20


def us_per_launch(calls, steps=64, warmup=8):
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
    n = 8192
    px = n * n
    T = torch.from_numpy(hpdct.default_transform()).to(dev)
    sets = 4
    # output start - input start, MiB (the fp32 input is 256 MiB, the u8 input 64 MiB)
    dists = [256, 257, 258, 264, 288, 320, 384, 512, 513, 768, 1024, 1025, 1280, 1536, 2048]
    pool_bytes = max(dists) * MiB + 4 * px + 4 * MiB
    pools = [torch.empty(pool_bytes, dtype=torch.uint8, device=dev) for _ in range(sets)]
    print(f"pool bases mod 256 MiB: {[p.data_ptr() % (256 * MiB) // MiB for p in pools]} MiB", flush=True)
    tmp = torch.empty((n, n), dtype=torch.uint8, device=dev)
    fin = [pools[s][:4 * px].view(torch.float32).view(n, n) for s in range(sets)]
    for s in range(sets):
        hpdct.fill_hash_u8(tmp, seed=s)
        fin[s].copy_(tmp.float())
    if len(sys.argv) > 1 and sys.argv[1] == "fwd":
        # adjacency (out = in + 256 MiB = right after the fp32 input) vs 1 MiB further, per forward variant
        for d in (256, 257, 256, 257):
            outs = [pools[s][d * MiB:d * MiB + 4 * px].view(torch.float32).view(n, n) for s in range(sets)]
            r = {}
            r["runtime-T"] = us_per_launch([hpdct.bind("fwd", fin[s], outs[s], transform=T) for s in range(sets)])
            r["builtin-T"] = us_per_launch([hpdct.bind("fwd", fin[s], outs[s]) for s in range(sets)])
            r["no-quant"] = us_per_launch([hpdct.bind("fwd", fin[s], outs[s], quantise=False) for s in range(sets)])
            hpdct.set_mapping("tile")
            r["tile runtime-T"] = us_per_launch(
                [hpdct.bind("fwd", fin[s], outs[s], transform=T) for s in range(sets)])
            hpdct.set_mapping("auto")
            print(f"out - in = {d:5d} MiB  " + "  ".join(f"{k} {v:7.2f}" for k, v in r.items()), flush=True)
        return
    for d in dists:
        outs = [pools[s][d * MiB:d * MiB + 4 * px].view(torch.float32).view(n, n) for s in range(sets)]
        f32 = us_per_launch([hpdct.bind("fwd", fin[s], outs[s], transform=T) for s in range(sets)])
        inv = us_per_launch([hpdct.bind("inv", fin[s], outs[s]) for s in range(sets)])
        # u8 -> fp32: the u8 input is the first 64 MiB of the pool (bytes of the fp32 plane)
        u8 = us_per_launch([hpdct.bind("fwd", pools[s][:px].view(n, n), outs[s]) for s in range(sets)])
        print(f"out - in = {d:5d} MiB   fwd f32 runtime-T {f32:8.2f}   inv f32 {inv:8.2f}   fwd u8->f32 {u8:8.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
