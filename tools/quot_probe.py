"""Quotient-path probe (development tool, not the product): the fp32 ->
fp32 forward with the caller's T, with the standard JPEG table (integers:
the range-checked 3-op quotient) and with the same table + 0.5 (not integers:
IEEE division throughout), steady-state, at several widths.
Usage: python tools/quot_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import hpdct  # noqa: E402


def us_per_launch(calls, steps=64, warmup=64):
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
    T = torch.from_numpy(hpdct.default_transform()).to(dev)
    q_int = hpdct.default_quant_table().astype(np.float32)
    q_frac = q_int + np.float32(0.5)
    for h, w in [(8192, 8192), (8192, 4096), (16384, 2048), (32768, 1024)]:
        tmp = torch.empty((h, w), dtype=torch.uint8, device=dev)
        ins, outs = [], []
        for s in range(4):
            hpdct.fill_hash_u8(tmp, seed=s)
            ins.append(tmp.float())
            outs.append(torch.empty((h, w), dtype=torch.float32, device=dev))
        res = {}
        for name, q in (("int Q (checked 3-op)", q_int), ("Q+0.5 (IEEE)", q_frac), ("int Q again", q_int)):
            hpdct.set_quant_table(q)
            res[name] = us_per_launch([hpdct.bind("fwd", ins[s], outs[s], transform=T) for s in range(4)])
        hpdct.set_quant_table(q_int)
        px = h * w
        print(f"{h:6d} x {w:6d}  " + "  ".join(f"{k} {v * 64 * 2**20 / px:7.2f}" for k, v in res.items()) +
              "  us per 64 Mpx", flush=True)
        del ins, outs, tmp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
