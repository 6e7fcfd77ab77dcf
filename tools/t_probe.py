"""Caller's-T probe (development tool, not the product): fp32 -> fp32
forward and inverse (duo kernels) with no T (built-in), with the caller's
standard T (bitwise the built-in one: the kernel takes the immediate-operand
code), and with a T one ulp away in one zero entry (the generic runtime-T
code), steady-state, at several frame shapes.  Usage: python tools/t_probe.py"""
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
    t_std = hpdct.default_transform()
    t_off = t_std.copy()
    zero = np.argwhere(t_off == 0.0)[0]
    t_off[tuple(zero)] = np.float32(1e-45)  # smallest denormal: a different T, same work
    Ts = {"builtin (no T)": None, "caller's std T": torch.from_numpy(t_std).to(dev),
          "caller's other T": torch.from_numpy(t_off).to(dev)}
    for h, w in [(8192, 8192), (4096, 4096), (8192, 4096), (32768, 1024)]:
        tmp = torch.empty((h, w), dtype=torch.uint8, device=dev)
        ins, outs = [], []
        for s in range(4):
            hpdct.fill_hash_u8(tmp, seed=s)
            ins.append(tmp.float())
            outs.append(torch.empty((h, w), dtype=torch.float32, device=dev))
        px = h * w
        line = f"{h:6d} x {w:6d}"
        for name, T in Ts.items():
            fw = us_per_launch([hpdct.bind("fwd", ins[s], outs[s], transform=T) for s in range(4)])
            iv = us_per_launch([hpdct.bind("inv", outs[s], ins[s], transform=T) for s in range(4)])
            line += f"  | {name}: fwd {fw * 64 * 2**20 / px:6.2f} inv {iv * 64 * 2**20 / px:6.2f}"
        print(line + "  (us per 64 Mpx)", flush=True)
        del ins, outs, tmp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
