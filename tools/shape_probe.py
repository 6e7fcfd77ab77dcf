"""Frame-shape probe (development tool, not the product): forward u8 -> fp32
time per 64 Mpx for frames of the same pixel count and different widths, to
see whether the row stride matters.  Usage: python tools/shape_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402


def us_per_launch(calls, steps=80, warmup=8):
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
    shapes = [(8192, 8192), (4096, 16384), (2048, 32768), (16384, 4096), (8192, 8200), (4096, 16392),
              (16384, 16384), (2048, 16384), (2048, 16392)]
    if len(sys.argv) > 1 and sys.argv[1] == "video":
        # common video widths (not multiples of 512 px) against power-of-2 neighbours
        shapes = [(32768, 1024), (32768, 1280), (16384, 1920), (16384, 2048), (8192, 3840), (8192, 4096),
                  (4320, 7680), (4096, 8192)]
    steps = 80
    if len(sys.argv) > 1 and sys.argv[1] == "pmc":
        # short runs for counter passes (tools/pmc_limits.sh): one shape per row stride
        shapes = [(8192, 8192), (16384, 4096), (4096, 16384), (2048, 16384), (16384, 16384)]
        steps = 16
    if len(sys.argv) > 1 and sys.argv[1] == "ab":
        shapes = [(8192, 8192), (2048, 16384), (16384, 1920), (32768, 1280), (8192, 8200)]
    if len(sys.argv) > 1 and sys.argv[1] == "f32":
        # fp32 -> fp32 forward with the caller's T (the compat path's kernel) and
        # the fp32 inverse, power-of-two vs video widths
        T = torch.from_numpy(hpdct.default_transform()).to(dev)
        for h, w in [(32768, 1024), (32768, 1280), (16384, 2048), (16384, 1920), (8192, 4096), (8192, 3840),
                     (8192, 8192), (8192, 8200)]:
            ins = [torch.empty((h, w), dtype=torch.uint8, device=dev) for _ in range(4)]
            for s_, t in enumerate(ins):
                hpdct.fill_hash_u8(t, seed=s_)
            f32 = [t.float() for t in ins]
            del ins
            outs = [torch.empty((h, w), dtype=torch.float32, device=dev) for _ in range(4)]
            # each measured after an untimed pass of the same loop (steady clocks: tools/seq_probe.py)
            fcalls = [hpdct.bind("fwd", f32[s_], outs[s_], transform=T) for s_ in range(4)]
            us_per_launch(fcalls)
            fw = us_per_launch(fcalls)
            icalls = [hpdct.bind("inv", outs[s_], f32[s_]) for s_ in range(4)]
            us_per_launch(icalls)
            iv = us_per_launch(icalls)
            px = h * w
            print(f"{h:6d} x {w:6d}  fwd f32 runtime-T {fw * 64 * 2**20 / px:8.2f}  inv f32 {iv * 64 * 2**20 / px:8.2f}"
                  "  us per 64 Mpx", flush=True)
            del f32, outs
            torch.cuda.empty_cache()
        return
    for h, w in shapes:
        sets = 4
        ins = [torch.empty((h, w), dtype=torch.uint8, device=dev) for _ in range(sets)]
        for s, t in enumerate(ins):
            hpdct.fill_hash_u8(t, seed=s)
        outs = [torch.empty((h, w), dtype=torch.float32, device=dev) for _ in range(sets)]
        us = us_per_launch([hpdct.bind("fwd", ins[s], outs[s]) for s in range(sets)], steps=steps)
        px = h * w
        print(f"{h:6d} x {w:6d}  {us:9.2f} us  {us * 64 * 2**20 / px:8.2f} us per 64 Mpx  "
              f"{5 * px / us / 1e6:7.3f} TB/s", flush=True)
        del ins, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
