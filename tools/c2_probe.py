"""C2 (1024^2 frames) launch-overhead probe (development tool, not the
product): per-frame time of back-to-back single-frame launches, of the same
launches captured in a HIP graph and replayed, and of frames stacked into one
launch.  Usage: python tools/c2_probe.py [frames_per_batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402


def per_frame_us(fn, frames_per_call, calls=200, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(calls):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (calls * frames_per_call)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = 1024
    dev = torch.device("cuda:0")
    hpdct.load_library()
    stack_in = torch.empty((nb * n, n), dtype=torch.uint8, device=dev)
    hpdct.fill_hash_u8(stack_in, seed=42)
    stack_out = torch.empty((nb * n, n), dtype=torch.float32, device=dev)
    frames_in = [stack_in[f * n:(f + 1) * n] for f in range(nb)]
    frames_out = [stack_out[f * n:(f + 1) * n] for f in range(nb)]
    single = [hpdct.bind("fwd", frames_in[f], frames_out[f]) for f in range(nb)]

    def loop():
        for c in single:
            c()
    res = {"single-frame launches, back to back": per_frame_us(loop, nb)}
    stacked = hpdct.bind("fwd", stack_in, stack_out)
    res[f"{nb} frames stacked, one launch"] = per_frame_us(stacked, nb)
    ref = stack_out.clone()
    # the same nb single-frame launches captured once and replayed
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        captured = [hpdct.bind("fwd", frames_in[f], frames_out[f]) for f in range(nb)]
        torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cap = [hpdct.bind("fwd", frames_in[f], frames_out[f]) for f in range(nb)]
        for c in cap:
            c()
    del captured
    stack_out.zero_()
    g.replay()
    torch.cuda.synchronize()
    res["graph check (bit-exact vs launches)"] = float(torch.equal(stack_out.view(torch.int32), ref.view(torch.int32)))
    res[f"graph of {nb} single-frame launches, replayed"] = per_frame_us(g.replay, nb)
    for k, v in res.items():
        print(f"{k:45s} {v:8.3f}", flush=True)


if __name__ == "__main__":
    main()
