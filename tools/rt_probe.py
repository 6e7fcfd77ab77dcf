"""Round-trip launch probe (development tool, not the product): times
hpdct_roundtrip_u8 at 8192^2 through the Python binding under several buffer
arrangements, to separate the kernel from its surroundings (sums memset,
recon-buffer reuse, input content).  Usage: python tools/rt_probe.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

import torch  # noqa: E402
import hpdct  # noqa: E402


def timeit(calls, steps=100, warmup=8):
    for i in range(warmup):
        calls[i % len(calls)]()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(steps):
        calls[i % len(calls)]()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps * 1e3  # us per launch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    dev = torch.device("cuda:0")
    hpdct.load_library()
    sets = 4
    imgs = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(sets)]
    for s, t in enumerate(imgs):
        hpdct.fill_hash_u8(t, seed=7 + s)
    coef = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(sets)]
    rec4 = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(sets)]
    sums = [torch.zeros(3, dtype=torch.int64, device=dev) for _ in range(sets)]
    res = {}
    res["fwd u8->f32 (headline)"] = timeit([hpdct.bind("fwd", imgs[s], coef[s]) for s in range(sets)])
    res["rt no sums, 4 recon"] = timeit([hpdct.bind_roundtrip(imgs[s], coef[s], rec4[s]) for s in range(sets)])
    res["rt sums, 4 recon, 1 sums buf"] = timeit(
        [hpdct.bind_roundtrip(imgs[s], coef[s], rec4[s], sums[0]) for s in range(sets)])
    res["rt sums, 4 recon, 4 sums bufs"] = timeit(
        [hpdct.bind_roundtrip(imgs[s], coef[s], rec4[s], sums[s]) for s in range(sets)])
    res["rt sums, 2 recon (bench layout)"] = timeit(
        [hpdct.bind_roundtrip(imgs[s], coef[s], rec4[s % 2], sums[0]) for s in range(sets)])
    res["rt sums only (no recon)"] = timeit([hpdct.bind_roundtrip(imgs[s], coef[s], None, sums[0]) for s in range(sets)])
    # the same after ~3 s of sustained load (the bench runs its extras after
    # the headline and the 3-launch baselines): clocks / power state
    heat = [hpdct.bind("fwd", imgs[s], coef[s]) for s in range(sets)]
    for i in range(60000):
        heat[i % sets]()
    res["rt sums, 4 recon, 4 sums bufs (after load)"] = timeit(
        [hpdct.bind_roundtrip(imgs[s], coef[s], rec4[s], sums[s]) for s in range(sets)])
    res["fwd u8->f32 (after load)"] = timeit([hpdct.bind("fwd", imgs[s], coef[s]) for s in range(sets)])
    T = torch.from_numpy(hpdct.default_transform()).to(dev)
    f32_in = [imgs[s].float() for s in range(2)]
    res["fwd f32 runtime-T, 2 sets"] = timeit(
        [hpdct.bind("fwd", f32_in[s], coef[s], transform=T) for s in range(2)])
    res["fwd f32 builtin-T, 2 sets"] = timeit([hpdct.bind("fwd", f32_in[s], coef[s]) for s in range(2)])
    f32_in += [imgs[s].float() for s in range(2, 4)]
    res["fwd f32 runtime-T, 4 sets"] = timeit(
        [hpdct.bind("fwd", f32_in[s], coef[s], transform=T) for s in range(4)])
    res["fwd f32 builtin-T, 4 sets"] = timeit([hpdct.bind("fwd", f32_in[s], coef[s]) for s in range(4)])
    for k, v in res.items():
        print(f"{k:40s} {v:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
