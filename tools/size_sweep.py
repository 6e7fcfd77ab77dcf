"""Per-size forward timing on MI355X, the reference README's benchmark table
(README.md:46-60: HpApprDCT / fastApprDCT forward at 256^2 .. 8192^2 on a T4).

Columns per size (ms per frame):
  driver   the reference's own measurement method: benchmark_hpdct (the
           HIP-native benchmark_newAppr.cu) prints the event-timed single-call
           "DCT"/"IDCT" lines of the compat entry points; mean of warm runs
Back-to-back launches over rotating buffers (Python launch rate bounds the
smallest sizes at ~3.5 us):
  compat   dct_all_blocks_cuda's data path: fp32 image (X-128 written back in
           place, as the reference's sub_matrix_scalar does), the caller's T
           in device memory, fp32 quantised coefficients -- the reference's
           timed region (3 kernels) as one launch of this build
  u8       the native u8 -> fp32 path (headline kernel / octet for small frames)
  ref3     the reference's own 3-launch structure re-expressed in HIP
           (hpdct_baseline.h, A/B only)
  fast3    the fastApprDCT 3-launch structure (A/B only)
Small frames are served from the Infinity Cache; the T4 column is copied from
the reference README for comparison, not measured here.

usage: python tools/size_sweep.py [sizes...]   (prints a markdown table)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

T4_HPAPPR_MS = {256: 0.07, 512: 0.12, 1024: 0.30, 2048: 1.04, 4096: 4.00, 8192: 14.70}  # README.md:50-55
T4_FASTAPPR_MS = {8192: 20.00}  # README.md:55


def driver_ms(n, runs=21):
    """The reference's own measurement, through the HIP-native driver
    (benchmark_hpdct = benchmark_newAppr.cu): the compat entry point's
    event-timed "DCT (n,n): x ms" / "IDCT" lines, mean over runs 2..N (run 1
    includes loading the code object).  Child process, started before this
    process touches the GPU."""
    import re
    import subprocess
    exe = os.path.join(ROOT, "cuda-dct-idct_amd", "bin", "benchmark_hpdct")
    out = subprocess.run([exe, str(n), str(runs)], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, HPDCT_COMPAT_QUIET="0")).stdout
    dct = [float(x) for x in re.findall(r"^DCT \(\d+,\d+\): ([0-9.]+) ms", out, re.M)]
    idct = [float(x) for x in re.findall(r"^IDCT \(\d+,\d+\): ([0-9.]+) ms", out, re.M)]
    mean = lambda v: sum(v[1:]) / max(1, len(v) - 1)  # noqa: E731
    return mean(dct), mean(idct)


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [256, 512, 1024, 2048, 4096, 8192]
    drv = {n: driver_ms(n) for n in sizes}

    import torch
    import hpdct

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    T = torch.from_numpy(hpdct.default_transform()).to(dev)
    print("| size | T4 HpApprDCT fwd (README) | MI355X `benchmark_hpdct` DCT / IDCT (reference method) | "
          "MI355X compat fp32, back-to-back | MI355X u8→fp32, back-to-back | MI355X reference 3-launch | "
          "MI355X fastApprDCT 3-launch | DCT speed-up vs T4 |")
    print("|---|---|---|---|---|---|---|---|")
    for n in sizes:
        px = n * n
        sets = max(2, min(8, (1 << 30) // (9 * px)))  # > 1 GiB of buffers where it fits
        img8 = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(sets)]
        for s, t in enumerate(img8):
            hpdct.fill_hash_u8(t, seed=42 + s)
        imgf = [t.float() for t in img8]
        outs = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(sets)]

        def region(calls, reps):
            for c in calls[:3]:
                c()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for i in range(reps):
                calls[i % len(calls)]()
            b.record(stream)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / reps

        reps = max(20, min(400, int(2e8 // px)))
        # compat: the X-128 write-back mutates the fp32 images; it does not
        # change the timing, and the coefficients are not checked here
        compat = [hpdct.bind("fwd", imgf[s], outs[s], transform=T, writeback_shift=True, stream=stream)
                  for s in range(sets)]
        u8 = [hpdct.bind("fwd", img8[s], outs[s], stream=stream) for s in range(sets)]
        t_compat = region(compat, reps)
        t_u8 = region(u8, reps)
        tmp = torch.empty_like(imgf[0])
        ref = [lambda s=s: hpdct.baseline_forward("reference_3pass", imgf[s], tmp, outs[s], T, stream=stream)
               for s in range(sets)]
        fast = [lambda s=s: hpdct.baseline_forward("fastappr_3pass", imgf[s], tmp, outs[s], T, stream=stream)
                for s in range(sets)]
        t_ref = region(ref, max(10, reps // 8))
        t_fast = region(fast, max(10, reps // 8))
        t4 = T4_HPAPPR_MS.get(n)
        d_ms, i_ms = drv[n]
        print(f"| {n}² | {t4 if t4 else '—'} | {d_ms:.4f} / {i_ms:.4f} | {t_compat:.4f} | {t_u8:.4f} | "
              f"{t_ref:.4f} | {t_fast:.4f} | {(t4 / d_ms) if t4 and d_ms else float('nan'):.0f}× |", flush=True)
        del img8, imgf, outs, tmp
        torch.cuda.empty_cache()
        time.sleep(0.1)


if __name__ == "__main__":
    main()
