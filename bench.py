#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: Gpixel/s of the forward 8x8 DCT +
standard-Q quantisation on 8192x8192 grayscale frames (config C3), plus the
achieved fraction of the MI355X HBM roofline, at 1/2/4/8 GPUs.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

With --gpus N > 1 and no launcher (WORLD_SIZE unset) the parent process does
not import torch or touch the GPU: it starts N child processes of this script
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set),
waits for all of them and exits non-zero if any fails.

A step = one launch of the fused gfx950 forward kernel over one 8192x8192
frame already resident in HBM (uint8 pixels in, fp32 quantised coefficients
out, reference layout; 5 algorithmic bytes per pixel).  Frames rotate over
enough buffer sets that the INPUT planes alone total >= 4x the 256 MiB
Infinity Cache (16 sets at 8192^2): non-temporal output stores do not
allocate there, so with fewer sets (4 x 64 MiB inputs fit it exactly) the
reads would be served from the cache, not HBM (tools/kbench2 set sweep,
profiles/r02/kbench2_sets_r02.log).  Weak scaling: every rank processes its own frame per step (the
frames are independent), no collective in the timed region; value = pixels
of all ranks / max-over-ranks time.

Also reported (not the headline): the other kernels of the path (fp32 compat
kernel 8 B/px, int8 wire output 2 B/px, inverse 8 B/px), the C3 round-trip
PEEN/MSE, the C4 16384^2 row-sharded run with its RCCL gather timed
separately, and the CPU baseline (the oracle, one thread, rank 0, N=1).
The CPU oracle is used ONLY for that baseline and for a parity spot-check;
every timed number is the HIP kernel.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))

METRIC = "Gpixel/s fwd-DCT (8192×8192) + achieved HBM % at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
T4_FWD_8192_MS = 14.70         # README.md:55, T4
BYTES_PER_PX = {"u8_f32": 5, "f32_f32": 8, "u8_i8": 2, "inv_f32_f32": 8,
                "compat_fwd": 12, "compat_inv": 8, "compat_inv_wb": 12}
EXTRA_STEPS = 100              # timed launches per extra (independent of --steps)
EXTRA_WARM_S = 0.02            # untimed steady-state lead-in per extra (>= 20 ms)
HEADLINE_LEAD_S = 0.02         # the headline's warm-up reaches at least this much wall time
MALL_BYTES = 256 << 20         # MI355X Infinity Cache (MI355X_MICROARCH.md)
INPUT_FOOTPRINT = 4 * MALL_BYTES  # rotating inputs must total at least this
WATCHDOG_EXIT = 3              # exit code when the extras watchdog fired (headline line printed)
HEADLINE_KERNEL_PMC = "fdct_duo_u8_kernel"  # the headline's kernel as profiles/pmc_traffic.json names it
CEIL_CAPS = (0, 4, 6, 7, 8, 10, 12, 16, 20, 24)  # residency caps (waves per CU) of the copy ceilings; 0 = none
DONE_FRAC = 0.9                # a kernel at >= this fraction of its copy ceiling is "done"


def sets_for(input_bytes: int, minimum: int = 2) -> int:
    """Rotating buffer sets so that the inputs of all sets total
    >= INPUT_FOOTPRINT: every launch then reads its input from HBM, not from
    the Infinity Cache (which the output stores, non-temporal, do not fill)."""
    return max(minimum, -(-INPUT_FOOTPRINT // max(1, input_bytes)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=8192, help="square frame side (C3: 8192)")
    ap.add_argument("--sets", type=int, default=None,
                    help="rotating buffer sets per GPU (default: inputs total >= 4x the 256 MiB Infinity Cache)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--sustain-s", type=float, default=4.0,
                    help="seconds of back-to-back headline launches after the timed region (0 = off): a steady "
                         "GPU-busy phase long enough for an external utilisation sampler, reported beside the "
                         "headline, never as it")
    ap.add_argument("--c4-size", type=int, default=16384)
    ap.add_argument("--c5-size", type=int, default=4096)
    ap.add_argument("--c5-frames", type=int, default=512)
    ap.add_argument("--no-c4c5", action="store_true",
                    help="skip the C4/C5 extras (PMC passes: every kernel then runs at the C3 size only)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank flow with several ranks on one GPU)")
    ap.add_argument("--extras-timeout-s", type=float, default=420.0,
                    help="watchdog on the extras (the other kernels, C4's RCCL gather, C5): if they have not "
                         "finished by then, rank 0 prints the headline line with extras marked as timed out "
                         "and every rank exits; 0 disables it")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """One child process per rank (no torch, no HIP in this parent), the
    torch.distributed env contract set for each; returns the first non-zero
    child exit code (the others are then terminated), else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:  # a peer is gone: the others would block in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if args.gpus < 1:
        print("--gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the ONE JSON line is the only thing this process writes to stdout: the
    # libraries' own banners (RCCL prints its version block to stdout when a
    # communicator is created) are sent to stderr by pointing fd 1 there; the
    # line goes out through a duplicate of the original stdout
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    import hpdct

    # one process per GPU: LOCAL_RANK is the device (modulo the visible devices,
    # so a gloo rehearsal can put several ranks on one GPU)
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > 1 and world > ndev:
        # RCCL needs one GPU per rank (it refuses two ranks on one device only
        # after every rank is already inside communicator setup): say so now,
        # before any RCCL or HIP call
        print(f"--backend nccl needs one GPU per rank: WORLD_SIZE={world} ranks but {ndev} visible device(s); "
              "use --backend gloo to rehearse several ranks on fewer GPUs", file=sys.stderr)
        return 2
    local_dev = local % ndev if ndev else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    # a launcher (torchrun, or launch_ranks) sets WORLD_SIZE: then the process
    # group is initialised even at WORLD_SIZE=1, so the RCCL init path runs
    use_pg = world > 1 or "WORLD_SIZE" in os.environ
    if use_pg:
        # collectives raise (instead of aborting the process) if a peer dies, so
        # rank 0 can still print the headline line; generous timeout
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        import datetime
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=240))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=240))

    def barrier():
        if use_pg:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not use_pg:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    hpdct.load_library()
    n = args.size
    px = n * n
    if args.sets is None:
        args.sets = sets_for(px, minimum=4)
    stream = torch.cuda.current_stream()

    # ---- inputs resident in HBM: set 0 = the reference's benchmark frame
    # (srand(42), rand()%256, benchmark_newAppr.cu:46-51), others device-hashed
    imgs, outs = [], []
    for s in range(args.sets):
        x = torch.empty((n, n), dtype=torch.uint8, device=dev)
        if s == 0:
            x.copy_(torch.from_numpy(hpdct.fill_rand_u8(px, 42).reshape(n, n)))
        else:
            hpdct.fill_hash_u8(x, seed=1000 * rank + s)
        imgs.append(x)
        outs.append(torch.empty((n, n), dtype=torch.float32, device=dev))
    torch.cuda.synchronize()

    hip = HipEvents(stream)

    lead_in = {"launches": 0}

    def timed_loop(calls, steps, warmup):
        """warmup untimed, then exactly `steps` back-to-back launches bracketed
        by barrier + sync, timed by a HIP event pair on the launch stream
        (hipEventRecord via ctypes).  The average launch duration is
        region / steps: it includes any gap between consecutive kernels, so it
        upper-bounds the kernel time (rocprofv3 agrees to ~2 %).  A marker per
        launch would add ~2.8 us each (tools/launch_gap.py), so there is none.
        The warm-up is the W launches plus, if they took less, untimed
        launches up to HEADLINE_LEAD_S of wall time, so the timed region runs
        at steady-state clocks: after 5 launches (0.3 ms) the first timed
        launches still ran ~2 % slow (profiles/r04/d/trace_summary.md: the
        20 timed launches 58.3 us, all 70,266 launches of the run 57.05)."""
        t_lead = time.perf_counter()
        for i in range(warmup):
            calls[i % len(calls)]()
        torch.cuda.synchronize()
        extra = 0
        while time.perf_counter() - t_lead < HEADLINE_LEAD_S:
            for _ in range(len(calls)):
                calls[(warmup + extra) % len(calls)]()
                extra += 1
            torch.cuda.synchronize()
        lead_in["launches"] = extra
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hip.record(0)
        for i in range(steps):
            calls[i % len(calls)]()
        hip.record(1)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        barrier()
        region_ms = hip.elapsed(0, 1)
        return region_ms, np.array([region_ms / steps]), wall

    # ------------------------------------------------------------ headline
    fwd_calls = [hpdct.bind("fwd", imgs[s], outs[s], stream=stream) for s in range(args.sets)]
    region_ms, kern_ms, wall = timed_loop(fwd_calls, args.steps, args.warmup)
    headline_lead_in = lead_in["launches"]
    region_ms = max_over_ranks(region_ms)
    ms_per_step = region_ms / args.steps
    value = world * px * args.steps / (region_ms * 1e-3) / 1e9  # Gpixel/s, whole job
    kavg = float(kern_ms.mean())
    achieved = BYTES_PER_PX["u8_f32"] * px / (kavg * 1e-3) / 1e9  # GB/s per GPU
    kavg_max = max_over_ranks(kavg)

    # parity spot-check of the timed output (set 0) against the oracle
    parity = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        try:
            import oracle
            crop = np.ascontiguousarray(imgs[0][:256, :512].cpu().numpy())
            ref = oracle.fdct(crop)
            got = outs[0][:256, :512].cpu().numpy()
            parity = bool(np.array_equal(ref.view(np.uint32), got.view(np.uint32)))
        except Exception as e:  # oracle missing on the box: report, do not hide
            parity = f"unchecked: {e}"

    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            with open(prof) as fh:
                pm = json.load(fh)
            k = pm.get("kernels", {}).get("fdct_u8_f32")
            # only a record of the kernel this build launches (round 6: the duo forward)
            if k and k.get("size") == n and k.get("kernel", "").startswith(HEADLINE_KERNEL_PMC):
                traffic = k.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Gpixel/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (px / (T4_FWD_8192_MS * 1e-3) / 1e9), 2) if n == 8192 else None,
        "dtype": "f32",
        "data": "synthetic: set0 = srand(42) rand()%256 (benchmark_newAppr.cu:46-51), sets1.. device hash; "
                f"{args.sets} rotating buffer sets ({args.sets * 5 * px / 2**30:.2f} GiB/GPU; inputs "
                f"{args.sets * px / 2**30:.2f} GiB = {args.sets * px / MALL_BYTES:.1f}x the Infinity Cache)",
        "config": {
            "workload": f"C3: {n}x{n} uint8 frame -> fp32 quantised 8x8 DCT coefficients (HpApprDCT, "
                        "standard JPEG Q), one fused kernel launch per frame",
            "frame": [n, n], "frames_per_gpu_per_step": 1, "input": "u8", "output": "f32 (reference layout)",
            "parallelism": f"dp{world} (independent frames per GPU, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json: rocprofv3 FETCH_SIZE/WRITE_SIZE (separate passes, "
                              "calibrated on known-byte kernels, tools/pmc_traffic.sh)" if traffic else None,
            "kernel": "hpdct::fdct_duo_u8_kernel<2> (two lanes per tile, default JPEG table's quotient forms, "
                      "16 waves per CU)",
            "bytes_per_px": BYTES_PER_PX["u8_f32"],
            "kernel_us_avg": round(kavg * 1e3, 2),
            "kernel_us_max_over_ranks": round(kavg_max * 1e3, 2),
            "timing": "HIP events around the timed region on the launch stream; avg launch = region / steps",
        },
        "vs_baseline_ref": "T4 14.70 ms (README.md:55) = 4.57 Gpixel/s, fp32-in 3-kernel path",
        "parity_spot_check": parity,
        "host_wall_s": round(wall, 4),
        "warmup_lead_in_launches": headline_lead_in,
        # which sources built the library that was timed (src_digest.py): the
        # digest stamped at build time vs the digest of this tree's sources
        "provenance": hpdct.provenance(),
    }

    # ------------------------------------------------------------ sustained headline
    if args.sustain_s > 0:
        result["sustained"] = _sustained(torch, hip, fwd_calls, args.sustain_s, px, world, barrier,
                                         max_over_ranks)

    # ------------------------------------------------------------ other kernels of the path
    if not args.no_extras:
        extras = {}
        # A hang in the extras (a first multi-GPU run of the RCCL gather, say)
        # must not cost the headline line: the watchdog prints it and exits.
        watchdog = None
        if args.extras_timeout_s > 0:
            import threading

            def _extras_timed_out():
                if rank == 0:
                    line = dict(result)
                    line["extras"] = {"error": f"extras did not finish within {args.extras_timeout_s:.0f} s "
                                               "(watchdog); headline measured before them"}
                    print(json.dumps(line), file=json_out, flush=True)
                # non-zero: a hang in C4/C5 (a stuck RCCL gather, say) must not
                # read as a successful run to a caller that checks the exit
                # code; the headline line is already out
                os._exit(WATCHDOG_EXIT)

            watchdog = threading.Timer(args.extras_timeout_s, _extras_timed_out)
            watchdog.daemon = True
            watchdog.start()
        try:
            _extras(args, hpdct, torch, dist, dev, world, rank, stream, barrier, max_over_ranks, timed_loop, imgs,
                    outs, px, n, extras)
        except Exception as e:  # report, keep the headline line
            extras["error"] = f"{type(e).__name__}: {e}"[:500]
        if watchdog is not None:
            watchdog.cancel()
        result["extras"] = extras
        hc = extras.get("headline_ceiling")
        if hc:
            # the headline kernel against the copy of its own bytes (1 B in,
            # 4 B NT out), beside its fraction of the 8 TB/s spec
            result["roofline"]["copy_ceiling_us"] = hc["us"]
            result["roofline"]["frac_of_copy_ceiling"] = round(hc["us"] / (kavg * 1e3), 4)
        c4 = extras.get("c4", {})
        # the north_star row-shard figures (C4, 16384^2 over the ranks), top level
        for key in ("compute_speedup_vs_1gpu", "predicted_compute_speedup_2", "predicted_compute_speedup_4",
                    "predicted_compute_speedup_8", "one_gpu_full_frame_ms", "gather_ms", "gather_decode_int8_ms",
                    "decode_int8_ms", "int8_wire_equals_fp32", "end_to_end_ms", "end_to_end_int8_ms", "sharded_equals_unsharded"):
            if key in c4:
                result["c4_" + key] = c4[key]
        if "compute_ms_max_rank" in c4:
            result["c4_compute_ms_max_rank"] = c4["compute_ms_max_rank"]
        # who took part in the C4 gather: the RCCL
        # communicator's size and the process group's, both == n_gpus
        for key in ("rccl_nranks", "pg_world", "gather_bytes_to_root", "gather_bytes_expected"):
            if key in c4:
                result["c4_" + key] = c4[key]

    # ------------------------------------------------------------ CPU baseline
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = _cpu_baseline(n)

    if "extras" in result:
        # last in the line, so a record that keeps only the line's tail still
        # holds every kernel against its ceiling
        result["kernel_status"] = kernel_status(result)
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if use_pg:
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    return 0


def kernel_status(result):
    """{kernel: [us, ceiling_us, frac_of_ceiling, status]} for every timed
    kernel of the line that has a reachable ceiling: the
    copy of the same bytes (hpdct_copy_ceiling) for the HBM kernels, the
    same-bytes copy on the forward's own grid for C2 (cache-resident), the
    copy-only PCIe pipeline for C5 (frames/s, higher is better; frac = rate /
    ceiling).  status: "done" at >= DONE_FRAC of the ceiling, else "open"."""
    ex = result.get("extras", {})
    out = {}

    def put(name, us, ceil_us):
        if us and ceil_us:
            f = round(ceil_us / us, 3)
            out[name] = [round(us, 2), round(ceil_us, 2), f, "done" if f >= DONE_FRAC else "open"]

    rf = result.get("roofline", {})
    put("headline_fwd_u8_f32", rf.get("kernel_us_avg"), rf.get("copy_ceiling_us"))
    for key in ("fwd_u8_i8", "inv_f32_f32", "fwd_f32_f32_runtimeT"):
        if key in ex:
            put(key, ex[key].get("kernel_us_avg"), ex[key].get("ceiling_us"))
    for key, line in ex.get("dropin", {}).items():
        put("dropin." + key.split(" ")[0] + ("_cublasv2" if "cublas" in key else ""), line.get("kernel_us_avg"),
            line.get("ceiling_us"))
    c3 = ex.get("c3_roundtrip", {})
    for key in ("one_pass", "one_pass_f32_recon", "one_pass_sums_ring"):
        if key in c3:
            put("c3." + key, c3[key].get("kernel_us_avg"), c3[key].get("ceiling_us"))
    fl = ex.get("c2_fwd_u8_f32", {}).get("floor", {})
    put("c2_fwd_u8_f32", fl.get("forward_us"), fl.get("copy_same_bytes_us"))
    for k in ("f32", "i8"):
        c5 = ex.get("c5", {}).get(k)
        if c5 and c5.get("copy_only_ceiling_frames_per_s"):
            f = round(c5["frames_per_s_total"] / c5["copy_only_ceiling_frames_per_s"], 3)
            out["c5_" + k + "_frames_per_s"] = [c5["frames_per_s_total"], c5["copy_only_ceiling_frames_per_s"], f,
                                               "done" if f >= DONE_FRAC else "open"]
    return out


def _extras(args, hpdct, torch, dist, dev, world, rank, stream, barrier, max_over_ranks, timed_loop0, imgs, outs, px,
            n, extras):
    def timed_loop(calls, steps, warmup):
        """Steady state, independent of --steps: untimed launches for at least
        max(20 ms, the timed region's expected length), then `steps` (>= 100
        for the short kernels) timed launches.  The VALU-heavy kernels run
        ~8 % slow for the first few ms after a change of load (memory-bound
        headline loop, or idle): a clock ramp, not the kernel
        (tools/seq_probe.py, profiles/r01/seq_probe.log)."""
        k = len(calls)
        t0 = time.perf_counter()
        for i in range(max(warmup, 2 * k)):
            calls[i % k]()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t0) / max(warmup, 2 * k)
        target = max(EXTRA_WARM_S, per * steps)
        i, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < target:
            for _ in range(8):
                calls[i % k]()
                i += 1
            torch.cuda.synchronize()
        return timed_loop0(calls, steps, 0)

    steps = EXTRA_STEPS
    ceil_jobs = []

    def ceiling_later(line, srcs, o0s, o1s=None):
        """Queue the copy ceiling of the kernel `line` describes (VERDICT r5
        item 2): hpdct_copy_ceiling moving the kernel's own bytes per pixel
        over the kernel's OWN rotating planes (its inputs, its outputs, its
        write-back plane; the two-output patterns vary by ~10 % with where the
        planes sit, so the ceiling must share the kernel's), timed like the
        kernel at each residency cap of CEIL_CAPS, the fastest kept.  The
        copies overwrite those outputs, so they run after every leg that
        reads them (run_ceilings)."""
        ceil_jobs.append((line, srcs, o0s, o1s))

    def measure_ceiling(srcs, o0s, o1s):
        by = {}
        for cap in CEIL_CAPS:
            calls = [hpdct.bind_copy_ceiling(srcs[i], o0s[i % len(o0s)], o1s[i % len(o1s)] if o1s else None,
                                             cap_waves=cap, stream=stream) for i in range(len(srcs))]
            rms, _, _ = timed_loop(calls, steps, 5)
            by[str(cap)] = round(rms / steps * 1e3, 2)
        best = min(by, key=by.get)
        size = {torch.uint8: 1, torch.int8: 1, torch.float32: 4}
        key = (size[srcs[0].dtype], size[o0s[0].dtype], size[o1s[0].dtype] if o1s else 0)
        return {"us": by[best], "cap_waves": int(best), "by_cap_us": by, "bytes_per_px": sum(key),
                "pattern": f"{key[0]} B in, {key[1]}" + (f" + {key[2]}" if key[2] else "") + " B out"}

    def run_ceilings():
        """ceiling_us / frac_of_ceiling beside hbm_frac, and each kernel's
        status: done at >= DONE_FRAC of the copy of its own bytes"""
        for line, srcs, o0s, o1s in ceil_jobs:
            ceil = measure_ceiling(srcs, o0s, o1s)
            if "kernel_us_avg" not in line:  # the headline's own entry
                line.update(ceil)
                continue
            line["ceiling_us"] = ceil["us"]
            line["frac_of_ceiling"] = round(ceil["us"] / line["kernel_us_avg"], 4)
            line["ceiling"] = ceil
            line["status"] = "done" if line["frac_of_ceiling"] >= DONE_FRAC else "open"
        ceil_jobs.clear()

    if True:
        # fp32 in -> fp32 out (the reference's own data types; compat kernel)
        f32_in = [imgs[s].float() for s in range(args.sets)]
        f32_out = outs[:len(f32_in)]
        T = torch.from_numpy(hpdct.default_transform()).to(dev)
        calls = [hpdct.bind("fwd", f32_in[i], f32_out[i], transform=T, stream=stream) for i in range(len(f32_in))]
        rms, k, _ = timed_loop(calls, steps, 5)
        extras["fwd_f32_f32_runtimeT"] = _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["f32_f32"], world,
                                               "fdct_f32_f32_duo_runtimeT", n)
        ceiling_later(extras["fwd_f32_f32_runtimeT"], f32_in, f32_out)
        # the headline's own copy ceiling (1 B in, 4 B out), beside its roofline
        extras["headline_ceiling"] = {}
        ceiling_later(extras["headline_ceiling"], imgs, outs)
        # u8 -> int8 wire format
        i8 = [torch.empty((n, n), dtype=torch.int8, device=dev) for _ in range(args.sets)]
        calls = [hpdct.bind("fwd", imgs[s], i8[s], stream=stream) for s in range(args.sets)]
        rms, k, _ = timed_loop(calls, steps, 5)
        extras["fwd_u8_i8"] = _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["u8_i8"], world, "fdct_u8_i8", n)
        ceiling_later(extras["fwd_u8_i8"], imgs, i8)
        # inverse fp32 -> fp32 (idct_all_blocks_cuda's data path)
        rec = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(2)]
        calls = [hpdct.bind("inv", outs[s], rec[s % 2], stream=stream) for s in range(args.sets)]
        rms, k, _ = timed_loop(calls, steps, 5)
        extras["inv_f32_f32"] = _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["inv_f32_f32"], world,
                                      "idct_f32_f32_duo", n)
        ceiling_later(extras["inv_f32_f32"], outs, rec)
        # the drop-in surface: exactly what the compat entry points launch
        # (hpdct_compat.cpp), i.e. what a caller of the reference's functions
        # gets: fp32 planes, the caller's T, and the reference's in-place side
        # effects (X-128 left in the image, main_newAppr.cu:273; q*Q left in the
        # coefficients by the cublasDCTv2 inverse, main_cublass_2.cu:285).  The
        # write-backs change the inputs from launch to launch; the kernels' time
        # does not depend on the values.
        dropin = {}
        calls = [hpdct.bind("fwd", f32_in[i], f32_out[i], transform=T, writeback_shift=True, stream=stream)
                 for i in range(len(f32_in))]
        rms, k, _ = timed_loop(calls, steps, 5)
        dropin["dct_all_blocks_cuda"] = dict(
            _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["compat_fwd"], world, "compat_fwd_f32_wb", n),
            launches="fdct_duo_kernel<quant, runtime T, writeback>",
            bytes_note="4 B read + 4 B coefficients + 4 B X-128 written back")
        calls = [hpdct.bind("inv", outs[s], rec[s % 2], transform=T, stream=stream) for s in range(args.sets)]
        rms, k, _ = timed_loop(calls, steps, 5)
        dropin["idct_all_blocks_cuda"] = dict(
            _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["compat_inv"], world, "compat_inv_f32", n),
            launches="idct_duo_kernel<dequant, runtime T>", bytes_note="4 B read + 4 B written")
        calls = [hpdct.bind("fwd", f32_in[i], f32_out[i], transform=T, writeback_shift=True, row_first=True,
                            stream=stream) for i in range(len(f32_in))]
        rms, k, _ = timed_loop(calls, steps, 5)
        dropin["dct_all_blocks (cublasDCTv2)"] = dict(
            _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["compat_fwd"], world, "compat_fwd_rowfirst_wb", n),
            launches="rowfirst_duo_kernel<forward, quant, runtime T, writeback>",
            bytes_note="4 B read + 4 B coefficients + 4 B X-128 written back")
        calls = [hpdct.bind("inv", outs[s], rec[s % 2], transform=T, row_first=True, writeback_dequant=True,
                            stream=stream) for s in range(args.sets)]
        rms, k, _ = timed_loop(calls, steps, 5)
        dropin["idct_all_blocks (cublasDCTv2)"] = dict(
            _line(px, rms / steps, float(k.mean()), BYTES_PER_PX["compat_inv_wb"], world, "compat_inv_rowfirst_wb",
                  n),
            launches="rowfirst_duo_kernel<inverse, dequant, runtime T, writeback>",
            bytes_note="4 B read + 4 B pixels + 4 B q*Q written back")
        extras["dropin"] = dropin
        # the drop-in kernels' ceilings: their own planes, the write-back plane
        # being the input (X-128) or the coefficient plane (q*Q) in place
        ceiling_later(dropin["dct_all_blocks_cuda"], f32_in, f32_out, f32_in)
        ceiling_later(dropin["idct_all_blocks_cuda"], outs, rec)
        ceiling_later(dropin["dct_all_blocks (cublasDCTv2)"], f32_in, f32_out, f32_in)
        ceiling_later(dropin["idct_all_blocks (cublasDCTv2)"], outs, rec, outs)
        # the write-backs above changed the fp32 inputs / coefficients: the
        # later extras recompute what they read
        # the reference's own two GPU decompositions of the same arithmetic, on
        # this GPU (include/hpdct_baseline.h): 3 launches per frame, fp32 in/out
        T = torch.from_numpy(hpdct.default_transform()).to(dev)
        bimg = imgs[0].float()
        btmp = torch.empty_like(bimg)
        bres = torch.empty_like(bimg)
        for kind in ("reference_3pass", "fastappr_3pass"):
            calls = [lambda k=kind: hpdct.baseline_forward(k, bimg, btmp, bres, T, stream=stream)]
            bsteps = 40
            rms, k, _ = timed_loop(calls, bsteps, 3)
            extras["baseline_" + kind] = {
                "ms_per_frame": round(rms / bsteps, 4), "gpx_s": round(px / (rms / bsteps * 1e-3) / 1e9, 2),
                "note": "the reference's 3-launch structure re-expressed in HIP on this MI355X (fp32 in/out, "
                        "X-128 in place); same arithmetic, bit-identical output"}
        del bimg, btmp, bres
        # C3 round trip quality on the reference's frame
        hpdct.forward(imgs[0], outs[0])
        r = hpdct.inverse(outs[0], rec[0])
        r8 = hpdct.inverse(outs[0], out_dtype=torch.uint8)  # clamp + truncate (utils.cu:18-24)
        # C3 round trip timed: forward u8 -> fp32 coefficients, inverse -> u8 pixels
        rt_px = [torch.empty((n, n), dtype=torch.uint8, device=dev) for _ in range(2)]
        fwd = [hpdct.bind("fwd", imgs[s], outs[s], stream=stream) for s in range(args.sets)]
        inv = [hpdct.bind("inv", outs[s], rt_px[s % 2], stream=stream) for s in range(args.sets)]
        pair = [lambda s=s: (fwd[s](), inv[s]()) for s in range(args.sets)]
        rms, _, _ = timed_loop(pair, steps, 4)
        rt_ms = rms / steps
        x = imgs[0].double()
        sx = float((x * x).sum())
        se = float(((x - r.double()) ** 2).sum())
        se8 = float(((x - r8.double()) ** 2).sum())
        # the same round trip in ONE pass (hpdct_roundtrip_u8): fp32 coefficients
        # + uint8 reconstruction + the PEEN/MSE sums, 6 B/px of HBM
        sums_buf = torch.zeros(3, dtype=torch.int64, device=dev)
        one = [hpdct.bind_roundtrip(imgs[s], outs[s], rt_px[s % 2], sums_buf, stream=stream)
               for s in range(args.sets)]
        rms1, k1, _ = timed_loop(one, steps, 4)
        one[0]()
        qd = hpdct.quality_from_sums(hpdct.sums_from_buffer(sums_buf), px)
        one_ms = rms1 / steps
        sums_one = hpdct.sums_from_buffer(sums_buf)
        # the same with the fp32 reconstruction (R + 128 unclamped, the
        # reference's float output): coefficients + fp32 pixels + sums, 9 B/px.
        # Checked: set 0's fp32 pixels equal the two-kernel inverse's, and its
        # sums equal the uint8-reconstruction pass's (the same definition)
        r_ref = r.clone()
        sums_f = torch.zeros(3, dtype=torch.int64, device=dev)
        onef = [hpdct.bind_roundtrip(imgs[s], outs[s], rec[s % 2], sums_f, stream=stream)
                for s in range(args.sets)]
        rmsf, kf, _ = timed_loop(onef, steps, 4)
        onef[0]()
        torch.cuda.synchronize()
        f32_recon_exact = bool(torch.equal(rec[0], r_ref))
        f32_sums_equal = hpdct.sums_from_buffer(sums_f) == sums_one
        f32_ms = rmsf / steps
        del onef, sums_f, r_ref
        # the same with a caller-zeroed ring of per-frame sums slots
        # (hpdct_roundtrip_u8_accumulate: the frame's sums are added to its
        # slot by the same finish kernel).  The warm-up runs the timed launches
        # themselves into the ring (so every ring entry has its library slot, as
        # in a pipeline that reuses its ring: a first use allocates), then the
        # ring is zeroed outside the timed region and the timed launches go one
        # per entry, so after the region every entry must hold exactly its
        # frame's sums (ring_sums_exact)
        ref_sums = []
        for s in range(args.sets):
            b = torch.zeros(3, dtype=torch.int64, device=dev)
            hpdct.bind_roundtrip(imgs[s], outs[s], rt_px[0], b, stream=stream)()
            ref_sums.append(b)
        ring_n = steps
        ring = torch.zeros((ring_n, 3), dtype=torch.int64, device=dev)
        acc = [hpdct.bind_roundtrip(imgs[i % args.sets], outs[i % args.sets], rt_px[i % 2], ring[i], stream=stream,
                                    accumulate=True) for i in range(ring_n)]
        i, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < EXTRA_WARM_S or i < 2 * len(acc):
            acc[i % len(acc)]()
            i += 1
            if i % 16 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        ring.zero_()
        torch.cuda.synchronize()
        barrier()
        ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev_a.record(stream)
        for c in acc:
            c()
        ev_b.record(stream)
        torch.cuda.synchronize()
        acc_ms = ev_a.elapsed_time(ev_b) / ring_n
        want = torch.stack(ref_sums)[torch.arange(ring_n, device=dev) % args.sets]
        ring_exact = bool(torch.equal(ring, want))
        qa = hpdct.quality_from_sums(hpdct.sums_from_buffer(ring[0]), px)
        k2 = np.array([acc_ms])
        rms2 = acc_ms * steps
        # the device sums against torch's on the two-kernel output: the integer
        # fields exactly (double is exact below 2^53)
        sums_exact = sums_one["sse_u8"] == int(se8) and sums_one["sum_x2"] == int(sx)
        extras["c3_roundtrip"] = {
            "mse_f32": se / px, "peen_f32_pct": 100.0 * (se / sx) ** 0.5,
            "mse_u8": se8 / px, "peen_u8_pct": 100.0 * (se8 / sx) ** 0.5,
            "two_kernels": {"ms_per_frame": round(rt_ms, 5), "gpx_s": round(world * px / (rt_ms * 1e-3) / 1e9, 2),
                            "bytes_per_px": 10, "note": "forward u8->f32 then inverse f32->u8, PEEN/MSE by torch"},
            "one_pass": dict(_line(px, one_ms, float(k1.mean()), 6, world, "roundtrip_u8_f32_u8_sums", n),
                             quality_from_device_sums=qd, sums_exact_vs_two_kernels=sums_exact,
                             note="hpdct_roundtrip_u8: coefficients + u8 reconstruction + PEEN/MSE sums in one "
                                  "pass (the round trip + a one-wave kernel that moves the sums from the library's "
                                  "slot over the caller's struct); bit-identical to the two kernels"),
            "one_pass_f32_recon": dict(_line(px, f32_ms, float(kf.mean()), 9, world),
                                       recon_equals_two_kernels=f32_recon_exact, sums_equal_u8_pass=f32_sums_equal,
                                       note="hpdct_roundtrip_u8 with HPDCT_F32: coefficients + fp32 R+128 (the "
                                            "reference's float output) + PEEN/MSE sums in one pass"),
            "one_pass_sums_ring": dict(_line(px, acc_ms, float(k2.mean()), 6, world), quality_from_device_sums=qa,
                                       ring_sums_exact=ring_exact,
                                       note="hpdct_roundtrip_u8_accumulate, one ring entry per timed launch; the "
                                            "warm-up runs the same launches into the ring, which is then zeroed "
                                            "outside the timed region; ring_sums_exact: every entry equals its "
                                            "frame's hpdct_roundtrip_u8 sums"),
            "note": "uniform-noise frame: not comparable with README's 'Circuit' image (4.66 %)"}
        c3 = extras["c3_roundtrip"]
        ceiling_later(c3["one_pass"], imgs, outs, rt_px)
        ceiling_later(c3["one_pass_f32_recon"], imgs, outs, rec)
        ceiling_later(c3["one_pass_sums_ring"], imgs, outs, rt_px)
        # every leg that reads these planes has run: the copies may overwrite them
        run_ceilings()
        del f32_in, i8, rec, r8, x, rt_px, sums_buf, ring, acc, ref_sums, want
        # C2: 1024^2 forward + quantise (u8 -> fp32); 8 frame sets = 40 MB, so it
        # is served from the 256 MiB Infinity Cache: the HBM fraction is not meaningful
        c2 = 1024
        c2_in = [torch.empty((c2, c2), dtype=torch.uint8, device=dev) for _ in range(8)]
        for s, t in enumerate(c2_in):
            hpdct.fill_hash_u8(t, seed=42 + s)
        c2_out = [torch.empty((c2, c2), dtype=torch.float32, device=dev) for _ in range(8)]
        calls = [hpdct.bind("fwd", c2_in[s], c2_out[s], stream=stream) for s in range(8)]
        rms, k, _ = timed_loop(calls, 8 * steps, 10)
        line = _line(c2 * c2, rms / (8 * steps), float(k.mean()), BYTES_PER_PX["u8_f32"], world)
        line["note"] = "cache-resident (40 MB working set < 256 MiB MALL): hbm_frac not meaningful"
        # the floors of that launch (hpdct_floor_probe): an empty kernel on the
        # forward's own grid, and the same grid copying the same bytes (1 B
        # read + 4 B NT write per pixel, no transform); VERDICT r4 item 5
        floor = {}
        for name, kind in (("empty_kernel_us", hpdct.PROBE_EMPTY), ("copy_same_bytes_us", hpdct.PROBE_COPY)):
            pc = [hpdct.bind_floor_probe(kind, c2_in[s], c2_out[s], c2, c2, stream=stream) for s in range(8)]
            frms, _, _ = timed_loop(pc, 8 * steps, 10)
            floor[name] = round(frms / (8 * steps) * 1e3, 3)
        fwd_us = rms / (8 * steps) * 1e3
        floor["forward_us"] = round(fwd_us, 3)
        floor["forward_minus_copy_us"] = round(fwd_us - floor["copy_same_bytes_us"], 3)
        # the mapping A/B the floor asks for when the gap exceeds 1 us: the
        # tile mapping (256 waves of 64 tiles) against AUTO's octet (2,048 waves)
        try:
            hpdct.set_mapping("tile")
            tc = [hpdct.bind("fwd", c2_in[s], c2_out[s], stream=stream) for s in range(8)]
            trms, _, _ = timed_loop(tc, 8 * steps, 10)
            floor["forward_tile_mapping_us"] = round(trms / (8 * steps) * 1e3, 3)
        finally:
            hpdct.set_mapping("auto")
        line["floor"] = floor
        extras["c2_fwd_u8_f32"] = line
        del c2_in, c2_out
        # C2 frames batched: a 1024^2 frame is 256 tile sets, one per CU, so a
        # single-frame launch is dominated by the per-dispatch cost (~4 us; a
        # HIP graph of the same launches does not remove it,
        # profiles/r01/c2_probe.log).  32 frames stacked as one (32*1024) x 1024
        # image (the C-ABI's batch layout) make one launch; 32 MiB of input per
        # launch, rotated over sets_for() sets (1 GiB of inputs)
        nb = 32
        nbs = sets_for(nb * c2 * c2)
        c2b_in = [torch.empty((nb * c2, c2), dtype=torch.uint8, device=dev) for _ in range(nbs)]
        for s, t in enumerate(c2b_in):
            hpdct.fill_hash_u8(t, seed=4242 + s)
        c2b_out = [torch.empty((nb * c2, c2), dtype=torch.float32, device=dev) for _ in range(nbs)]
        calls = [hpdct.bind("fwd", c2b_in[s], c2b_out[s], stream=stream) for s in range(nbs)]
        rms, k, _ = timed_loop(calls, steps, 5)
        line = _line(nb * c2 * c2, rms / steps, float(k.mean()), BYTES_PER_PX["u8_f32"], world)
        line["us_per_frame"] = round(rms / steps / nb * 1e3, 3)
        line["note"] = f"{nb} 1024^2 frames per launch, stacked (C-ABI batch layout), {nbs} rotating sets"
        extras["c2_batched_fwd_u8_f32"] = line
        del c2b_in, c2b_out
        # C2 frames as a LIST of separately allocated 1024^2 planes
        # (hpdct_forward_frames): 64 frames per call = one launch, lists rotated
        # over sets_for() so the inputs come from HBM
        nf = 64
        nls = sets_for(nf * c2 * c2)
        fl_in = [[torch.empty((c2, c2), dtype=torch.uint8, device=dev) for _ in range(nf)] for _ in range(nls)]
        for s, lst in enumerate(fl_in):
            for k, t in enumerate(lst):
                hpdct.fill_hash_u8(t, seed=7000 + 100 * s + k)
        fl_out = [[torch.empty((c2, c2), dtype=torch.float32, device=dev) for _ in range(nf)] for _ in range(nls)]
        calls = [hpdct.bind_frames(fl_in[s], fl_out[s], stream=stream) for s in range(nls)]
        rms, k, _ = timed_loop(calls, steps, 5)
        line = _line(nf * c2 * c2, rms / steps, float(k.mean()), BYTES_PER_PX["u8_f32"], world)
        line["us_per_frame"] = round(rms / steps / nf * 1e3, 3)
        ok = all(torch.equal(hpdct.forward(fl_in[0][j]).view(torch.int32), fl_out[0][j].view(torch.int32))
                 for j in (0, nf - 1))
        line["equals_per_frame_forward"] = ok
        line["note"] = (f"{nf} separately allocated 1024^2 frames per call (hpdct_forward_frames, one launch), "
                        f"{nls} rotating lists")
        extras["c2_frame_list_fwd_u8_f32"] = line
        del fl_in, fl_out, calls
        torch.cuda.empty_cache()
        if not args.no_c4c5:
            use_pg = world > 1 or "WORLD_SIZE" in os.environ  # as main()
            extras["c4"] = _c4(args, hpdct, torch, dist, dev, world, rank, stream, barrier, max_over_ranks,
                               timed_loop, use_pg)
            extras["c5"] = _c5(args, hpdct, torch, world, rank, barrier, max_over_ranks)


class HipEvents:
    """hipEventCreate/Record/ElapsedTime through ctypes on the HIP runtime
    torch already loaded (libamdhip64.so.7): ~1 us of host time per record.
    Event i+1 ends launch i and starts launch i+1, so each kernel's duration
    is the gap between consecutive events on its stream."""

    def __init__(self, stream, n=4):
        import ctypes
        self.ct = ctypes
        self.lib = ctypes.CDLL("libamdhip64.so.7")
        self.lib.hipEventCreate.argtypes = [ctypes.c_void_p]
        self.lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.hipEventElapsedTime.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        self.stream = ctypes.c_void_p(stream.cuda_stream)
        self.ev = []
        for _ in range(n):
            e = ctypes.c_void_p()
            if self.lib.hipEventCreate(ctypes.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(e)
        self._rec = self.lib.hipEventRecord

    def record(self, i):
        self._rec(self.ev[i], self.stream)

    def elapsed(self, a, b):
        ms = self.ct.c_float()
        if self.lib.hipEventElapsedTime(self.ct.byref(ms), self.ev[a], self.ev[b]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value


def _pmc(key, n):
    """PMC-measured HBM traffic of one kernel (profiles/pmc_traffic.json,
    tools/pmc_traffic.sh), if recorded at this frame size."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            k = json.load(fh).get("kernels", {}).get(key)
        if k and k.get("size") == n:
            return k
    except (OSError, ValueError):
        pass
    return None


def _line(px, ms_step, kern_ms, bpp, world, pmc_key=None, n=None):
    gbs = bpp * px / (kern_ms * 1e-3) / 1e9
    out = {"gpx_s": round(world * px / (ms_step * 1e-3) / 1e9, 3), "ms_per_step": round(ms_step, 5),
           "kernel_us_avg": round(kern_ms * 1e3, 2), "bytes_per_px": bpp, "achieved_GBs": round(gbs, 1),
           "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
    k = _pmc(pmc_key, n) if pmc_key else None
    if k:
        out["traffic"] = k["hbm_bytes_per_launch"]
        out["traffic_over_algorithmic"] = k["traffic_over_algorithmic"]
    return out


def _sustained(torch, hip, calls, seconds, px, world, barrier, max_over_ranks):
    """The headline launches back to back for `seconds` of wall time (chunks of
    64, one host sync per chunk so the queue stays bounded), timed by the same
    HIP event pair.  It keeps the GPU busy long enough for a utilisation
    sampler outside the process to see it, and shows the headline rate holds
    over thousands of launches (clocks and power at steady state)."""
    barrier()
    torch.cuda.synchronize()
    i, t0 = 0, time.perf_counter()
    hip.record(0)
    while time.perf_counter() - t0 < seconds:
        for _ in range(64):
            calls[i % len(calls)]()
            i += 1
        torch.cuda.synchronize()
    hip.record(1)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier()
    ms = hip.elapsed(0, 1)
    us = max_over_ranks(ms * 1e3 / i)  # the slowest rank's time per launch
    return {"seconds": round(wall, 3), "launches_rank0": i, "us_per_launch_max_rank": round(us, 2),
            "gpx_s": round(world * px / (us * 1e-6) / 1e9, 3),
            "note": "headline kernel back to back for the whole period, incl. one host sync per 64 launches; "
                    "whole job = ranks x the slowest rank's rate"}


def _steady_ms(torch, calls, steps, stream):
    """Rank-local steady-state timing (no barrier): >= 20 ms of untimed
    launches, then `steps` launches between two events on `stream`."""
    i, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < EXTRA_WARM_S or i < 2 * len(calls):
        calls[i % len(calls)]()
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for i in range(steps):
        calls[i % len(calls)]()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def _c4(args, hpdct, torch, dist, dev, world, rank, stream, barrier, max_over_ranks, timed_loop, use_pg):
    """C4: one 16384^2 frame row-sharded over the ranks (device-generated by
    the stateless hash so no H2D), the forward kernel per slab, the gather of
    the coefficient slabs to rank 0.  Reported:

      compute_ms_max_rank        this run's slab kernel, max over ranks;
      one_gpu_full_frame_ms      the whole frame on one GPU (rank 0);
      predicted_compute_speedup_{2,4,8}
                                 full frame / the rank-0 slab of a k-way split,
                                 both timed on THIS GPU at every world size
                                 (world 1 included): the compute-phase node
                                 speedup k GPUs would give (north_star >= 6x
                                 at 8), measured without k GPUs;
      gather_ms                  the fp32 gather alone (the root computes its
                                 own slab in place in the frame, so only peer
                                 bytes move: 0 at world 1);
      gather_decode_int8_ms      the int8 wire's gather: peers' int8 slabs to
                                 the root, decoded there into its fp32 frame
                                 (peer rows only; the root's own slab is fp32
                                 in place: nothing at world 1);
      decode_int8_ms             the root's int8 -> fp32 decode kernel over a
                                 whole frame, inputs rotated past the Infinity
                                 Cache (decode_int8_sets frames);
      end_to_end_ms / end_to_end_int8_ms
                                 slab forward + gather (+ decode) between two
                                 barriers, max over ranks: what a caller that
                                 needs the whole fp32 frame on one GPU waits.

    With the nccl backend the gather is the native C-ABI
    (include/hpdct_dist.h: hpdct_gather_rows, ncclSend/ncclRecv over xGMI) on a
    communicator of its own; the gloo rehearsal (several ranks on one GPU,
    which RCCL cannot serve) uses torch.distributed's gather; a single process
    without a process group has nothing to gather."""
    from hpdct_dist import gather_slabs
    n = args.c4_size
    r0, rows = hpdct.shard_rows_native(n, world, rank)
    reps = EXTRA_STEPS

    def slab_ms(first, nrows):
        """steady-state time of the forward over an nrows x n slab (rows from
        `first` of the frame), inputs rotated past the Infinity Cache"""
        nsl = sets_for(nrows * n)
        xs = [torch.empty((nrows, n), dtype=torch.uint8, device=dev) for _ in range(nsl)]
        for t in xs:
            hpdct.fill_hash_u8(t, seed=42, first_index=first * n)
        ys = [torch.empty((nrows, n), dtype=torch.float32, device=dev) for _ in range(nsl)]
        calls = [hpdct.bind("fwd", xs[i], ys[i], stream=stream) for i in range(nsl)]
        ms = _steady_ms(torch, calls, reps, stream)
        del xs, ys, calls
        torch.cuda.empty_cache()
        return ms, nsl

    # this run's slab, timed on every rank together
    nsl = sets_for(rows * n)
    xs = [torch.empty((rows, n), dtype=torch.uint8, device=dev) for _ in range(nsl)]
    for t in xs:
        hpdct.fill_hash_u8(t, seed=42, first_index=r0 * n)
    ys = [torch.empty((rows, n), dtype=torch.float32, device=dev) for _ in range(nsl)]
    calls = [hpdct.bind("fwd", xs[i], ys[i], stream=stream) for i in range(nsl)]
    rms, _, _ = timed_loop(calls, reps, 4)
    compute_ms = max_over_ranks(rms / reps)
    x = xs[0]
    del xs[1:], ys, calls
    torch.cuda.empty_cache()
    out = {"frame": [n, n], "rows_per_rank": rows, "slab_sets": nsl, "compute_ms_max_rank": round(compute_ms, 4),
           "compute_gpx_s": round(n * n / (compute_ms * 1e-3) / 1e9, 2),
           "compute_hbm_frac_max_rank": round(5 * rows * n / (compute_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    # the full frame and the k-way rank-0 slabs on this GPU (rank 0; the others wait)
    if rank == 0:
        full_ms, _ = slab_ms(0, n)
        out["one_gpu_full_frame_ms"] = round(full_ms, 4)
        pred = {}
        for k in (2, 4, 8):
            f0, kr = hpdct.shard_rows_native(n, k, 0)
            ms, _ = slab_ms(f0, kr)
            pred[str(k)] = {"rows": kr, "slab_ms": round(ms, 4), "speedup": round(full_ms / ms, 2)}
        out["predicted_compute"] = pred
        for k in (2, 4, 8):
            out[f"predicted_compute_speedup_{k}"] = pred[str(k)]["speedup"]
        if world > 1:
            out["compute_speedup_vs_1gpu"] = round(full_ms / compute_ms, 2)
    barrier()

    comm = None
    if args.backend == "nccl" and (use_pg or world == 1):
        if world == 1:
            comm = hpdct.Comm.init_all([dev.index])[0]
        else:
            uid = [hpdct.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = hpdct.Comm.init_rank(world, uid[0], rank, dev.index)
        out["gather_path"] = ("native RCCL: hpdct_gather_rows (ncclSend/ncclRecv group), libhpdct_dist.so; the "
                              "root's slab computed in place in the frame")
    elif use_pg:
        out["gather_path"] = "torch.distributed gather (gloo rehearsal, staged through host memory)"
    else:
        out["gather_path"] = "none (one process, no process group: the slab is the frame)"

    # The root's own slab is computed fp32 in place in its frame for BOTH wire
    # formats: the int8 wire carries only the peers' slabs, which the root
    # receives into an int8 scratch frame and decodes into the fp32 frame
    # (hpdct_gather_decode_i8).  Other ranks: slab buffers.
    frame = torch.empty((n, n), dtype=torch.float32, device=dev) if rank == 0 else None
    frame8 = torch.empty((n, n), dtype=torch.int8, device=dev) if rank == 0 else None
    in_place = comm is not None or not use_pg
    if rank == 0 and in_place:
        y = frame[r0:r0 + rows]
    else:
        y = torch.empty((rows, n), dtype=torch.float32, device=dev)
    # int8 slab: every rank but a native/one-process root (the gloo rehearsal's
    # gather takes every rank's slab, the root's own included)
    y8 = None if (rank == 0 and in_place) else torch.empty((rows, n), dtype=torch.int8, device=dev)
    own_f32 = frame[r0:r0 + rows] if rank == 0 else None

    def forward(dst):
        if comm is not None:
            hpdct.forward_slab(comm, x, dst, n, n, stream=stream)
        else:
            hpdct.forward(x, dst)

    def gather(slab, full):
        if comm is not None:
            hpdct.gather_rows(comm, slab, full, n, n, root=0, stream=stream)
            return full
        if not use_pg:
            return full  # computed in place: the slab is the frame
        got = gather_slabs(slab, n, n, root=0)
        if rank == 0:
            full.copy_(got)
        return full

    def forward_i8():
        if rank == 0:
            forward(own_f32)  # the root's rows: fp32, in place
            if y8 is not None:
                forward(y8)
        else:
            forward(y8)

    def gather_i8():
        """peers' int8 slabs -> the root's int8 scratch -> decoded into its fp32
        frame, peer rows only"""
        if comm is not None:
            hpdct.gather_decode_i8(comm, y8 if rank != 0 else None, frame8, frame, n, n, root=0, stream=stream)
            return
        if not use_pg:
            return  # one process: no peers
        got = gather_slabs(y8, n, n, root=0)
        if rank == 0:
            frame8.copy_(got)
            if r0 > 0:
                hpdct.decode_i8_f32(frame8[:r0], frame[:r0], stream=stream)
            if r0 + rows < n:
                hpdct.decode_i8_f32(frame8[r0 + rows:], frame[r0 + rows:], stream=stream)

    def timed(fn, tries=3):
        best = None
        for _ in range(tries):
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            best = ms if best is None else min(best, ms)
        return round(max_over_ranks(best), 4)

    peer_rows = n - rows
    out.update(c4_identity(args.gpus, dist.get_world_size() if use_pg else 1,
                           comm.size if comm is not None else None, rank, n, rows))
    forward(y)
    out["gather_ms"] = timed(lambda: gather(y, frame))
    forward_i8()
    out["gather_decode_int8_ms"] = timed(gather_i8)
    out["gather_int8_bytes_to_root"] = peer_rows * n if rank == 0 else None
    out["decoded_rows_on_root"] = peer_rows if rank == 0 else None
    if rank == 0:
        # the decode kernel over a whole frame, from HBM: inputs rotated over
        # sets_for() int8 frames (>= 4x the Infinity Cache), like every timed kernel
        nd = sets_for(n * n)
        q8s = [torch.empty((n, n), dtype=torch.int8, device=dev) for _ in range(nd)]
        for i, q in enumerate(q8s):
            xi = torch.empty((n, n), dtype=torch.uint8, device=dev)
            hpdct.fill_hash_u8(xi, seed=77 + i, first_index=0)
            hpdct.forward(xi, q)
            del xi
        decs = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(nd)]
        calls = [(lambda i=i: hpdct.decode_i8_f32(q8s[i], decs[i], stream=stream)) for i in range(nd)]
        dec_ms = _steady_ms(torch, calls, reps // 4, stream)
        out["decode_int8_ms"] = round(dec_ms, 4)
        out["decode_int8_sets"] = nd
        out["decode_int8_hbm_frac"] = round(5 * n * n / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        del q8s, decs, calls
        torch.cuda.empty_cache()

    def e2e_f32():
        forward(y)
        gather(y, frame)

    def e2e_i8():
        forward_i8()
        gather_i8()

    out["end_to_end_int8_ms"] = timed(e2e_i8)
    if rank == 0:
        # the frame assembled through the int8 wire equals the one-GPU fp32 forward
        xf = torch.empty((n, n), dtype=torch.uint8, device=dev)
        hpdct.fill_hash_u8(xf, seed=42, first_index=0)
        ref = hpdct.forward(xf)
        torch.cuda.synchronize()
        out["int8_wire_equals_fp32"] = bool(torch.equal(frame, ref))  # by value: a -0.0 decodes as +0.0
        del xf
    out["end_to_end_ms"] = timed(e2e_f32)
    out["end_to_end_note"] = ("slab forward + gather (int8: the peers' slabs decoded on the root, whose own slab "
                              "is fp32 in place) between barriers, host clock, best of 3, max over ranks; compare "
                              "one_gpu_full_frame_ms (the whole frame on one GPU)")
    if rank == 0:
        # sharded + gathered == the whole frame computed on one GPU, bit for bit
        out["sharded_equals_unsharded"] = bool(torch.equal(ref.view(torch.int32), frame.view(torch.int32)))
        del ref
    barrier()
    if comm is not None:
        comm.destroy()
    del x, y, y8, frame, frame8, own_f32
    torch.cuda.empty_cache()
    return out


def c4_identity(gpus, pg_world, rccl_nranks, rank, n, rows):
    """Who takes part in the C4 gather, for the line: the
    process group's size (`pg_world`, dist.get_world_size(), 1 without a
    group) and the RCCL communicator's (`rccl_nranks`, hpdct_comm_size; None
    when the gather is not native RCCL, e.g. the gloo rehearsal).  Both must
    equal --gpus, or the leg fails loudly instead of reporting a gather over
    fewer ranks.  On the root, gather_bytes_to_root is what the peers send it:
    the frame's rows outside its own slab, fp32, i.e. (N-1)/N of the frame for
    N ranks and equal slabs, 0 at N = 1 (the root's slab is computed in place);
    gather_bytes_expected is that fraction of the frame's fp32 bytes."""
    if pg_world != gpus or (rccl_nranks is not None and rccl_nranks != gpus):
        raise RuntimeError(f"C4 gather over the wrong ranks: --gpus {gpus}, process group {pg_world}, "
                           f"RCCL communicator {rccl_nranks}")
    out = {"rccl_nranks": rccl_nranks, "pg_world": pg_world}
    if rank == 0:
        out["gather_bytes_to_root"] = (n - rows) * n * 4
        out["gather_bytes_expected"] = n * n * 4 * (gpus - 1) // gpus if n // 8 % gpus == 0 else None
        if out["gather_bytes_expected"] is not None and out["gather_bytes_to_root"] != out["gather_bytes_expected"]:
            raise RuntimeError(f"C4 root receives {out['gather_bytes_to_root']} B, expected "
                               f"{out['gather_bytes_expected']} B for {gpus} ranks")
    else:
        out["gather_bytes_to_root"] = None
    return out


def _c5(args, hpdct, torch, world, rank, barrier, max_over_ranks):
    """C5: a batch of independent 4096^2 frames streamed from pinned host memory
    through H2D -> forward kernel -> D2H (hpdct_stream_forward); replicas only:
    every rank takes its share of the batch, no collective.  Host frames: a
    pool of 8 pinned frames (srand(seed), seeds 42..49) cycled over the batch.

    The product pipeline (2 streams, each H2D -> kernel -> D2H for its frames)
    is the reported figure; beside it 3 streams, the rejected round-4 layout
    (one stream per engine over a ring of device slots,
    HPDCT_STREAM_PIPELINE=engines) and the copy-only ceiling of the same bytes
    (the pipeline's H2D and D2H copies with no kernel: what PCIe allows)."""
    n = args.c5_size
    frames_total = args.c5_frames
    mine = frames_total // world + (1 if rank < frames_total % world else 0)
    pool_in = []
    for k in range(8):
        t = torch.empty((n, n), dtype=torch.uint8).pin_memory()
        t.copy_(torch.from_numpy(hpdct.fill_rand_u8(n * n, 42 + k).reshape(n, n)))
        pool_in.append(t)
    res = {"frame": [n, n], "frames_total": frames_total, "frames_per_rank": mine}

    def run(frames, outs, slots, layout):
        old = os.environ.get("HPDCT_STREAM_PIPELINE")
        os.environ["HPDCT_STREAM_PIPELINE"] = layout
        try:
            hpdct.stream_forward(frames[:8], outs[:8], nstreams=slots)  # warm-up
            barrier()
            return max_over_ranks(hpdct.stream_forward(frames, outs, nstreams=slots))
        finally:
            if old is None:
                del os.environ["HPDCT_STREAM_PIPELINE"]
            else:
                os.environ["HPDCT_STREAM_PIPELINE"] = old

    for out_dtype, name, obytes in ((torch.float32, "f32", 4), (torch.int8, "i8", 1)):
        pool_out = [torch.empty((n, n), dtype=out_dtype).pin_memory() for _ in range(8)]
        frames = [pool_in[i % 8] for i in range(mine)]
        outs = [pool_out[i % 8] for i in range(mine)]
        moved = mine * n * n * (1 + obytes)
        variants = {"streams_2": run(frames, outs, 2, "streams"), "streams_3": run(frames, outs, 3, "streams"),
                    "engines_2": run(frames, outs, 2, "engines"), "engines_3": run(frames, outs, 3, "engines")}
        ms = variants["streams_2"]  # the product's default (hpdct_stream_forward, 2 streams)
        res[name] = {"ms": round(ms, 2), "frames_per_s_total": round(frames_total / (ms * 1e-3), 1),
                     "gpx_s_total": round(frames_total * n * n / (ms * 1e-3) / 1e9, 2),
                     "pcie_GBs_per_rank": round(moved / (ms * 1e-3) / 1e9, 1), "pipeline": "streams_2",
                     "by_pipeline_frames_per_s": {k: round(frames_total / (v * 1e-3), 1) for k, v in variants.items()}}
        # correctness bit: two of the streamed output frames
        # against hpdct.forward of their pool frame on the device (outside the
        # timed runs; the copy-only ceiling below overwrites the outputs)
        ok = True
        for kf in sorted({0, min(5, mine - 1)}):
            ref = hpdct.forward(pool_in[kf].to("cuda"), out_dtype=out_dtype)
            got = pool_out[kf].to("cuda")
            torch.cuda.synchronize()
            ok = ok and (torch.equal(got.view(torch.int32), ref.view(torch.int32)) if out_dtype == torch.float32
                         else torch.equal(got, ref))
        res[name]["equals_forward"] = bool(ok) if mine > 0 else None
        # the copy-only ceiling: the same H2D and D2H bytes on two streams, no kernel
        dev_in = [torch.empty((n, n), dtype=torch.uint8, device="cuda") for _ in range(2)]
        dev_out = [torch.empty((n, n), dtype=out_dtype, device="cuda") for _ in range(2)]
        s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
        ev = [torch.cuda.Event() for _ in range(2)]

        def copies():
            for f in range(mine):
                k = f % 2
                with torch.cuda.stream(s_in):
                    dev_in[k].copy_(frames[f], non_blocking=True)
                with torch.cuda.stream(s_out):
                    outs[f].copy_(dev_out[k], non_blocking=True)
            s_in.synchronize()
            s_out.synchronize()

        copies()
        barrier()
        t0 = time.perf_counter()
        copies()
        cms = max_over_ranks((time.perf_counter() - t0) * 1e3)
        res[name]["copy_only_ceiling_frames_per_s"] = round(frames_total / (cms * 1e-3), 1)
        res[name]["copy_only_GBs_per_rank"] = round(moved / (cms * 1e-3) / 1e9, 1)
        del pool_out, outs, dev_in, dev_out, ev
    return res


def _cpu_baseline(n):
    """The oracle (sequential restatement of the reference arithmetic, the
    README's "DCT on CPU (Sequential)" column) on this host, one thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    img = oracle.rand_u8(n * n, 42).reshape(n, n)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.fdct(img)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    # all-cores variant, reported separately: the same oracle over
    # bands of tile rows, one thread each; the box's CPU share is OMP_NUM_THREADS
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1)))
    mt = []
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.fdct_threads(img, threads)
        mt.append(time.perf_counter() - t0)
    mt_med = float(np.median(mt))
    return {"value": round(n * n / med / 1e9, 5), "unit": "Gpixel/s", "cores": 1, "kind": "port",
            "sample": f"full {n}x{n} frame (srand(42) rand()%256), forward DCT + quantise, median of 3 runs "
                      f"({med:.3f} s each), 1 thread, gcc -O3 -ffp-contract=off",
            "ms_per_frame": round(med * 1e3, 1), "host_cpu": model, "host_nproc": os.cpu_count(),
            "all_cores": {"value": round(n * n / mt_med / 1e9, 5), "unit": "Gpixel/s", "cores": threads,
                          "ms_per_frame": round(mt_med * 1e3, 1),
                          "sample": "same frame and oracle, tile-row bands on a thread pool, median of 3"}}


if __name__ == "__main__":
    sys.exit(main())
