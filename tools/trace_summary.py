#!/usr/bin/env python3
"""Per-launch summary of a rocprofv3 --kernel-trace CSV, grouped by kernel and
launch shape, set beside the bench JSON line recorded in the same session.

  python tools/trace_summary.py <kernel_trace.csv> [--bench <bench.json>]
         [--warmup W] [--steps K] [--out summary.md]

The bench's headline kernel (fdct_duo_u8_kernel<2> since round 6, before it
fdct_kernel<u8, f32, ...>, at the 8192^2 grid) is also launched later by
other extras at the same shape, so the headline's own launches are picked by
dispatch order: after W warm-up launches and the bench's untimed lead-in
(`warmup_lead_in_launches` of the bench line, when --bench is given), the
next K are the timed region.
Every other group is summarised whole (count, mean, median, min, max) and
over its last 100 launches (the extras' timed region).
"""
import argparse
import csv
import json
import re
import statistics
import sys


def short_name(name: str) -> str:
    m = re.match(r"(?:void )?([\w:]+)(<[^()]*>)?", name)
    if not m:
        return name[:80]
    base = m.group(1).replace("hpdct::", "")
    targs = m.group(2) or ""
    targs = targs.replace("unsigned char", "u8").replace("signed char", "i8").replace("float", "f32")
    targs = targs.replace("true", "T").replace("false", "F").replace(" ", "")
    return base + targs


def load(path):
    rows = []
    with open(path, newline="") as fh:
        for r in csv.DictReader(fh):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append({
                "id": int(r["Dispatch_Id"]),
                "name": short_name(r["Kernel_Name"]),
                "grid": int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1),
                "wg": int(r["Workgroup_Size_X"]),
                "vgpr": int(r.get("VGPR_Count", 0) or 0),
                "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
            })
    rows.sort(key=lambda r: r["id"])
    return rows


def stats(us):
    return {"calls": len(us), "mean_us": round(statistics.fmean(us), 2), "median_us": round(statistics.median(us), 2),
            "min_us": round(min(us), 2), "max_us": round(max(us), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bench", help="file holding the bench JSON line of the same session")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--headline-grid", type=int, default=(8192 * 8192 // 64 // 32) * 64,
                    help="threads of the headline launch (duo forward: one wave per 32 tiles; the round-5 tile "
                         "kernel: (8192*8192//64//64)*64)")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.trace)
    groups = {}
    for r in rows:
        groups.setdefault((r["name"], r["grid"], r["wg"]), []).append(r)
    lines = ["| kernel | grid (threads) | wg | VGPR | calls | mean us | median | min | max | last-100 mean |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    summary = {"groups": []}
    for (name, grid, wg), rs in sorted(groups.items(), key=lambda kv: -sum(r["us"] for r in kv[1])):
        us = [r["us"] for r in rs]
        st = stats(us)
        st.update(kernel=name, grid=grid, wg=wg, vgpr=rs[0]["vgpr"],
                  last100_mean_us=round(statistics.fmean(us[-100:]), 2))
        summary["groups"].append(st)
        lines.append(f"| `{name}` | {grid} | {wg} | {rs[0]['vgpr']} | {st['calls']} | {st['mean_us']} | "
                     f"{st['median_us']} | {st['min_us']} | {st['max_us']} | {st['last100_mean_us']} |")
    head = [r for r in rows if r["name"].startswith(("fdct_duo_u8_kernel<", "fdct_kernel<u8,f32,")) and
            r["grid"] == a.headline_grid]
    line = None
    if a.bench:
        with open(a.bench) as fh:
            for ln in fh:
                ln = ln.strip()
                if ln.startswith("{") and '"metric"' in ln:
                    line = json.loads(ln)
    lead = int((line or {}).get("warmup_lead_in_launches", 0) or 0)
    first = a.warmup + lead
    out = "\n".join(lines) + "\n"
    if len(head) >= first + a.steps:
        timed = [r["us"] for r in head[first:first + a.steps]]
        hs = stats(timed)
        summary["headline_timed"] = hs
        out += (f"\nHeadline timed region (launches {first}..{first + a.steps - 1} of "
                f"`{head[0]['name']}` at grid {a.headline_grid}): mean {hs['mean_us']} us, median "
                f"{hs['median_us']}, min {hs['min_us']}, max {hs['max_us']}\n")
        frac = 5 * 8192 * 8192 / (hs["mean_us"] * 1e-6) / 8e12
        out += f"  -> 5 B/px x 8192^2 / mean = {frac:.4f} of 8 TB/s\n"
    if a.bench:
        if line:
            summary["bench"] = {"ms_per_step": line["ms_per_step"], "frac": line["roofline"]["frac"],
                                "kernel_us_avg": line["roofline"]["kernel_us_avg"]}
            out += (f"\nBench line of the same session: ms_per_step {line['ms_per_step']} "
                    f"(kernel_us_avg {line['roofline']['kernel_us_avg']}), frac {line['roofline']['frac']}\n")
            if "headline_timed" in summary:
                out += (f"  traced mean / bench avg = "
                        f"{summary['headline_timed']['mean_us'] / line['roofline']['kernel_us_avg']:.4f}\n")
            for key, ex in sorted((line.get("extras") or {}).items()):
                if isinstance(ex, dict) and "kernel_us_avg" in ex:
                    out += f"  extras.{key}: kernel_us_avg {ex['kernel_us_avg']} (hbm_frac {ex.get('hbm_frac')})\n"
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(out)
        with open(a.out.rsplit(".", 1)[0] + ".json", "w") as fh:
            json.dump(summary, fh, indent=1)
    sys.stdout.write(out)


if __name__ == "__main__":
    main()
