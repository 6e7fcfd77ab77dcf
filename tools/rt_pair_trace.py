#!/usr/bin/env python3
"""Start/end stamps of consecutive (round trip, sums fold) pairs in a
rocprofv3 --kernel-trace CSV: does the traced duration of
the one-wave rt_spread_finish_kernel overlap the round trip before it, and
what does one pair cost from one round trip's start to the next's?

  python tools/rt_pair_trace.py <kernel_trace.csv> [--grid N] [--name SUBSTR] [--last K] [--out pairs.md]

A pair is a roundtrip_duo_kernel dispatch followed, on the same queue, by an
rt_spread_finish_kernel dispatch.  Per pair (times in us):
  rt        round trip end - start
  fin       fold end - start
  gap       fold start - round-trip end (negative: the fold's traced start
            lies before the round trip has ended)
  tail      fold end - round-trip end (what the fold adds behind the round trip)
  period    next pair's round-trip start - this round-trip start, when the
            next dispatch on the queue is that next round trip (back to back)
Development tool; reads a trace, runs nothing.
"""
import argparse
import csv
import statistics
import sys


def load(path):
    rows = []
    with open(path, newline="") as fh:
        for r in csv.DictReader(fh):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append({"id": int(r["Dispatch_Id"]), "queue": r.get("Queue_Id", "0"), "name": r["Kernel_Name"],
                         "grid": int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1),
                         "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])})
    rows.sort(key=lambda r: r["id"])
    return rows


def pairs(rows, grid=None, name=None):
    by_q = {}
    for r in rows:
        by_q.setdefault(r["queue"], []).append(r)
    out = []
    for q in by_q.values():
        for i in range(len(q) - 1):
            a, b = q[i], q[i + 1]
            if "roundtrip_duo_kernel" not in a["name"] or "rt_spread_finish_kernel" not in b["name"]:
                continue
            if grid is not None and a["grid"] != grid:
                continue
            if name is not None and name not in a["name"]:
                continue
            nxt = q[i + 2] if i + 2 < len(q) else None
            period = None
            if nxt is not None and nxt["name"] == a["name"] and nxt["grid"] == a["grid"]:
                period = (nxt["t0"] - a["t0"]) / 1e3
            out.append({"name": a["name"][:60], "grid": a["grid"], "rt": (a["t1"] - a["t0"]) / 1e3,
                        "fin": (b["t1"] - b["t0"]) / 1e3, "gap": (b["t0"] - a["t1"]) / 1e3,
                        "tail": (b["t1"] - a["t1"]) / 1e3, "period": period})
    return out


def legs(rows, name=None, min_pairs=50):
    """Runs of back-to-back pairs (round trip, fold, round trip, fold, ... with
    nothing else in between on the queue): one per bench leg.  Per leg, over
    its last 100 pairs (the leg's timed launches): mean period, round trip,
    fold, and the two gaps (fold start - round-trip end, next round-trip
    start - fold end)."""
    by_q = {}
    for r in rows:
        by_q.setdefault(r["queue"], []).append(r)
    out = []
    for q in by_q.values():
        found = [(i, q[i], q[i + 1]) for i in range(len(q) - 1)
                 if "roundtrip_duo_kernel" in q[i]["name"] and "rt_spread_finish_kernel" in q[i + 1]["name"] and
                 (name is None or name in q[i]["name"])]
        cur = []
        for x in found:
            if cur and (x[0] != cur[-1][0] + 2 or x[1]["name"] != cur[-1][1]["name"]):
                if len(cur) >= min_pairs:
                    out.append(cur)
                cur = []
            cur.append(x)
        if len(cur) >= min_pairs:
            out.append(cur)
    res = []
    for leg in out:
        tail = leg[-100:]
        per = [(tail[k + 1][1]["t0"] - tail[k][1]["t0"]) / 1e3 for k in range(len(tail) - 1)]
        res.append({"pairs": len(leg), "name": leg[0][1]["name"][:60],
                    "period": statistics.fmean(per) if per else None,
                    "rt": statistics.fmean((x[1]["t1"] - x[1]["t0"]) / 1e3 for x in tail),
                    "fin": statistics.fmean((x[2]["t1"] - x[2]["t0"]) / 1e3 for x in tail),
                    "gap_rt_fin": statistics.fmean((x[2]["t0"] - x[1]["t1"]) / 1e3 for x in tail),
                    "gap_fin_next": statistics.fmean((tail[k + 1][1]["t0"] - tail[k][2]["t1"]) / 1e3
                                                     for k in range(len(tail) - 1)) if len(tail) > 1 else None})
    return res


def summary(vals):
    vals = [v for v in vals if v is not None]
    if not vals:
        return "-"
    return (f"{statistics.fmean(vals):.2f} / {statistics.median(vals):.2f} / {min(vals):.2f} / {max(vals):.2f}"
            f" (n={len(vals)})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--grid", type=int, default=None, help="only round trips of this grid size (threads)")
    ap.add_argument("--name", default=None, help="only round trips whose kernel name contains this")
    ap.add_argument("--last", type=int, default=0, help="only the last K pairs (a bench leg's timed launches)")
    ap.add_argument("--out")
    a = ap.parse_args()
    ps = pairs(load(a.trace), a.grid, a.name)
    if a.last:
        ps = ps[-a.last:]
    if not ps:
        print("no (roundtrip_duo_kernel, rt_spread_finish_kernel) pairs found", file=sys.stderr)
        return 1
    lines = ["| per pair, us | mean / median / min / max |", "|---|---|"]
    for k, label in (("rt", "round trip (end - start)"), ("fin", "fold (end - start)"),
                     ("gap", "fold start - round-trip end"), ("tail", "fold end - round-trip end"),
                     ("period", "round-trip start to next round-trip start (back to back)")):
        lines.append(f"| {label} | {summary([p[k] for p in ps])} |")
    overlap = sum(1 for p in ps if p["gap"] < 0)
    lines.append("")
    lines.append(f"{len(ps)} pairs ({ps[0]['name']}, grid {ps[0]['grid']}); fold's traced start before the round "
                 f"trip's end in {overlap} of them.")
    bb = [p for p in ps if p["period"] is not None]
    if bb:
        lines.append(f"Back-to-back pairs: mean period {statistics.fmean(p['period'] for p in bb):.2f} us against "
                     f"mean rt + fin {statistics.fmean(p['rt'] + p['fin'] for p in bb):.2f} us and mean "
                     f"rt + tail {statistics.fmean(p['rt'] + p['tail'] for p in bb):.2f} us.")
    lg = legs(load(a.trace), a.name)
    if lg:
        lines += ["", "Per leg (runs of back-to-back pairs), over each leg's last 100 pairs, us:", "",
                  "| pairs | period | round trip | fold | fold start - rt end | next rt start - fold end |",
                  "|---|---|---|---|---|---|"]
        for x in lg:
            f = lambda v: "-" if v is None else f"{v:.2f}"  # noqa: E731
            lines.append(f"| {x['pairs']} | {f(x['period'])} | {f(x['rt'])} | {f(x['fin'])} | {f(x['gap_rt_fin'])} |"
                         f" {f(x['gap_fin_next'])} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
