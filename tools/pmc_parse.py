#!/usr/bin/env python3
"""Turn the rocprofv3 PMC passes of tools/pmc_traffic.sh into per-launch HBM
bytes for the path's kernels (profiles/pmc_traffic.json): the headline
u8 -> fp32 kernel, the int8 forward, the fp32 duo forward / inverse, the
fp32 -> u8 duo inverse and the one-pass round trip.

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch.  Each is scaled by
the ratio (known bytes / counted bytes) measured on a calibration kernel of
the same access width (tools/membench calib): dwordx2 loads for the uint8
reads, dwordx4 loads for fp32, dwordx4 / dwordx2 non-temporal stores
(MI355X_MICROARCH.md "HBM": FETCH_SIZE reads 1/2 of a wide streaming read on
gfx950; other widths must be calibrated).

usage: tools/pmc_parse.py gpurun_out/pmc [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

CALIB_BYTES = 256 << 20


def per_dispatch(dirpath, counter):
    """{(kernel_name, grid_size): [value per dispatch]} from a rocprofv3 counter csv."""
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    files += glob.glob(dirpath + ".counter_collection.csv")  # the flattened copies under profiles/
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            out.setdefault((r["Kernel_Name"], int(r.get("Grid_Size") or 0)), []).append(float(r["Counter_Value"]))
    return out


def pick(d, needle, exclude=(), grid=None):
    """dispatch values of the first kernel whose name holds needle (and none of
    exclude), at the given grid size (threads) when one is given: since round 3
    the headline kernel also runs the C2 batch (same name, a smaller grid)"""
    for (name, g), v in d.items():
        if needle in name and not any(e in name for e in exclude) and (grid is None or g == grid):
            return v
    raise KeyError(needle)


# kernel key -> (name needle, exclude, read width, write width, B/px read, B/px written); a write
# width may be a {width: B/px} mix, calibrated per part (the round trip stores fp32 rows and u8 rows)
KERNELS = {
    # round 6: the headline runs on the duo forward (hpdct_rt_duo.hpp fdct_duo_u8_kernel)
    "fdct_u8_f32": ("fdct_duo_u8_kernel<2>", (), "x2", "x4nt", 1, 4),
    "fdct_u8_i8": ("fdct_kernel<unsigned char, signed char, true, true, false", (), "x2", "x2nt", 1, 1),
    "fdct_f32_f32_duo_runtimeT": ("fdct_duo_kernel<true, false, false", (), "x4", "x4nt", 4, 4),
    "idct_f32_f32_duo": ("idct_duo_kernel<true, true", ("unsigned char",), "x4", "x4nt", 4, 4),
    "idct_f32_u8_duo": ("idct_duo_kernel<true, true, 8208u, unsigned char>", (), "x4", "x2nt", 4, 1),
    # round 5: the two-lanes-per-tile kernel (hpdct_rt_duo.hpp) is what hpdct_roundtrip_u8 launches at 8192^2
    "roundtrip_u8_f32_u8_sums": ("roundtrip_duo_kernel<true, 2, 1, true, 256, 6", (), "x2", {"x4nt": 4, "x2nt": 1}, 1, 5),
    # the drop-in surface (bench.py extras "dropin": what hpdct_compat.cpp launches)
    "compat_fwd_f32_wb": ("fdct_duo_kernel<true, false, true", (), "x4", "x4nt", 4, 8),  # write-back NT since r05
    "compat_inv_f32": ("idct_duo_kernel<true, false", ("unsigned char",), "x4", "x4nt", 4, 4),
    "compat_fwd_rowfirst_wb": ("rowfirst_duo_kernel<false, true, false, true", (), "x4", "x4nt", 4, 8),
    "compat_inv_rowfirst_wb": ("rowfirst_duo_kernel<true, true, false, true", (), "x4", "x4nt", 4, 8),
}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    fetch = per_dispatch(os.path.join(src, "bench_FETCH_SIZE"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(src, "bench_WRITE_SIZE"), "WRITE_SIZE")
    cf = per_dispatch(os.path.join(src, "calib_FETCH_SIZE"), "FETCH_SIZE")
    cw = per_dispatch(os.path.join(src, "calib_WRITE_SIZE"), "WRITE_SIZE")
    counted = {
        "x2": statistics.median(pick(cf, "calib_read_x2")) * 1024,
        "x4": statistics.median(pick(cf, "read_only")) * 1024,
        "x4nt": statistics.median(pick(cw, "write_only<true>")) * 1024,
        "x4plain": statistics.median(pick(cw, "write_only<false>")) * 1024,
    }
    try:
        counted["x2nt"] = statistics.median(pick(cw, "calib_write_x2_nt")) * 1024
    except KeyError:  # older calibration run without the dwordx2 NT store kernel
        counted["x2nt"] = float(CALIB_BYTES)
    scale = {k: CALIB_BYTES / v for k, v in counted.items()}
    n = 8192
    kernels = {}
    for key, (needle, excl, rw, ww, rb, wb) in KERNELS.items():
        # launch grid at 8192^2: one lane per tile for the tile kernels, two for duo
        grid = n * n // 32 if "duo" in needle else n * n // 64
        try:
            kf = statistics.median(pick(fetch, needle, excl, grid))
            kw = statistics.median(pick(write, needle, excl, grid))
        except KeyError:
            continue
        read_b = kf * 1024 * scale[rw]
        if isinstance(ww, dict):  # bytes-weighted mean of the parts' calibration scales
            write_b = kw * 1024 * sum(scale[w] * b for w, b in ww.items()) / sum(ww.values())
            ww = "+".join(ww)
        else:
            write_b = kw * 1024 * scale[ww]
        alg = (rb + wb) * n * n
        kernels[key] = {
            "kernel": needle,
            "size": n,
            "fetch_size_kib_raw": kf, "write_size_kib_raw": kw,
            "read_width": rw, "write_width": ww,
            "hbm_read_bytes_per_launch": round(read_b),
            "hbm_write_bytes_per_launch": round(write_b),
            "hbm_bytes_per_launch": round(read_b + write_b),
            "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": round((read_b + write_b) / alg, 4),
        }
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/pmc_traffic.sh",
        "calibration": {
            "known_bytes": CALIB_BYTES,
            "counted": counted,
            "scale": scale,
        },
        "kernels": kernels,
    }
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
