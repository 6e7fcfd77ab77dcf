#!/usr/bin/env python3
"""Turn the rocprofv3 PMC passes of tools/pmc_traffic.sh into per-launch HBM
bytes for the headline kernel (profiles/pmc_traffic.json).

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch.  Each is scaled by
the ratio (known bytes / counted bytes) measured on a calibration kernel of
the same access width (tools/membench calib): dwordx2 loads for the uint8
reads, dwordx4 non-temporal stores for the fp32 writes
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
    """{kernel_name: [value per dispatch]} from a rocprofv3 counter csv."""
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def pick(d, needle, exclude=()):
    for k, v in d.items():
        if needle in k and not any(e in k for e in exclude):
            return v
    raise KeyError(needle)


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    fetch = per_dispatch(os.path.join(src, "bench_FETCH_SIZE"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(src, "bench_WRITE_SIZE"), "WRITE_SIZE")
    cf = per_dispatch(os.path.join(src, "calib_FETCH_SIZE"), "FETCH_SIZE")
    cw = per_dispatch(os.path.join(src, "calib_WRITE_SIZE"), "WRITE_SIZE")
    kf = statistics.median(pick(fetch, "fdct_kernel<unsigned char, float"))
    kw = statistics.median(pick(write, "fdct_kernel<unsigned char, float"))
    read_x2 = statistics.median(pick(cf, "calib_read_x2")) * 1024
    read_x4 = statistics.median(pick(cf, "read_only")) * 1024
    wr_nt = statistics.median(pick(cw, "write_only<true>")) * 1024
    wr_plain = statistics.median(pick(cw, "write_only<false>")) * 1024
    f_scale = CALIB_BYTES / read_x2
    w_scale = CALIB_BYTES / wr_nt
    n = 8192
    alg_read, alg_write = n * n, 4 * n * n
    read_b = kf * 1024 * f_scale
    write_b = kw * 1024 * w_scale
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/pmc_traffic.sh",
        "calibration": {
            "known_bytes": CALIB_BYTES,
            "fetch_dwordx2_counted": read_x2, "fetch_dwordx4_counted": read_x4,
            "write_dwordx4_nt_counted": wr_nt, "write_dwordx4_plain_counted": wr_plain,
            "fetch_scale_used": f_scale, "write_scale_used": w_scale,
        },
        "kernels": {
            "fdct_u8_f32": {
                "size": n,
                "fetch_size_kib_raw": kf, "write_size_kib_raw": kw,
                "hbm_read_bytes_per_launch": round(read_b),
                "hbm_write_bytes_per_launch": round(write_b),
                "hbm_bytes_per_launch": round(read_b + write_b),
                "algorithmic_bytes_per_launch": alg_read + alg_write,
                "traffic_over_algorithmic": round((read_b + write_b) / (alg_read + alg_write), 4),
            }
        },
    }
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
