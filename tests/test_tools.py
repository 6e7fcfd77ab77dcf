"""The exhaustive arithmetic proofs the kernels rely on (DESIGN.md
"Arithmetic contract"), re-run on the CPU:

- verify_round3.c: trunc(x + copysign(0.49999997f, x)) == roundf(x) for all
  2^32 fp32 bit patterns (~20 s);
- verify_fastdiv.c, sampled: the 3-op quotient rounds like IEEE C/Q for the
  JPEG divisors (the exhaustive CPU and GPU logs are committed next to it).
"""
import os
import re
import subprocess

import pytest

TOOLS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools")
JPEG_Q = "16 11 10 24 40 51 61 12 14 19 26 58 60 55 13 57 69 56 17 22 29 87 80 62 18 37 68 109 103 77 35 64 " \
         "81 104 113 92 49 78 121 120 101 72 95 98 112 100 99".split()


def _build(tmp_path, src, extra=()):
    exe = tmp_path / (os.path.splitext(src)[0])
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", *extra, "-o", str(exe), os.path.join(TOOLS, src), "-lm"],
                   check=True)
    return str(exe)


def test_round3_exhaustive(tmp_path):
    exe = _build(tmp_path, "verify_round3.c")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout
    assert "checked 4294967296 patterns: 0 mismatches" in p.stdout


def test_fastdiv_sampled_jpeg_table(tmp_path):
    exe = _build(tmp_path, "verify_fastdiv.c", ("-fopenmp",))
    p = subprocess.run([exe, "--stride", "61", *JPEG_Q], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout
    assert re.search(r"checked 47 divisors x \d+ floats: \d+ quotient mismatches, 0 rounding mismatches", p.stdout)


@pytest.mark.parametrize("log,pattern", [
    ("verify_fastdiv.cpu.log", r"checked 47 divisors x 1166016513 floats: \d+ quotient mismatches, 0 rounding"),
    ("verify_fastdiv.gpu.log", r"divisors 1\.\.255 x 1166016513 values: 0 rounding mismatches"),
])
def test_committed_exhaustive_logs(log, pattern):
    text = open(os.path.join(TOOLS, log)).read()
    assert re.search(pattern, text)


def test_rt_pair_trace_reads_overlap_and_period(tmp_path):
    """tools/rt_pair_trace.py: on a synthetic trace where
    each fold's traced start lies 3 us before its round trip's end, it reports
    the overlap, the fold's tail behind the round trip and the pair period."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(TOOLS), "..", "tools"))
    import rt_pair_trace as rp
    csv_path = tmp_path / "kernel_trace.csv"
    rows = ["Kind,Dispatch_Id,Queue_Id,Kernel_Name,Grid_Size_X,Start_Timestamp,End_Timestamp"]
    t = 1_000_000
    for i in range(4):
        rows.append(f"KERNEL_DISPATCH,{2 * i},1,\"void hpdct::roundtrip_duo_kernel<true, 2>(...)\",2097152,"
                    f"{t},{t + 73000}")
        rows.append(f"KERNEL_DISPATCH,{2 * i + 1},1,\"void hpdct::rt_spread_finish_kernel<64>(...)\",64,"
                    f"{t + 70000},{t + 74900}")
        t += 75000
    csv_path.write_text("\n".join(rows) + "\n")
    ps = rp.pairs(rp.load(str(csv_path)), 2097152)
    assert len(ps) == 4
    assert all(abs(p["gap"] + 3.0) < 1e-9 and abs(p["tail"] - 1.9) < 1e-9 and abs(p["fin"] - 4.9) < 1e-9
               for p in ps)
    assert [p["period"] for p in ps] == [75.0, 75.0, 75.0, None]
