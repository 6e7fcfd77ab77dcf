"""Host-side logic of bench.py (no GPU): the JSON line's derived numbers and
the CPU-baseline block, so the driver's contract fields are checked on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_line_derives_rates_from_times():
    px, ms_step, kern_ms = 8192 * 8192, 0.05, 0.05
    line = bench._line(px, ms_step, kern_ms, 5, 1)
    assert line["gpx_s"] == pytest.approx(px / 50e-6 / 1e9, rel=1e-3)
    assert line["achieved_GBs"] == pytest.approx(5 * px / 50e-6 / 1e9, rel=1e-3)
    assert line["hbm_frac"] == pytest.approx(line["achieved_GBs"] / bench.HBM_PEAK_GBS, rel=1e-3)
    # whole-job throughput scales with the rank count, the per-GPU HBM fraction does not
    line8 = bench._line(px, ms_step, kern_ms, 5, 8)
    assert line8["gpx_s"] == pytest.approx(8 * line["gpx_s"], rel=1e-3)
    assert line8["hbm_frac"] == line["hbm_frac"]


def test_cpu_baseline_block_small_frame():
    res = bench._cpu_baseline(256)
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in res
    assert res["unit"] == "Gpixel/s" and res["cores"] == 1 and res["kind"] == "port"
    assert res["value"] > 0
    assert res["all_cores"]["cores"] >= 1 and res["all_cores"]["value"] > 0


def test_defaults_are_the_driver_contract(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()
    assert args.gpus == 1 and args.size == 8192 and args.sets >= 3
    assert args.steps > 0 and args.warmup > 0 and args.backend == "nccl"
    assert bench.BYTES_PER_PX["u8_f32"] == 5 and bench.HBM_PEAK_GBS == 8000.0
