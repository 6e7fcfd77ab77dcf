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
    assert args.gpus == 1 and args.size == 8192 and args.sets is None  # derived from the frame size
    assert args.steps > 0 and args.warmup > 0 and args.backend == "nccl"
    assert bench.BYTES_PER_PX["u8_f32"] == 5 and bench.HBM_PEAK_GBS == 8000.0


def test_rotating_sets_keep_inputs_out_of_the_infinity_cache():
    """Inputs of all rotating sets total >= 4x the 256 MiB Infinity Cache, so
    every timed launch reads HBM (4 sets of 64 MiB u8 frames fit the cache:
    profiles/r02/kbench2_sets_r02.log, 50 vs 61 us)."""
    mall = 256 << 20
    assert bench.MALL_BYTES == mall
    for in_bytes in (8192 * 8192, 16384 * 16384, 2048 * 16384, 32 << 20, 1 << 30):
        k = bench.sets_for(in_bytes)
        assert k * in_bytes >= 4 * mall and k >= 2
    assert bench.sets_for(8192 * 8192, minimum=4) == 16
    assert bench.sets_for(16384 * 16384) == 4
    assert bench.sets_for(2048 * 16384) == 32


def test_gpus_n_self_launches_ranks_without_torch(tmp_path):
    """`python bench.py --gpus 2` with no launcher: the parent starts 2 child
    processes with the torch.distributed env contract and never imports torch
    (no HIP in the parent: the children own the GPUs)."""
    import subprocess
    script = tmp_path / "probe.py"
    script.write_text(f"""
import json, sys
sys.path.insert(0, {ROOT!r})
import bench
seen = []
class FakeProc:
    def __init__(self, cmd, env):
        seen.append({{k: env[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}})
        self.cmd = cmd
    def poll(self):
        return 0
    def terminate(self):
        pass
bench.subprocess.Popen = FakeProc
sys.argv = ["bench.py", "--gpus", "2", "--steps", "3"]
rc = bench.main()
print(json.dumps({{"rc": rc, "seen": seen, "torch": "torch" in sys.modules}}))
""")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120)
    import json
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["rc"] == 0 and res["torch"] is False
    assert [s["RANK"] for s in res["seen"]] == ["0", "1"]
    assert all(s["WORLD_SIZE"] == "2" and s["MASTER_ADDR"] == "127.0.0.1" for s in res["seen"])
    assert len({s["MASTER_PORT"] for s in res["seen"]}) == 1


def test_gpus_n_fails_when_a_rank_fails(tmp_path):
    """A failing child makes the parent exit non-zero (and stops its peers)."""
    import subprocess
    script = tmp_path / "probe.py"
    script.write_text(f"""
import sys
sys.path.insert(0, {ROOT!r})
import bench
class FakeProc:
    n = 0
    def __init__(self, cmd, env):
        self.rank = int(env["RANK"]); self.killed = False
    def poll(self):
        return 3 if self.rank == 1 else (-15 if self.killed else None)
    def terminate(self):
        self.killed = True
bench.subprocess.Popen = FakeProc
sys.argv = ["bench.py", "--gpus", "4"]
sys.exit(bench.main())
""")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 3


def test_world_size_mismatch_is_an_error(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.main() == 2


def test_nccl_refuses_more_ranks_than_gpus():
    """--backend nccl with WORLD_SIZE > visible GPUs (0 here) exits 2 with a
    clear message before any process group, RCCL or HIP call (VERDICT r3 item
    5); gloo is the way to rehearse several ranks on fewer GPUs."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "nccl"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 2, out.stderr[-2000:]
    assert "one GPU per rank" in out.stderr and "WORLD_SIZE=2" in out.stderr
    assert out.stdout.strip() == ""


def test_sustained_phase_reports_the_slowest_rank_rate():
    """The sustained headline phase (a GPU-busy period long enough for an
    outside sampler) launches in chunks until its wall time is spent and
    rates the whole job from the slowest rank's time per launch."""
    launched = []

    class FakeTorch:
        class cuda:
            @staticmethod
            def synchronize():
                pass

    class FakeHip:
        def record(self, i):
            pass

        def elapsed(self, a, b):  # 50 us per launch on this rank
            return len(launched) * 0.05

    calls = [lambda: launched.append(1)]
    res = bench._sustained(FakeTorch, FakeHip(), calls, 0.01, 8192 * 8192, 2, lambda: None,
                           lambda x: 2 * x)  # the other rank is twice as slow
    assert res["launches_rank0"] == len(launched) and len(launched) % 64 == 0 and len(launched) > 0
    assert res["us_per_launch_max_rank"] == pytest.approx(100.0)
    assert res["gpx_s"] == pytest.approx(2 * 8192 * 8192 / 100e-6 / 1e9, rel=1e-3)


def test_sustained_phase_default_on_and_switchable(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.parse().sustain_s > 0
    monkeypatch.setattr(sys, "argv", ["bench.py", "--sustain-s", "0"])
    assert bench.parse().sustain_s == 0


def test_kernel_status_puts_every_kernel_beside_its_ceiling():
    """the line ends with {kernel: [us, ceiling_us, frac,
    status]}; "done" at >= DONE_FRAC of the copy of the kernel's own bytes,
    C5 as frames/s against the copy-only pipeline."""
    line = lambda us, ceil: {"kernel_us_avg": us, "ceiling_us": ceil}  # noqa: E731
    res = {"roofline": {"kernel_us_avg": 56.0, "copy_ceiling_us": 54.0},
           "extras": {"fwd_u8_i8": line(31.0, 22.0), "inv_f32_f32": line(86.0, 85.0),
                      "dropin": {"dct_all_blocks_cuda": line(126.0, 122.0),
                                 "idct_all_blocks (cublasDCTv2)": line(133.0, 122.0)},
                      "c3_roundtrip": {"one_pass": line(75.0, 63.0)},
                      "c2_fwd_u8_f32": {"floor": {"forward_us": 3.6, "copy_same_bytes_us": 3.3}},
                      "c5": {"i8": {"frames_per_s_total": 2500.0, "copy_only_ceiling_frames_per_s": 2800.0}}}}
    ks = bench.kernel_status(res)
    assert ks["headline_fwd_u8_f32"] == [56.0, 54.0, round(54 / 56, 3), "done"]
    assert ks["fwd_u8_i8"][3] == "open" and ks["inv_f32_f32"][3] == "done"
    assert ks["dropin.dct_all_blocks_cuda"][3] == "done"
    assert ks["dropin.idct_all_blocks_cublasv2"][2] == round(122 / 133, 3)
    assert ks["c3.one_pass"][3] == "open" and ks["c2_fwd_u8_f32"][3] == "done"
    assert ks["c5_i8_frames_per_s"] == [2500.0, 2800.0, round(2500 / 2800, 3), "open"]
