#!/bin/bash
# One GPU-box session (round 2): smoke -> parity tests -> the driver's exact
# bench command, plain and under rocprofv3 --kernel-trace --stats in the same
# session (the profiled bench prints its own line, committed beside the
# summary) -> the N=2 self-launched gloo rehearsal.
# Stops at the first step that faults / aborts / times out; a plain test
# failure (pytest exit 1) still lets the bench run.
# Usage (from the repo root on the box): tools/gpu_r02.sh [steps...]
#   steps: any of smoke tests bench prof n2 (default: all, in that order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    return $rc
}

want=${*:-smoke tests bench prof n2}
for s in $want; do
    case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    tests)
        step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
        rc=$?; [ $rc -le 1 ] || exit $rc ;;
    bench) step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    prof)
        (cd /tmp && step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/prof_bench" -o hpdct -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5) || exit $?
        python3 tools/trace_summary.py "$(ls "$OUT"/prof_bench/*/hpdct_kernel_trace.csv "$OUT"/prof_bench/hpdct_kernel_trace.csv 2>/dev/null | head -n1)" \
            --bench "$OUT/rocprof_bench.log" --warmup 5 --steps 20 --out "$OUT/trace_summary.md" > /dev/null || true ;;
    n2) step bench_n2_gloo 600 python3 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo ALLDONE
