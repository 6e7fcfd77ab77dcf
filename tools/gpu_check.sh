#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults / aborts / times out (exit >= 2 or a
# signal); a plain test failure (pytest exit 1) still lets the bench run.
# Usage (from the repo root on the box): tools/gpu_check.sh [bench args...]
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
    tail -5 "$OUT/$name.log"
    return $rc
}

step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
rc=$?; [ $rc -le 1 ] || exit $rc
step bench 600 python bench.py "$@" || exit $?
cd /tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o hpdct -- \
    python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-extras || exit $?
# every kernel of the path (extras: fp32 duo/octet kernels, int8, baselines, C4, C5)
step rocprof_full 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_full" -o hpdct -- \
    python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --c5-frames 64 || exit $?
echo ALLDONE
