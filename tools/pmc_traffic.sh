#!/bin/bash
# HBM traffic of the path's kernels (headline, int8, fp32 duo forward and
# inverse; every launch at 8192^2) from rocprofv3 PMC counters, collected
# as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE and WRITE_SIZE in
# SEPARATE passes (they do not fit one pass), counters only (no trace
# domains), plus calibration kernels of known byte count with the same access
# widths (tools/membench calib) to correct the gfx950 FETCH_SIZE under-count.
# Output: gpurun_out/pmc/*  ->  tools/pmc_parse.py -> profiles/pmc_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/bench_$ctr" -o run -- \
        python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-c4c5 --sustain-s 0 > "$OUT/bench_$ctr.log" 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/calib_$ctr" -o run -- \
        "$ROOT/tools/membench" calib > "$OUT/calib_$ctr.log" 2>&1 || exit $?
done
echo PMCDONE
