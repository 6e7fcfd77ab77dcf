#!/bin/bash
# One GPU-box session (round 3): smoke -> GPU tests -> the driver's exact bench
# command, plain and under rocprofv3 --kernel-trace --stats (the profiled bench
# prints its own line) -> the single-process sharded driver at --gpus 1 -> the
# N=2 self-launched gloo rehearsal -> PMC passes on the headline kernel and its
# LDS-DMA variant (tools/kbench3 "fwd" group).
# Stops at the first step that faults / aborts / times out; a plain test
# failure (pytest exit 1) still lets the bench run.
# Usage (from the repo root on the box): tools/gpu_r03.sh [steps...]
#   steps: any of smoke tests bench prof shard n2 pmcdma (default: all but pmcdma)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r03
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
pmc() {  # pmc <name> <counters> -- cmd...   (counter-only pass, its own run and time limit)
    local name=$1 ctr=$2; shift 3
    echo "== pmc $name: $ctr" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$name" -o run -- "$@" \
        > "$OUT/pmc_$name.log" 2>&1)
    local rc=$?
    echo "== pmc $name rc=$rc" | tee -a "$OUT/steps.log"
    return $rc
}

want=${*:-smoke tests bench prof shard n2}
for s in $want; do
    case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    tests)
        step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
        rc=$?; [ $rc -le 1 ] || exit $rc ;;
    bench) step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    prof)
        (cd /tmp && step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/prof_bench" -o hpdct -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5) || exit $?
        python3 tools/trace_summary.py "$(ls "$OUT"/prof_bench/*/hpdct_kernel_trace.csv "$OUT"/prof_bench/hpdct_kernel_trace.csv 2>/dev/null | head -n1)" \
            --bench "$OUT/rocprof_bench.log" --warmup 5 --steps 20 --out "$OUT/trace_summary.md" > /dev/null || true ;;
    shard)
        step shard_f32 120 cuda-dct-idct_amd/bin/benchmark_hpdct 16384 5 --gpus 1 || exit $?
        step shard_i8 120 cuda-dct-idct_amd/bin/benchmark_hpdct 16384 5 --gpus 1 --int8 || exit $? ;;
    n2) step bench_n2_gloo 600 python3 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline || exit $? ;;
    pmcdma)
        pmc dma_tcc "TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" \
            -- "$ROOT/tools/kbench3" 8192 16 1 fwd 16 || exit $?
        pmc dma_sq "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            -- "$ROOT/tools/kbench3" 8192 16 1 fwd 16 || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo ALLDONE
