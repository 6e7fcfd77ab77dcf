#!/bin/bash
# One GPU-box session, any mix of named steps, run in order; replaces the
# per-session scripts of rounds 1-3 (gpu_check.sh, gpu_r02.sh, gpu_r03*.sh).
#
#   tools/gpu_session.sh <out> <step>...        (from the repo root on the box)
#
# <out>: directory under gpurun_out/ for the logs (steps.log lists every step
# with its exit code).  Steps:
#   smoke                 __graft_entry__.smoke()
#   tests                 pytest -m gpu (thread timeout per test)
#   tests:<expr>          pytest -m gpu -k <expr>
#   bench                 the driver's exact bench command
#   prof                  the same under rocprofv3 --kernel-trace --stats, plus
#                         tools/trace_summary.py over its kernel trace
#   shard                 benchmark_hpdct 16384 --gpus 1 (fp32 and int8)
#   n2                    bench.py --gpus 2 --backend gloo (two ranks, one GPU)
#   kb:<args>             tools/kbench3 with <args> (':' separated), e.g.
#                         kb:8192:64:3:occsz:16 -> log kb3_occsz_8192.log
#   pmcsq:<args>          SQ/GRBM counter pass over kbench3 <args>
#   pmctcc:<args>         TCC/TA counter pass over kbench3 <args>
#   pmcrd:<args>          TCC read and write request pass over kbench3 <args>
#   verify_quant:<xmax>   tests/tools/verify_quant1 (exhaustive quantiser proof)
#   kbd[:<args>]          tools/kb_decode (int8 -> fp32 decode A/B)
#   devinfo               HIP device attributes the launch code reads
#   pmctraffic            HBM bytes of the path's kernels: tools/pmc_traffic.sh (FETCH_SIZE and
#                         WRITE_SIZE in separate passes + calibration), parsed into
#                         <out>/pmc_traffic.json by tools/pmc_parse.py
# The session stops at the first step that faults, aborts or times out (exit
# >= 2 or a signal); a plain test failure (pytest exit 1) lets later steps run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
[ $# -ge 1 ] || { echo "usage: $0 <out> <step>..."; exit 2; }
OUT=$ROOT/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
TCC="TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE"
RD="TCC_EA0_RDREQ TCC_EA0_WRREQ GRBM_GUI_ACTIVE"

step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    return $rc
}
pmc() {  # pmc <name> <counters> <kbench3 args...>: a counter-only pass, its own run
    local name=$1 ctr=$2; shift 2
    echo "== pmc $name: $ctr" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$name" -o run \
        -- "$ROOT/tools/kbench3" "$@" > "$OUT/pmc_$name.log" 2>&1)
    local rc=$?
    echo "== pmc $name rc=$rc" | tee -a "$OUT/steps.log"
    return $rc
}
bench_cmd=(python3 bench.py --gpus 1 --steps 20 --warmup 5)

for s in "$@"; do
    IFS=: read -r -a p <<< "$s"
    case ${p[0]} in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    tests)
        k=()
        [ ${#p[@]} -gt 1 ] && k=(-k "${p[1]}")
        step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread "${k[@]}"
        rc=$?; [ $rc -le 1 ] || exit $rc ;;
    bench) step bench 600 "${bench_cmd[@]}" || exit $? ;;
    prof)
        (cd /tmp && step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/prof_bench" -o hpdct -- "${bench_cmd[@]/#bench.py/$ROOT/bench.py}") || exit $?
        python3 tools/trace_summary.py "$(ls "$OUT"/prof_bench/*/hpdct_kernel_trace.csv \
            "$OUT"/prof_bench/hpdct_kernel_trace.csv 2>/dev/null | head -n1)" \
            --bench "$OUT/rocprof_bench.log" --warmup 5 --steps 20 --out "$OUT/trace_summary.md" > /dev/null || true
        python3 tools/rt_pair_trace.py "$(ls "$OUT"/prof_bench/*/hpdct_kernel_trace.csv \
            "$OUT"/prof_bench/hpdct_kernel_trace.csv 2>/dev/null | head -n1)" --grid 2097152 \
            --out "$OUT/rt_pairs.md" > /dev/null || true ;;
    shard)
        step shard_f32 120 cuda-dct-idct_amd/bin/benchmark_hpdct 16384 5 --gpus 1 || exit $?
        step shard_i8 120 cuda-dct-idct_amd/bin/benchmark_hpdct 16384 5 --gpus 1 --int8 || exit $? ;;
    n2) step bench_n2_gloo 600 python3 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
            || exit $? ;;
    kb) step "kb3_${p[4]}_${p[1]}" 300 tools/kbench3 "${p[@]:1}" || exit $? ;;
    pmcsq) pmc "sq_${p[4]}_${p[1]}" "$SQ" "${p[@]:1}" || exit $? ;;
    pmctcc) pmc "tcc_${p[4]}_${p[1]}" "$TCC" "${p[@]:1}" || exit $? ;;
    pmcrd) pmc "rd_${p[4]}_${p[1]}" "$RD" "${p[@]:1}" || exit $? ;;
    verify_quant) step "verify_quant1_${p[1]:-4096}" 300 tests/tools/verify_quant1 "${p[1]:-4096}" || exit $? ;;
    devinfo) step devinfo 120 python3 tools/devinfo.py || exit $? ;;
    kbd) step kb_decode 300 tools/kb_decode "${p[@]:1}" || exit $? ;;
    pmctraffic)
        step pmc_traffic 900 tools/pmc_traffic.sh || exit $?
        python3 tools/pmc_parse.py gpurun_out/pmc "$OUT/pmc_traffic.json" > "$OUT/pmc_parse.log" 2>&1 || true ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo ALLDONE
