#!/bin/bash
# What limits the int8 forward and the wide-row headline:
# SQ instruction / cycle counters on tools/kbench2's int8 group (product kernel
# and its phase splits: no load, no store, math only) and on the headline
# kernel across frame shapes (tools/shape_probe.py pmc).  Counter-only passes
# (no trace domains), each in its own run under its own time limit, within the
# per-pass slot limits (SQ <= 8, GRBM <= 2, TA <= 2, TCC <= 4).
# Usage: tools/pmc_limits.sh [list] [i8] [shape] [shape_tcc]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_limits
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAVE_CYCLES"
pass() {  # pass <name> <counters> -- cmd...
    local name=$1 ctr=$2; shift 3
    echo "== $name: $ctr"
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o run -- "$@" \
        > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    return $rc
}
for step in ${*:-list i8 shape}; do
    case $step in
    list) timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?" ;;
    i8)
        pass i8_sq1 "$SQ1" -- "$ROOT/tools/kbench2" 8192 16 1 i8 || exit $?
        pass i8_sq2 "$SQ2" -- "$ROOT/tools/kbench2" 8192 16 1 i8 || exit $? ;;
    shape)
        pass shape_sq1 "$SQ1" -- python3 "$ROOT/tools/shape_probe.py" pmc || exit $?
        pass shape_sq2 "$SQ2" -- python3 "$ROOT/tools/shape_probe.py" pmc || exit $? ;;
    shape_tcc)
        # per-channel write requests and write latency / stalls; TLB misses
        pass shape_tcc1 "TCC_EA0_WRREQ TCC_EA0_WRREQ_LEVEL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_TOO_MANY_EA_WRREQS_STALL TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY" \
            -- python3 "$ROOT/tools/shape_probe.py" pmc || exit $?
        pass shape_tcc2 "TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_STALL TCC_TAG_STALL TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_REQUEST TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS TCP_TCC_WRITE_REQ_LATENCY GRBM_GUI_ACTIVE GRBM_EA_BUSY" \
            -- python3 "$ROOT/tools/shape_probe.py" pmc || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo PMCDONE
