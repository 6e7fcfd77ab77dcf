#!/bin/bash
# Counter passes for round 5's limiter questions:
#   - the C3 round trip: tile-per-lane vs two-lanes-per-tile kernel, with and
#     without sums (tools/kb_rt groups pmc_*);
#   - the headline: the product kernel at cap 7 and its access pattern alone
#     at caps 4 and 7 (tools/kbench3 groups lim1 / lim4 / lim7).
# Each (group, counter set) is a rocprofv3 run of its own (SQ: 7 SQ + 1 GRBM;
# TCC: 2 TCC + 2 TA + 1 GRBM; RD: 2 TCC + 1 GRBM), never combined with
# tracing; results are summarised by tools/pmc_table.py into <out>/table.txt.
#   tools/pmc_limiter.sh <out>      (from the repo root on the GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
TCC="TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE"
RD="TCC_EA0_RDREQ TCC_EA0_WRREQ GRBM_GUI_ACTIVE"

pass() {  # pass <name> <counters> <program> <args...>
    local name=$1 ctr=$2; shift 2
    echo "== $name: $ctr" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o run \
        -- "$@" > "$OUT/$name.log" 2>&1)
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    return $rc
}

RT_GROUPS=${RT_GROUPS:-pmc_tile pmc_duo pmc_duo_nosums pmc_tile_nosums}
LIM_GROUPS=${LIM_GROUPS-lim1 lim4 lim7}
for g in $RT_GROUPS; do
    for set in SQ TCC RD; do
        pass "${g}_${set}" "${!set}" "$ROOT/tools/kb_rt" 8192 16 1 "$g" || exit $?
    done
done
for g in $LIM_GROUPS; do
    for set in SQ TCC RD; do
        pass "${g}_${set}" "${!set}" "$ROOT/tools/kbench3" 8192 16 1 "$g" 16 || exit $?
    done
done
python3 "$ROOT/tools/pmc_table.py" "$OUT" > "$OUT/table.txt" 2>&1
echo ALLDONE
