#!/bin/bash
# Round 3, session 3: occupancy-cap A/B (tools/kbench3 groups occsz, occi8b,
# invb, dropin at 8192^2; occsz at 16384^2, 4096^2 and 2048x16384 with enough
# rotating sets to exceed the Infinity Cache).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r03m
mkdir -p "$OUT"
run() {  # run <log> <timeout> args...
    local log=$1 t=$2; shift 2
    echo "== $log: kbench3 $*"
    timeout -k 10 "$t" tools/kbench3 "$@" > "$OUT/$log.log" 2>&1
}
for g in ${GROUPS8192:-occsz occi8b invb dropin}; do run "kb3_${g}_8192" 240 8192 64 3 "$g" 16 || exit $?; done
[ -n "$NOSIZES" ] && exit 0
run kb3_occsz_16384 300 16384 32 3 occsz 16 || exit $?
run kb3_occsz_4096 240 4096 128 3 occsz 64 || exit $?
run kb3_occsz_2048x16384 240 2048x16384 64 3 occsz 32 || exit $?
