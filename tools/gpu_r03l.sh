#!/bin/bash
# Round-3 probe session l: packed round trip A/B; packed vs scalar forward,
# more rounds, two sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r03l
mkdir -p "$OUT"
timeout -k 10 300 tools/kbench3 8192 64 4 rtpk 16 > "$OUT/kb3_rtpk16.log" 2>&1 || exit $?
timeout -k 10 300 tools/kbench3 8192 128 6 pk 16 > "$OUT/kb3_pk16_r6.log" 2>&1 || exit $?
timeout -k 10 300 tools/kbench3 16384 32 4 pk 4 > "$OUT/kb3_pk16384.log" 2>&1 || exit $?
grep -hv "^check set" "$OUT"/*.log
echo ALLDONE
