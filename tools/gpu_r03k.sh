#!/bin/bash
# Round-3 probe session k: VALU issue cost of v_fma_f32 vs v_pk_fma_f32 at
# 1/2/4 waves per SIMD, the banded forward with the packed transform, and the
# product-shaped forward with the packed transform (fp32 and int8 out).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r03k
mkdir -p "$OUT"
for g in ${*:-issue bandpk}; do
    timeout -k 10 300 tools/kbench3 8192 64 3 $g 16 > "$OUT/kb3_${g}16.log" 2>&1 || exit $?
done
echo ALLDONE
