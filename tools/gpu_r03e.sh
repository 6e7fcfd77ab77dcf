# round 3, session e: the exhaustive check of two shorter quantiser forms
# (tests/tools/verify_quant1.hip), the SDWA level-shift convert A/B and the
# row-by-row first pass A/B
mkdir -p gpurun_out/r03e
timeout -k 10 240 tests/tools/verify_quant1 4096 > gpurun_out/r03e/verify_quant1.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 cvt 16 > gpurun_out/r03e/kb3_cvt16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 cvti8 16 > gpurun_out/r03e/kb3_cvti8_16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 rows 16 > gpurun_out/r03e/kb3_rows16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 rowsi8 16 > gpurun_out/r03e/kb3_rowsi8_16.log 2>&1 || exit $?
echo done
