# round 3, session f: smallest mismatching |C| of the shorter quantiser forms
# per divisor (tests/tools/verify_quant1.hip), their timing A/B, and the
# row-by-row first pass again
mkdir -p gpurun_out/r03f
timeout -k 10 240 tests/tools/verify_quant1 1100 > gpurun_out/r03f/verify_quant1_1100.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 fq 16 > gpurun_out/r03f/kb3_fq16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 fqi8 16 > gpurun_out/r03f/kb3_fqi8_16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 rows 16 > gpurun_out/r03f/kb3_rows16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 rowsi8 16 > gpurun_out/r03f/kb3_rowsi8_16.log 2>&1 || exit $?
echo done
