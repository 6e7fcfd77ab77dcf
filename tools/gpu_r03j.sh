# round 3, session j: staggered start of the first workgroups (the per-launch ramp)
mkdir -p gpurun_out/r03j
timeout -k 10 200 tools/kbench3 8192 64 3 stag 16 > gpurun_out/r03j/kb3_stag16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 stagi8 16 > gpurun_out/r03j/kb3_stagi8_16.log 2>&1 || exit $?
echo done
