# round 3, session i: the int8 forward's per-launch overhead (VERDICT r2 item
# 5): the two library forward kernels at 8192^2 and 16384^2 (more iterations
# than session h), and SQ / GRBM counters of the int8 kernel at both sizes
mkdir -p gpurun_out/r03i
export TMPDIR=/tmp
# wave-specialised forward (tools/kbench_spec.hpp): pattern first, then the real kernel
timeout -k 10 120 tools/kbench3 8192 64 3 specpat 16 > gpurun_out/r03i/kb3_specpat16.log 2>&1 || exit $?
timeout -k 10 120 tools/kbench3 8192 64 3 spec 16 > gpurun_out/r03i/kb3_spec16.log 2>&1 || exit $?
for spec in "8192 16" "16384 4"; do
    set -- $spec
    timeout -k 10 200 tools/kbench3 $1 128 5 libi8 $2 > gpurun_out/r03i/kb3_libi8_$1.log 2>&1 || exit $?
    timeout -k 10 200 tools/kbench3 $1 128 5 libf32 $2 > gpurun_out/r03i/kb3_libf32_$1.log 2>&1 || exit $?
    (cd /tmp && timeout -k 10 -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r03i/pmc_i8_$1" -o run -- "$GRAFT_REPO_ROOT/tools/kbench3" $1 16 1 libi8 $2 \
        > "$GRAFT_REPO_ROOT/gpurun_out/r03i/pmc_i8_$1.log" 2>&1) || exit $?
done
echo done
