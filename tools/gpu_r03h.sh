# round 3, session h: PMC traffic of every kernel the bench times (the drop-in
# surface included; tools/pmc_traffic.sh) and a frame-size sweep of the two
# library forward kernels (is the int8 kernel's gap to its math time a fixed
# per-launch cost?)
mkdir -p gpurun_out/r03h
for spec in "4096 64" "8192 16" "8192x16384 8" "16384 4"; do
    set -- $spec
    timeout -k 10 200 tools/kbench3 $1 64 3 libi8 $2 > gpurun_out/r03h/kb3_libi8_$1.log 2>&1 || exit $?
    timeout -k 10 200 tools/kbench3 $1 64 3 libf32 $2 > gpurun_out/r03h/kb3_libf32_$1.log 2>&1 || exit $?
done
bash tools/pmc_traffic.sh > gpurun_out/r03h/pmc_traffic.log 2>&1 || exit $?
echo done
