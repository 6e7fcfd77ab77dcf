mkdir -p gpurun_out/r03d
timeout -k 10 200 tools/kbench3 8192 64 3 band 16 > gpurun_out/r03d/kb3_band16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 bandi8 16 > gpurun_out/r03d/kb3_bandi8_16.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_roundtrip.py tests/test_gpu_frames.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d/pytest_dist_rt.log 2>&1
echo "pytest rc=$?"
