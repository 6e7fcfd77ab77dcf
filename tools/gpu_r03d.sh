# round 3, session d: banded-schedule A/B, then the GPU tests of the new
# native pieces (RCCL row-shard layer at world 1, round-trip sums flag,
# frame lists, C5 stream context)
mkdir -p gpurun_out/r03d
timeout -k 10 200 tools/kbench3 8192 64 3 band 16 > gpurun_out/r03d/kb3_band16.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench3 8192 64 3 bandi8 16 > gpurun_out/r03d/kb3_bandi8_16.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_roundtrip.py tests/test_gpu_frames.py \
    "tests/test_gpu_configs.py::test_c5_stream_batch_vs_oracle" "tests/test_gpu_configs.py::test_c5_stream_context_reused_across_batches" \
    -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03d/pytest_dist_rt.log 2>&1
echo "pytest rc=$?"
