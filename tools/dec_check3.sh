set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -m gpu -x -k "decode or sampler or cache or eval or device_state" --timeout 120 --timeout-method thread > gpurun_out/dc_test.log 2>&1
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dc_bench.log 2>&1
timeout -k 10 300 python -u tools/decode_bench.py --frames 8 > gpurun_out/dc_bench8.log 2>&1
