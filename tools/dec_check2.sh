set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "decode_split or attention_fwd" --timeout 120 --timeout-method thread > gpurun_out/dc_ktest.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -m gpu -x -k "decode or sampler or cache or eval" --timeout 120 --timeout-method thread > gpurun_out/dc_test.log 2>&1
OWLK_FWD_SPLIT=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dc_bench_nosplit.log 2>&1
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dc_bench.log 2>&1
