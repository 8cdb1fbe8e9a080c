set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "skinny" --timeout 120 --timeout-method thread > gpurun_out/dg_test.log 2>&1
OWLK_GEMM_DECODE=0 timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dg_old_1.log 2>&1
timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dg_new_1.log 2>&1
