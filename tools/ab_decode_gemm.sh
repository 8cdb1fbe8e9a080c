# decode GEMM plan A/B (OWLK_GEMM_DECODE 0 = split-K partials + reduce kernel, 1 = one launch) + tests
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "skinny or gemm" --timeout 120 --timeout-method thread > gpurun_out/dg_test.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -m gpu -x -k "decode or sampler or cache" --timeout 120 --timeout-method thread > gpurun_out/dg_test_model.log 2>&1
for i in 1 2; do
  OWLK_GEMM_DECODE=0 timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dg_old_$i.log 2>&1
  timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dg_new_$i.log 2>&1
done
OWLK_GEMM_DECODE=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dg_decode_old.log 2>&1
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dg_decode_new.log 2>&1
