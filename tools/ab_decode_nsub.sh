set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "skinny" --timeout 120 --timeout-method thread > gpurun_out/dn_test.log 2>&1
for n in 0 1 2 3 6; do
  OWLK_DECODE_NSUB=$n timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dn_$n.log 2>&1
done
OWLK_GEMM_DECODE=0 timeout -k 10 120 python tools/decode_gemm_bench.py > gpurun_out/dn_old.log 2>&1
