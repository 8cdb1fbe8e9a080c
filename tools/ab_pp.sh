# GEMM ping-pong vs previous 256^2 kernel: parity tests, then interleaved timing rounds.
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/pp_gemmtest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/pp_new$i.log 2>&1
  OWLK_GEMM_PP=0 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/pp_old$i.log 2>&1
done
