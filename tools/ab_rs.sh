set -e
cd "$GRAFT_REPO_ROOT"
OWLK_FWD_RS=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/rs_test.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/attn_bench.py --iters 5 > gpurun_out/rs_base_$i.log 2>&1
  OWLK_FWD_RS=1 timeout -k 10 200 python tools/attn_bench.py --iters 5 > gpurun_out/rs_new_$i.log 2>&1
done
