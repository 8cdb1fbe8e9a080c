# GEMM tile-order sweep (OWLK_GEMM_GROUP = tile rows per group; 0 = row-major)
set -e
cd "$GRAFT_REPO_ROOT"
for g in 2 4 8; do
  OWLK_GEMM_GROUP=$g timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or silu or gate or mlp" --timeout 120 --timeout-method thread > gpurun_out/gr_test_$g.log 2>&1
done
for i in 1 2; do
  for g in 0 2 4 8 16; do
    OWLK_GEMM_GROUP=$g timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gr_${g}_$i.log 2>&1
  done
done
