# split-K weight gradients: XCD-aware remap over the whole (tile, split) grid (OWLK_GEMM_SPLIT_REMAP=1) vs
# the per-tile remap (0).  GEMM parity with 1, then an interleaved A/B of the dit_v4 dW shapes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_GEMM_SPLIT_REMAP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "gemm" > $O/remap_tests.log 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    echo "== OWLK_GEMM_SPLIT_REMAP=$v round $r" >> $O/remap_ab.log
    OWLK_GEMM_SPLIT_REMAP=$v timeout -k 10 300 python -u tools/gemm_bench.py --wgrad-only >> $O/remap_ab.log 2>&1
  done
done
