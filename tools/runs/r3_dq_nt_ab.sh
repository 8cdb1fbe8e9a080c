# dQ queries per wave: OWLK_DQ_NT=3 (48, 192 per workgroup) vs 2 (32): attention parity with NT 3, then
# an interleaved A/B at the dit_v4 shape (24 heads x 98,304 tokens, global and window 16)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_DQ_NT=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "test_attention" > $O/dqnt_tests.log 2>&1
for r in 1 2; do
  for v in 2 3; do
    echo "== OWLK_DQ_NT=$v round $r" >> $O/dqnt_ab.log
    OWLK_DQ_NT=$v timeout -k 10 300 python -u tools/attn_bench.py --iters 5 --bwd-only >> $O/dqnt_ab.log 2>&1
  done
done
