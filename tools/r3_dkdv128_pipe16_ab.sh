# D=128 dK/dV: attn_bwd_dkdv16_k at one wave per SIMD with software-pipelined FULL tiles (OWLK_DKDV128=5:
# QT 2, 6: QT 1) vs the pipelined 32x32x16 attn_bwd_dkdv_k (3).  Attention parity with 5, then an
# interleaved A/B at 20 heads x 98,304 tokens (global; dK/dV alone and beside dQ on a side stream)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_DKDV128=5 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "test_attention" > $O/p16_tests.log 2>&1
for r in 1 2; do
  for v in 3 5 6; do
    echo "== OWLK_DKDV128=$v round $r" >> $O/p16_ab.log
    OWLK_DKDV128=$v timeout -k 10 300 python -u tools/attn_bench.py --heads 20 --dim 128 --iters 3 --bwd-only --windows none >> $O/p16_ab.log 2>&1
  done
done
