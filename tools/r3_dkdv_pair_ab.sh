# D=128 dK/dV variants (OWLK_DKDV128: 3 pipelined 32x32x16 one wave per SIMD; 4 / 7 wave pairs QT 1 / 2;
# 5 / 6 16x16x32 one wave per SIMD QT 2 / 1): parity at the test shapes, then an interleaved A/B at
# 20 heads x 98,304 tokens.   usage: bash tools/r3_dkdv_pair_ab.sh "4 5 6 7"
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
VARS=${1:-"4"}
for v in $VARS; do
  OWLK_DKDV128=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "(test_attention_fwd_bwd and 128) or (side_stream and 128)" > $O/pair_tests_$v.log 2>&1
done
for r in 1 2; do
  for v in 3 $VARS; do
    echo "== OWLK_DKDV128=$v round $r" >> $O/pair_ab.log
    OWLK_DKDV128=$v OWLK_BWD_SIDE_STREAM=0 timeout -k 10 300 python -u tools/attn_bench.py --heads 20 --dim 128 --iters 3 --bwd-only >> $O/pair_ab.log 2>&1
  done
done
