# D=64 backward tile height for long windowed sweeps: QT 2 (128-row tiles) from OWLK_BWD_QT2_MIN tokens of
# window (default 4096) vs QT 1 for every window (old rule).  Parity with QT 2 forced on every windowed
# case, then an interleaved A/B at mmdit_v2's shape (24 heads x 1000 frames x 65 tokens)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_BWD_QT2_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "test_attention" > $O/qt2_tests.log 2>&1
for r in 1 2; do
  for v in 1000000000 4096; do
    echo "== OWLK_BWD_QT2_MIN=$v round $r" >> $O/qt2_ab.log
    OWLK_BWD_QT2_MIN=$v timeout -k 10 300 python -u tools/attn_bench.py --tpf 65 --frames 1000 --windows 16,32,64,256 --iters 5 --bwd-only >> $O/qt2_ab.log 2>&1
  done
done
