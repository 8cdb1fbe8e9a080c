# Forward tile shapes: OWLK_FWD_KT128=1 (D 64: 128-key tiles on long sweeps) and OWLK_FWD_NQ3=1 (D 128: 48
# queries per wave).  Attention parity with both on, then interleaved A/Bs at the dit_v4 (24 x 64) and
# dit_v4_5B (20 x 128) shapes, 98,304 tokens, global and window 16
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_FWD_KT128=1 OWLK_FWD_NQ3=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "test_attention" > $O/fwdt_tests.log 2>&1
for r in 1 2; do
  for v in 0 1; do
    echo "== D64 OWLK_FWD_KT128=$v round $r" >> $O/fwdt_ab.log
    OWLK_FWD_KT128=$v timeout -k 10 300 python -u tools/attn_bench.py --iters 5 --fwd-only >> $O/fwdt_ab.log 2>&1
    echo "== D128 OWLK_FWD_NQ3=$v round $r" >> $O/fwdt_ab.log
    OWLK_FWD_NQ3=$v timeout -k 10 300 python -u tools/attn_bench.py --iters 3 --heads 20 --dim 128 --fwd-only >> $O/fwdt_ab.log 2>&1
  done
done
