# A/B: attn_bwd_dkdv (32x32x16) vs OWLK_DKDV16=1 (16x16x32) -- parity tests, then interleaved timings
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
OWLK_DKDV16=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k "attention" > $O/ab16_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --iters 5 --bwd-only > $O/ab16_base$i.log 2>&1
  OWLK_DKDV16=1 timeout -k 10 200 python -u tools/attn_bench.py --iters 5 --bwd-only > $O/ab16_new$i.log 2>&1
done
