# D=128 16x16x32 forward / dQ A/B at the dit_v4_5B attention shape (20 heads x 98,304 tokens)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for r in 1 2; do
  for v in 0 1; do
    echo "== OWLK_FWD16_128=$v OWLK_DQ16_128=$v round $r"
    OWLK_FWD16_128=$v OWLK_DQ16_128=$v timeout -k 10 300 python -u tools/attn_bench.py --heads 20 --dim 128 --iters 3
  done
done
