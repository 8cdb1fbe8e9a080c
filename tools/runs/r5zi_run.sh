# r5zi: single-pass backward chain grouping per XCD queue (OWLK_BWD_FUSED_GROUP: chains swept at a time,
# 0 = all) on the window-16 and window-4 layers, interleaved x3 (production: 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do for g in 1 2 3 0; do
  echo "== group $g $i"; OWLK_BWD_FUSED_GROUP=$g timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows 16,4 --iters 5 2>&1 | grep "fused" | cut -c1-40 || exit 1
done; done | tee gpurun_out/r5zi_ab.txt
