# fused backward on windowed layers: chains taken at a time per XCD queue (variant bits 2-5: 1, 2, 4, all)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
FUSED_VARIANTS="5,9,17,1" timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows 16,4 --iters 3 > gpurun_out/r4ae_$i.log 2>&1 || exit 1
grep "window=\|fused" gpurun_out/r4ae_$i.log | cut -c1-150
done
