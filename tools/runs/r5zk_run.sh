# r5zk: where the single pass's time goes -- timing-only builds (results WRONG): e1 no hand-off (no
# flag polls, no sum loads / stores), e3 also no dQ products, e7 also no dS image writes; e0 production.
# Global and window-16 layers, interleaved x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "e0 e1 e3 e7" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5zk_ab.txt
rm -f gpurun_out/libs_*.log
