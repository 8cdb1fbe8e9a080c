# fused backward: which rematerialised lane values pay (p1d / p2d / p4d / p8d, OWLK_FUSED_REMAT bits, all with
# the next item claimed in the epilogue) against HEAD (pa), the restructured source with none (p0), + the claim (p0d)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa p0 p0d p1d p2d p4d p8d" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done
