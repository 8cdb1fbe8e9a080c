# final round-4 tree: no-regression A/B of the packed-documents build, mmdit_v2 and dit_v4_5B benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# the packed-documents build (pb = HEAD) against the one before it (pa) on the document-free shapes
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pb" 2 --bwd-only --windows 16,none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done > gpurun_out/r4fin2_ab.txt; cat gpurun_out/r4fin2_ab.txt
timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --no-traffic --no-cpu-baseline > gpurun_out/r4fin_mmdit.log 2>&1 || exit 1
tail -1 gpurun_out/r4fin_mmdit.log | cut -c1-200
timeout -k 10 600 python -u bench.py --config configs/dit_v4_5B.yml --no-traffic --no-cpu-baseline > gpurun_out/r4fin_5b.log 2>&1 || exit 1
tail -1 gpurun_out/r4fin_5b.log | cut -c1-200
