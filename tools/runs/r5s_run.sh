# r5s: scheduler options for the attention forward / two-kernel backward files (f0 production;
# f1 trackers, f2 max-ilp, f3 max-memory-clause, f4 no memop clustering, f5 no unclustered high-RP
# reschedule, each on every file): D = 128 (dit_v4_5B) forward + dK/dV + dQ, D = 64 forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "f0 f1 f2 f3 f4 f5" 2 --dim 128 --heads 20 --windows none --iters 2 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd \|dkdv\|  dq " $f | cut -c1-40; done | tee gpurun_out/r5s_ab.txt
rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "f0 f1 f2 f3 f4 f5" 2 --fwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd " $f | cut -c1-40; done | tee -a gpurun_out/r5s_ab.txt
