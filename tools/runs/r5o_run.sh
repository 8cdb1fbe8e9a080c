# r5o: forward attention under the default (v0) and the production scheduler flags (v1); then our
# GEMMs beside torch.matmul (hipBLASLt) at the dit_v4 plain-store shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
bash tools/ab_libs.sh "v0 v1" 3 --fwd-only --windows none,16 --iters 5 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd " $f | cut -c1-40; done | tee gpurun_out/r5o_ab.txt
timeout -k 10 400 python -u tools/gemm_bench.py > gpurun_out/r5o_blaslt.log 2>&1 || exit 1
cat gpurun_out/r5o_blaslt.log | tee -a gpurun_out/r5o_ab.txt
