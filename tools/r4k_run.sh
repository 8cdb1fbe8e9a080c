# fused backward: tests (all variants), phase profile, PMC summary at the dit_v4 shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1; rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/r4k_tests.log
[ $rc -eq 0 ] || exit 1
OWLK_LIB=$L/libowlk_pf.so FUSED_VARIANTS="5" timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 2 > gpurun_out/r4k_prof.log 2>&1 || exit 1
grep "fused" gpurun_out/r4k_prof.log
rm -rf gpurun_out/pmc_bwd
FRAMES=1536 WHICH=bwd PROG=attn_fwd_only.py bash tools/pmc_attn.sh || exit 1
python3 tools/pmc_csv.py gpurun_out/pmc_bwd > gpurun_out/r4k_pmc_summary.txt 2>&1; cat gpurun_out/r4k_pmc_summary.txt
