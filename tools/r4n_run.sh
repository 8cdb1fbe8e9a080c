# fused dQ form A/B: 16x16x32 on all 8 waves (d16) vs 32x32x16 on waves 0-3 (d32), global and window 16
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_d16.so timeout -k 10 500 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1; rc=$?; echo "fused tests (d16) rc=$rc"; tail -2 gpurun_out/r4n_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "d32 d16" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "window=\|fused" $f; done
OWLK_LIB=$L/libowlk_d16pf.so FUSED_VARIANTS="5" timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 2 > gpurun_out/r4n_prof.log 2>&1 || exit 1
grep "fused" gpurun_out/r4n_prof.log
