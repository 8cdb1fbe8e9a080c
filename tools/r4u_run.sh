# fused backward: dK / dV stored as whole rows through LDS (pk) against 8-B lane pieces (pa)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_pk.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1; rc=$?; echo "fused tests (pk) rc=$rc"; tail -2 gpurun_out/r4u_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pk" 3 --bwd-only --windows 16,4,none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done
