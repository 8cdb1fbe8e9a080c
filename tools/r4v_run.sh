# fused backward: dK / dV rows stored after the next item's prologue loads (pk2) against stored at the
# item's end (pk), both through the LDS staging; pa = 8-B lane pieces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_pk2.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1; rc=$?; echo "fused tests (pk2) rc=$rc"; tail -2 gpurun_out/r4v_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pk pk2" 2 --bwd-only --windows 16,4,none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done > gpurun_out/r4v_summary.txt
cat gpurun_out/r4v_summary.txt
bash tools/r4w_run.sh
