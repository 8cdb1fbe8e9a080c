# fused backward: dQ read pipeline depth 1 / 2 (default) / 3 on the final code; fused tests for 1 and 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in q1 q3; do
OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread -k "oracle" > gpurun_out/r4ag_tests_$v.log 2>&1; rc=$?; echo "fused tests ($v) rc=$rc"; tail -1 gpurun_out/r4ag_tests_$v.log
[ $rc -eq 0 ] || exit 1
done
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "q1 q2 q3" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done > gpurun_out/r4ag_summary.txt; cat gpurun_out/r4ag_summary.txt
