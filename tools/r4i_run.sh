# round-4 check of the pipelined fused backward: its tests, A/B against m2, then the round check
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4i_tests_fused.log 2>&1; rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/r4i_tests_fused.log
[ $rc -eq 0 ] || exit 1
cp $L/libowlk.so $L/libowlk_main.so
rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "main m2" 2 --bwd-only --windows none --iters 3 || exit 1
rm -f $L/libowlk_main.so
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused\|dkdv\|dq " $f; done
bash tools/round_check.sh r4i || exit 1
tail -3 gpurun_out/r4i_gputests.log; tail -2 gpurun_out/r4i_smoke.log; tail -1 gpurun_out/r4i_bench.log | cut -c1-400
