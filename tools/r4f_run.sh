set -o pipefail
cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
VARS=${VARS:-"q16s q32s q32n"}
for x in q32t q16t q32l; do [ -f $L/libowlk_$x.so ] && VARS="$VARS $x"; done
for v in $VARS; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4f_tests_$v.log 2>&1; rc=$?; echo "tests $v rc=$rc"; tail -2 gpurun_out/r4f_tests_$v.log
  [ $rc -eq 0 ] || exit 1
done
bash tools/ab_libs.sh "$VARS" 2 --bwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused\|split\|dkdv\|dq " $f; done
if [ -f $L/libowlk_q32st.so ]; then
  OWLK_LIB=$L/libowlk_q32st.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 2 > gpurun_out/r4f_stats.log 2>&1 || exit 1
  grep "fused" gpurun_out/r4f_stats.log
fi
if [ -f $L/libowlk_q32pf.so ]; then
  OWLK_LIB=$L/libowlk_q32pf.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 2 > gpurun_out/r4f_prof.log 2>&1 || exit 1
  grep "fused" gpurun_out/r4f_prof.log
fi
