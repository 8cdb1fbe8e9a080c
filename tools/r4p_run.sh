# fused backward: flag poll before the ring DMA (pb) against after it (pa), global and window 16
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_pb.so timeout -k 10 500 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1; rc=$?; echo "fused tests (pb) rc=$rc"; tail -2 gpurun_out/r4p_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pb" 3 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "window=\|fused" $f; done
