# r5j: single pass with the next item's prologue loads issued in the current item's epilogue (p1)
# against the same source without (p0) and the committed library (x0): parity of p1, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_p1.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5j_tests_p1.log 2>&1 || { tail -30 gpurun_out/r5j_tests_p1.log; exit 1; }
tail -2 gpurun_out/r5j_tests_p1.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "x0 p0 p1" 2 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5j_ab.txt
