# r5f: early flag poll (p1), helper-loaded sums in flight over the barrier (h2), dQ products split over key halves with the helper (s1), against ring DMA by waves 4-7 only (d1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in p1 h2 s1; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -x -q \
    -k "oracle or counts or deterministic or timeout" --timeout 200 --timeout-method thread \
    > gpurun_out/r5f_tests_$v.log 2>&1 || { tail -30 gpurun_out/r5f_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r5f_tests_$v.log
done
FUSED_VARIANTS="5" bash tools/ab_libs.sh "d1 p1 h2 s1" 2 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5f_ab.txt
timeout -k 10 200 python -u tools/coresidency.py > gpurun_out/r5f_coresid.log 2>&1 || exit 1
cat gpurun_out/r5f_coresid.log
