# r6t: conflict-free ring / dS swizzles in the 8-wave kernel and the 16x16 forward's V image:
# full GPU suite, bitwise check (8-wave vs one-wave-per-SIMD), A/B against HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 200 python -u tools/fused4_check.py > gpurun_out/r6t_chk.log 2>&1 || exit 1
tail -1 gpurun_out/r6t_chk.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6t_gputests.log 2>&1 || { tail -30 gpurun_out/r6t_gputests.log; exit 1; }
tail -1 gpurun_out/r6t_gputests.log
cp owl-audio-exps_amd/owl_wms/_lib/libowlk.so owl-audio-exps_amd/owl_wms/_lib/libowlk_new.so
bash tools/ab_libs.sh "base new" 2 --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -hE "^  (fwd|fused) " $f | cut -c1-60; done | tee gpurun_out/r6t_ab.txt
