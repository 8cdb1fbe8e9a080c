# r6w: ring DMA / poll / check placement variants of the one-wave-per-SIMD step: bitwise check, A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in L1 L3 L4; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/fused4_check.py > gpurun_out/r6w_chk_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r6w_chk_$v.log)"
done
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base L1 L2 L3 L4" 2 --bwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6w_ab.txt
