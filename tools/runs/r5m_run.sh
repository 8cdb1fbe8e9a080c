# r5m: scheduler options on top of the production flags (t0): t1 no unclustered high-RP reschedule,
# t2 no clustered low-occupancy reschedule, t3 no memop clustering, t4 + post-RA machine scheduler;
# attention fwd / fused bwd (global, window 16) and the epilogue GEMMs, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
FUSED_VARIANTS="5" bash tools/ab_libs.sh "t0 t1 t2 t3 t4" 2 --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused\|  fwd " $f | cut -c1-40; done | tee gpurun_out/r5m_ab.txt
for v in t0 t1 t2 t3 t4; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py > gpurun_out/r5m_gemm_$v.log 2>&1 || exit 1
done
for f in gpurun_out/r5m_gemm_*.log; do echo "== $f"; grep "TF/s" $f; done | tee -a gpurun_out/r5m_ab.txt
