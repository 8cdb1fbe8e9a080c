# r5k: the whole library under LLVM scheduler options (s0 default, s1 max-ilp strategy, s2 AMDGPU
# register-pressure trackers, s3 max-memory-clause scheduler, s4 = s1 + s2): fused backward and the
# step's epilogue GEMMs, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
FUSED_VARIANTS="5" bash tools/ab_libs.sh "s0 s1 s2 s3 s4" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5k_ab.txt
for v in s0 s1 s2 s3 s4; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py > gpurun_out/r5k_gemm_$v.log 2>&1 || exit 1
done
for f in gpurun_out/r5k_gemm_*.log; do echo "== $f"; grep "TF/s" $f; done | tee -a gpurun_out/r5k_ab.txt
