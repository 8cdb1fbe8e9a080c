# r5h: (1) GEMM epilogues in paired-rounding form (g1), + straight from registers (g2) against the
# previous form (g0): bit-exact
# outputs, then interleaved timing; (2) EMPTY tiles without a branch around the dK / dV accumulators
# (e1: masked path, e2: S / dP skipped, dV / dK MFMAs on zeros) against production (e0): parity,
# then interleaved A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in g0 g1 g2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py --save gpurun_out/r5h_epi_$v.pt \
    > gpurun_out/r5h_gemm_${v}_1.log 2>&1 || { tail -20 gpurun_out/r5h_gemm_${v}_1.log; exit 1; }
done
python tools/gemm_epi_bench.py --compare gpurun_out/r5h_epi_g0.pt gpurun_out/r5h_epi_g1.pt | tee gpurun_out/r5h_epi_compare.txt
python tools/gemm_epi_bench.py --compare gpurun_out/r5h_epi_g0.pt gpurun_out/r5h_epi_g2.pt | tee -a gpurun_out/r5h_epi_compare.txt
for v in g0 g1 g2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py > gpurun_out/r5h_gemm_${v}_2.log 2>&1 || exit 1
done
for f in gpurun_out/r5h_gemm_g*_[12].log; do echo "== $f"; grep "TF/s" $f; done | tee gpurun_out/r5h_gemm_ab.txt
OWLK_LIB=$L/libowlk_e2.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5h_tests_e2.log 2>&1 || { tail -30 gpurun_out/r5h_tests_e2.log; exit 1; }
tail -2 gpurun_out/r5h_tests_e2.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "e0 e1 e2" 2 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5h_ab.txt
