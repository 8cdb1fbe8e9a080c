# r6ae: exact tests of the ping-pong GEMM's paired-rounding epilogues
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f owl-audio-exps_amd/owl_wms/_lib/libowlk_*.so
timeout -k 10 300 python -u -m pytest tests/test_gemm_epi_exact_gpu.py tests/test_kernels_gpu.py -k "gemm or epi" -x -v --timeout 120 --timeout-method thread > gpurun_out/r6ae_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r6ae_tests.log; exit $rc
