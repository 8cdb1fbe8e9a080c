# r6ap: out-projection qkv projection + QK-norm/RoPE in one GEMM epilogue: parity, model tests, GEMM timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_epi_exact_gpu.py > gpurun_out/r6ap_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/qk_rope_gemm_bench.py > gpurun_out/r6ap_micro.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/r6ap_model_tests.log 2>&1
