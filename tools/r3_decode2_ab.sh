# Decode GEMM: weight-stream-only gemm_decode2_k (OWLK_DECODE2=1, default) vs gemm_decode_k (0).
# GEMM + decode / sampler parity with the new kernel, then decode wall time per frame (dit_v4, dit_v4_5B)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "gemm or decode or sampler or kv_cache or graphed" > $O/dec2_tests.log 2>&1
for v in 0 1; do
  echo "== OWLK_DECODE2=$v" >> $O/dec2_ab.log
  OWLK_DECODE2=$v timeout -k 10 300 python -u tools/decode_gemm_bench.py >> $O/dec2_ab.log 2>&1
  OWLK_DECODE2=$v timeout -k 10 300 python -u tools/decode_bench.py >> $O/dec2_ab.log 2>&1
  OWLK_DECODE2=$v timeout -k 10 300 python -u tools/decode_bench.py --config configs/dit_v4_5B.yml >> $O/dec2_ab.log 2>&1
done
