# A/B: attention kernels on 32x32x16 MFMAs (default) vs the 16x16x32 variants (OWLK_FWD16,
# OWLK_DKDV16, OWLK_DQ16) -- parity tests with the variants on, then interleaved timings
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
export_all="OWLK_FWD16=1 OWLK_DKDV16=1 OWLK_DQ16=1"
env $export_all timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k "attention or gamerft or mmdit or packed or kv_cache or sampler" > $O/ab16_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --iters 5 > $O/ab16_base$i.log 2>&1
  env $export_all timeout -k 10 200 python -u tools/attn_bench.py --iters 5 > $O/ab16_new$i.log 2>&1
done
