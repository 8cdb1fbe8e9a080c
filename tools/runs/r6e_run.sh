# r6e: one-wave-per-SIMD single pass: dQ read pipeline 3 vs 7 k-steps (phase profiles + timing)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in prof3 prof7; do
OWLK_LIB=$L/libowlk_$v.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 > gpurun_out/r6e_$v.log 2>&1 || exit 1
done
FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 3 > gpurun_out/r6e_pf3.log 2>&1 || exit 1
OWLK_LIB=$L/libowlk_pf7.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 3 > gpurun_out/r6e_pf7.log 2>&1
