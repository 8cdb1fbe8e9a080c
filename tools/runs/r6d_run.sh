# r6d: one-wave-per-SIMD single pass, phase profile of variant 129 alone (timing-only build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OWLK_LIB=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prof.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 > gpurun_out/r6d_prof.log 2>&1
