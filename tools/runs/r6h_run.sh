# r6h: parity-specialised statements, ring DMA and flag poll inside: bitwise check, timing, phase profile
# statement: bitwise check against the 8-wave kernel, timing, phase profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/fused4_check.py --time > gpurun_out/r6h_check.log 2>&1 || exit 1
OWLK_LIB=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prof.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 > gpurun_out/r6h_prof.log 2>&1
