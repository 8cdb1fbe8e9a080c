# r6ab: the forward's 32x32x16 form (libowlk_w32) vs attn_fwd16_k on the check cases, then timing
# against the 16x16x32 form (base): fwd, global
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_w32.so timeout -k 10 120 python -u tools/fwd4_check.py > gpurun_out/r6ab_chk.log 2>&1
cat gpurun_out/r6ab_chk.log | grep -v amdgpu.ids
bash tools/ab_libs.sh "base w32" 2 --fwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fwd " $f | cut -c1-60; done | tee gpurun_out/r6ab_ab.txt
