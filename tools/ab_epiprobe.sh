set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 200 python tools/epi_probe.py > gpurun_out/ep_base.log 2>&1
OWLK_LIB=$L/libowlk_noepi.so timeout -k 10 200 python tools/epi_probe.py > gpurun_out/ep_noepi.log 2>&1
