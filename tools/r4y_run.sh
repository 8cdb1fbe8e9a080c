# PMC summary of the final single-pass backward at the dit_v4 global shape (MFMA busy, LDS, waits)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/r4z_run.sh || exit 1
rm -rf gpurun_out/pmc_bwd
FRAMES=1536 WHICH=bwd PROG=attn_fwd_only.py bash tools/pmc_attn.sh || exit 1
python3 tools/pmc_csv.py gpurun_out/pmc_bwd > gpurun_out/r4y_pmc_summary.txt 2>&1; cat gpurun_out/r4y_pmc_summary.txt
