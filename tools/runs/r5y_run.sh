# r5y: PMC of the production single-pass backward and forward (dit_v4 global layer, 512 frames):
# tools/pmc_attn.sh passes, summarised by tools/pmc_csv.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
WHICH=bwd bash tools/pmc_attn.sh || exit 1
WHICH=fwd bash tools/pmc_attn.sh || exit 1
{ python tools/pmc_csv.py gpurun_out/pmc_bwd; python tools/pmc_csv.py gpurun_out/pmc_fwd; } | tee gpurun_out/r5y_pmc_summary.txt
