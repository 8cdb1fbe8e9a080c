# r6al: CU reserve for the all-reduce micro-step: parity of the reduced grid, then the co-residency probe
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RESERVE=8,16,24,32,48 timeout -k 10 300 python -u tools/coresidency.py > gpurun_out/r6al_coresidency2.log 2>&1
