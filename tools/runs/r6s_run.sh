# r6s: SQ counters (LDS bank conflicts, waits) of the forward (global, w16) and the 8-wave backward (w16)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for cfg in "fwd none" "fwd 16" "bwd 16"; do
  set -- $cfg
  W=$2; [ "$W" = none ] && W=
  WINDOW=$W FRAMES=1536 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_r6s_$1_$2 -f csv -o p1 -- python3 $R/tools/attn_fwd_only.py $1 > $R/gpurun_out/pmc_r6s_$1_$2.log 2>&1 || exit 1
done
