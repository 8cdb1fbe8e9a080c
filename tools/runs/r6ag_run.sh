# r6ag: SQ counters of the production one-wave-per-SIMD kernels (global backward, global forward)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for which in bwd fwd; do
for i in 1 2 3; do
  case $i in
    1) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS";;
    2) C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC";;
    3) C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F SQ_ACTIVE_INST_VMEM SQ_CYCLES GRBM_GUI_ACTIVE";;
  esac
  FRAMES=1536 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_r6ag_$which -f csv -o p$i -- python3 $R/tools/attn_fwd_only.py $which > $R/gpurun_out/pmc_r6ag_${which}_$i.log 2>&1 || exit 1
done
python3 $R/tools/pmc_csv.py $R/gpurun_out/pmc_r6ag_$which > $R/gpurun_out/r6ag_${which}_pmc.txt
done
cat $R/gpurun_out/r6ag_*_pmc.txt
