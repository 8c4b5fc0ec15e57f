STEPS=ab AB_CASES="tile:linear:60" AB_LIBS="base diag1 diag3w2 diag4w2" bash tools/gpu_all.sh || exit 1
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
G3="GRBM_GUI_ACTIVE GRBM_COUNT"
for L in base diag3w2; do
  if [ $L = base ]; then P=spark-timeseries_amd/build/libsts_hip.so; else P=spark-timeseries_amd/build/var_$L/libsts_hip.so; fi
  STS_HIP_LIB=$P PROF_SERIES=1000 bash tools/pmc_kbench.sh "tile:linear:60" "$G1" "$G2" "$G3" || exit 1
  mkdir -p gpurun_out/sq_$L && mv gpurun_out/pmck_* gpurun_out/sq_$L/
done
