mkdir -p gpurun_out
STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_stamps.so timeout -k 10 120 python -u tools/stamps.py 2000 60 0 > gpurun_out/stamps_v7.json 2>gpurun_out/stamps.err || exit 1
PROF_SERIES=1000 bash tools/pmc_kbench.sh "tile:linear:60,tile:linear:0" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM"
