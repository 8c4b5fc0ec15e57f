#!/bin/bash
# SQ counters of the C2 pipeline for the product (recur_kernel, 16 series x 128-step chunks) and
# the measured-negative whole-row variant (rows_kernel, built from 7b06d88 with -DSTS_ROWS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in base rows; do
  L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
  STS_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    -d gpurun_out/c2sq_$V -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_$V.log 2>&1 || exit 1
done
