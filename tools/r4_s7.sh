#!/bin/bash
# Round-4 session 7: the AR(p) Gram's lag products on FP64 MFMA inside the C4 register kernel
# (STS_AR_MFMA variant) -- AR parity, C4 A/B, FP64 / MFMA counters of the variant; s_setprio
# around the C3 MFMA phase (var_prio_m) or the fill phase (var_prio_f) -- C3 kernel A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "ar_ or arima" --sts-lib spark-timeseries_amd/build/var_ar_mfma/libsts_hip.so > gpurun_out/pytest_ar_mfma.log 2>&1
bash tools/ab_bench.sh c4 base ar_mfma > gpurun_out/ab_c4_ar_mfma.jsonl
STS_HIP_LIB=spark-timeseries_amd/build/var_ar_mfma/libsts_hip.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_c4_ar_mfma -o bench --output-format csv -- python -u bench.py --workload c4 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c4_ar_mfma.log 2>&1
for rep in 1 2; do
  for V in base prio_m prio_f; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio.jsonl
  done
done
