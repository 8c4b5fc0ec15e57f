#!/bin/bash
# Round-4 session 6: early raw stores from the prefetch registers (STS_EARLY_ST) -- parity, C3
# kernel A/B (fill + ACF, fill only), C5 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    --sts-lib spark-timeseries_amd/build/var_est/libsts_hip.so > gpurun_out/pytest_est.log 2>&1
for rep in 1 2; do
  for V in base est; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60,tile:linear:0 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_est.jsonl
  done
done
bash tools/ab_bench.sh c5 base est > gpurun_out/ab_c5_est.jsonl
