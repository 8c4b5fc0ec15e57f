#!/bin/bash
# Round-4 session 18: wave priorities in the C4 AR kernel (remove + store phase at 2) and the C1
# short kernel (stores, or fill + stores, at 2; the ACF at 0) -- parity, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "ar_" --sts-lib spark-timeseries_amd/build/var_ar_prio/libsts_hip.so > gpurun_out/pytest_ar_prio.log 2>&1
for V in sh_prio_st sh_prio_fill; do
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
done
bash tools/ab_bench.sh c4 base ar_prio > gpurun_out/ab_c4_prio.jsonl
bash tools/ab_bench.sh c1 base sh_prio_st sh_prio_fill > gpurun_out/ab_c1_prio.jsonl
