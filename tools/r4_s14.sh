#!/bin/bash
# Round-4 session 14: lanes per series in recur_row_kernel -- parity of the 32- and 64-lane forms
# and C2 A/B of 16 (product) / 32 / 64 lanes, two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
for V in lps32 lps64; do
  timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      -k "recur or ewma or fill_diff" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
done
bash tools/ab_bench.sh c2 base lps32 lps64 > gpurun_out/ab_c2_lps.jsonl
