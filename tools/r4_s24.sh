#!/bin/bash
# Round-4 session 24: non-temporal 16-B stores for the C2 row kernel's span output (var_ntc2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "fill_diff or row_scan" --sts-lib spark-timeseries_amd/build/var_ntc2/libsts_hip.so > gpurun_out/pytest_ntc2.log 2>&1
bash tools/ab_bench.sh c2 base ntc2 > gpurun_out/ab_c2_nt.jsonl
bash tools/ab_bench.sh c2 base ntc2 >> gpurun_out/ab_c2_nt.jsonl
