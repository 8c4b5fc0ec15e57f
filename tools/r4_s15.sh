#!/bin/bash
# Round-4 session 15: recur_row_kernel launch shape on C2 -- 1 / 2 / 4 (product) waves per
# workgroup, XCD-contiguous span ranges; parity of the 1-wave form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "fill_diff or ewma or row_scan" --sts-lib spark-timeseries_amd/build/var_wpg1/libsts_hip.so > gpurun_out/pytest_wpg1.log 2>&1
bash tools/ab_bench.sh c2 base wpg1 wpg2 xcd > gpurun_out/ab_c2_shape.jsonl
