#!/bin/bash
# Round-4 session 17: with XCD-contiguous spans, lanes per series (16 / 32 product / 64) and
# 2-wave workgroups once more on C2; the product's recurrence tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s17.log 2>&1
bash tools/ab_bench.sh c2 base l16 l64 w2 > gpurun_out/ab_c2_s17.jsonl
