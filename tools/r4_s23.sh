#!/bin/bash
# Round-4 session 23: the row kernel's direct-access form on odd T (new test).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s23.log 2>&1
