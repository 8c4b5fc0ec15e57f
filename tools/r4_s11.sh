#!/bin/bash
# Round-4 session 11: recur_row_kernel with 16 lanes per series (4 series per wave, lane blocks of
# B = 26 steps for C2), rows through a per-wave LDS span (IO) or direct (noio) -- recurrence parity, then C2 A/B against the chunk kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "recur or ewma or fill_diff" > gpurun_out/pytest_rowscan3.log 2>&1
bash tools/ab_bench.sh c2 base noio chunk > gpurun_out/ab_c2_rowscan3.jsonl
