#!/bin/bash
# Round-4 session 13: recur_row_kernel with 32 lanes per series (2 series per wave, B = 14 for C2,
# 5 workgroups per CU) -- its recurrence parity, C2 A/B against the 16-lane product, and the SQ
# counters of the product's C2 kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "recur or ewma or fill_diff" --sts-lib spark-timeseries_amd/build/var_lps32/libsts_hip.so > gpurun_out/pytest_lps32.log 2>&1
bash tools/ab_bench.sh c2 base lps32 > gpurun_out/ab_c2_lps32.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    -d gpurun_out/c2sq_row -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_row.log 2>&1
