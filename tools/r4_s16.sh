#!/bin/bash
# Round-4 session 16: XCD-contiguous workgroup ranges -- the row kernel's product (remap on) on
# the recurrence tests and against noxcd on C2; the same remap as variants of the C1 short kernel
# and the C4 AR kernel (parity, then A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_xcd_recur.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_short_xcd/libsts_hip.so > gpurun_out/pytest_short_xcd.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "ar_" --sts-lib spark-timeseries_amd/build/var_ar_xcd/libsts_hip.so > gpurun_out/pytest_ar_xcd.log 2>&1
bash tools/ab_bench.sh c2 base noxcd > gpurun_out/ab_c2_xcd.jsonl
bash tools/ab_bench.sh c1 base short_xcd > gpurun_out/ab_c1_xcd.jsonl
bash tools/ab_bench.sh c4 base ar_xcd > gpurun_out/ab_c4_xcd.jsonl
