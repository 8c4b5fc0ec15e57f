#!/bin/bash
# Round-5 session 21: C5 with plain instead of non-temporal filled-output stores in the fill-only
# tile kernel (var_c5plain): parity of the fill / lag rows, then three alternating C5 rounds after one warm-up process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py tests/test_c5_length.py \
    -k "fill or lag or c5" --sts-lib spark-timeseries_amd/build/var_c5plain/libsts_hip.so > $O/c5plain_parity.log 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
bash tools/ab_bench.sh c5 base c5plain > $O/ab_c5plain.jsonl
bash tools/ab_bench.sh c5 c5plain base >> $O/ab_c5plain.jsonl
