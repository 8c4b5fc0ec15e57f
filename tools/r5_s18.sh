#!/bin/bash
# Round-5 session 18: RCCL collectives on one GPU (tests/test_rccl_gpu.py); non-temporal prefetch loads in the
# tile kernel (var_ntl): parity, C3 kernel A/B, C5 bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rccl_gpu.py > $O/rccl.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py -k "tile or fill_acf or c5 or lag" --sts-lib spark-timeseries_amd/build/var_ntl/libsts_hip.so > $O/ntl_parity.log 2>&1
RS_PARITY=0 RS_ARMS="base ntl" bash tools/r5_rs.sh
bash tools/ab_bench.sh c5 base ntl > $O/ab_c5_ntl.jsonl
