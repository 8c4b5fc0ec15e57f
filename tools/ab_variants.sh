#!/bin/bash
# Parity (tile/seg parity + golden tests) of each variant library, then tools/ab.sh over them.
# Usage: AB_CASES=... tools/ab_variants.sh var1 var2 ...   (variant dirs from tools/variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in "$@"; do
  lib=spark-timeseries_amd/build/var_$v/libsts_hip.so
  [ -f "$lib" ] || { echo "variant $v: $lib missing" >&2; exit 2; }
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --sts-lib "$lib" > gpurun_out/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/parity_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab.sh "${AB_CASES:-tile:linear:60}" main "$@" > gpurun_out/ab_variants.jsonl; rc=$?
cat gpurun_out/ab_variants.jsonl; exit $rc
