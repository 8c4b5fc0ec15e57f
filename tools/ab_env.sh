#!/bin/bash
# Env-knob A/B in one session: parity of the knob setting, then interleaved kbench rounds.
# Usage: AB_VAR=STS_TILE_W AB_VALUES="4096 2048" AB_CASES=tile:linear:60 tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_env_$v.log 2>&1
  rc=$?; echo "parity $AB_VAR=$v rc=$rc $(tail -1 gpurun_out/parity_env_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 300 python -u tools/kbench.py --series ${AB_SERIES:-2000} --cases "${AB_CASES:-tile:linear:60}" 2>/dev/null |
    sed "s/^{/{\"$AB_VAR\": \"$v\", \"round\": $r, /" | tee -a gpurun_out/ab_env.jsonl || exit 1
done; done
