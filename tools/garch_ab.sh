#!/bin/bash
# GARCH fit: parity tests (all pass-budget modes), then the garch_fit bench at several
# pass budgets (STS_GARCH_PASS_BUDGET; 0 = no tail kernel).  Every GPU step has its own
# time limit and a failing step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_garch.py -m gpu > gpurun_out/garch_tests.log 2>&1
for b in ${BUDGETS:-256 64 1024 0}; do
  echo "=== budget $b $(date +%T)"
  STS_GARCH_PASS_BUDGET=$b timeout -k 10 200 python -u bench.py --workload garch_fit --steps 1 --warmup 1 \
    --no-cpu-baseline > gpurun_out/garch_b$b.json 2> gpurun_out/garch_b$b.err
  tail -c 400 gpurun_out/garch_b$b.json
done
