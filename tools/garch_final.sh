#!/bin/bash
# GARCH fit at the defaults: parity tests, the bench line, rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_garch.py -m gpu > gpurun_out/garch_final_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload garch_fit > gpurun_out/garch_final_bench.json 2> gpurun_out/garch_final_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_garch -o garch --output-format csv -- \
  python -u bench.py --workload garch_fit --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_garch.log 2>&1
