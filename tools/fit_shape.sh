#!/bin/bash
# EWMA fit shape A/B (STS_EWMA_FIT_SHAPE) + GARCH fit at its new default shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_garch.py -m gpu > gpurun_out/fs_garch_tests.log 2>&1
timeout -k 10 300 env STS_EWMA_FIT_SHAPE=64x64 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/ -m gpu -k "ewma" > gpurun_out/fs_ewma_tests.log 2>&1
for sh in 32x64 64x64 32x64 64x64; do
  STS_EWMA_FIT_SHAPE=$sh timeout -k 10 200 python -u bench.py --workload ewma_fit --steps 5 --warmup 2 \
    --no-cpu-baseline > gpurun_out/ewma_s$sh.json 2> gpurun_out/ewma_s$sh.err
  echo "ewma shape=$sh $(python -c "import json; print(json.load(open('gpurun_out/ewma_s$sh.json'))['roofline']['avg_kernel_ms'])")"
done
timeout -k 10 300 python -u bench.py --workload garch_fit > gpurun_out/garch_final_bench.json 2> gpurun_out/garch_final_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_garch -o garch --output-format csv -- \
  python -u bench.py --workload garch_fit --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_garch.log 2>&1
