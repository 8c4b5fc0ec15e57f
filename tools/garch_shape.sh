#!/bin/bash
# A/B of garch_fit_kernel's shape (STS_GARCH_SHAPE: series per wave x chunk) on the garch_fit bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 env STS_GARCH_SHAPE=64x64 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_garch.py -m gpu -k "garch_fit" > gpurun_out/garch_shape_tests.log 2>&1
for sh in 32x64 64x64 32x64 64x64; do
  STS_GARCH_SHAPE=$sh timeout -k 10 200 python -u bench.py --workload garch_fit --steps 1 --warmup 1 \
    --no-cpu-baseline > gpurun_out/garch_s$sh.json 2> gpurun_out/garch_s$sh.err
  echo "shape=$sh $(python -c "import json; print(json.load(open('gpurun_out/garch_s$sh.json'))['roofline']['avg_kernel_ms'])")"
done
STS_GARCH_SHAPE=64x64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_garch64 -o garch --output-format csv -- \
  python -u bench.py --workload garch_fit --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_garch64.log 2>&1
