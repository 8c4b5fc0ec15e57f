#!/bin/bash
# A/B of the GARCH tail kernel's chunk length (STS_GARCH_TAIL_C) on the garch_fit bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 env STS_GARCH_TAIL_C=256 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_garch.py -m gpu -k "garch_fit" > gpurun_out/garch_tailc_tests.log 2>&1
for c in 128 256 64 128; do
  STS_GARCH_TAIL_C=$c timeout -k 10 200 python -u bench.py --workload garch_fit --steps 1 --warmup 1 \
    --no-cpu-baseline > gpurun_out/garch_c$c.json 2> gpurun_out/garch_c$c.err
  echo "C=$c $(python -c "import json; print(json.load(open('gpurun_out/garch_c$c.json'))['roofline']['avg_kernel_ms'])")"
done
