#!/bin/bash
# A/B of the seg kernel's segment length (STS_SEG_TILES) on the C1 shape, same process family.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do for v in ${SEG_VALUES:-128 3 2 1}; do
  STS_SEG_TILES=$v timeout -k 10 120 python -u bench.py --workload ${WL:-c1} --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/seg_ab_$v.json || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/seg_ab_$v.json')); print('seg_tiles=$v round=$r', round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'], d['roofline']['achieved'])" | tee -a gpurun_out/seg_ab.txt
done; done
