#!/bin/bash
# Round-4 session 20: C5 tiles per workgroup 1 vs 16 (A/B build knob), alternating three times,
# after one warm-up C5 process (the first C5 process on a box runs fast).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip.so timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
for rep in 1 2 3; do
  for L in ab:STS_TILES_PER_CHUNK=1 ab:STS_TILES_PER_CHUNK=16 base; do
    E=""; P=spark-timeseries_amd/build/libsts_hip.so
    case $L in ab:*) P=spark-timeseries_amd/build/libsts_hip_ab.so; E=${L#ab:} ;; esac
    env $E STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null \
      | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'workload': 'c5', 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/ab_c5_tpc2.jsonl || exit 1
  done
done
