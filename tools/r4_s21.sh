#!/bin/bash
# Round-4 session 21: one tile per workgroup for the fill-only / lag-matrix tile launches -- full
# GPU suite, C5 bench (four processes) with rocprof stats, fill-only kbench on the C3 shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="tests c5 prof_c5" bash tools/gpu_all.sh || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs4.jsonl || exit 1
done
timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:0,tile:nearest:0 > gpurun_out/kb_fill_tpc1.jsonl
