#!/bin/bash
# Round-4 final-tree evidence: GPU tests, every workload's bench line, rocprof stats of the C3
# and C5 bench commands, C3 HBM traffic and FP64 counters, C5 three consecutive runs, smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="tests c3 prof fetch write fp64_c3 c1 c2 c4 c5 prof_c5" bash tools/gpu_all.sh || exit $?
set -e
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs.jsonl
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
