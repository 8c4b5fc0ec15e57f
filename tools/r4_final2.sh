#!/bin/bash
# Round-4 final-tree evidence (second set, after the C2 row kernel and the C3 priorities): full GPU
# suite, every workload's bench line, rocprof stats of C3 / C2 / C5, FETCH / WRITE of C3 and C2,
# FP64 counters of C3, three more C5 processes, smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="tests c3 prof fetch write fp64_c3 c2 prof_c2 fetch_c2 write_c2 c1 c4 c5 prof_c5" bash tools/gpu_all.sh || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs2.jsonl || exit 1
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1
