#!/bin/bash
# Round-4 final-tree evidence (fourth set: + one tile per workgroup for fill-only / lag-matrix launches): full GPU
# suite, every workload's bench line, rocprof stats of C3 / C2 / C5, FETCH / WRITE of C3 and C2,
# FP64 counters of C3, three more C5 processes, smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="tests c3 prof fetch write fp64_c3 c2 prof_c2 fetch_c2 write_c2 c1 c4 c5 prof_c5" bash tools/gpu_all.sh || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs5.jsonl || exit 1
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke5.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    -d gpurun_out/c2sq_final5 -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_final5.log 2>&1
