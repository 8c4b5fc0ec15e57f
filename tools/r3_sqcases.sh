#!/bin/bash
# One SQ instruction-count pass over several kbench cases (per-dispatch rows, in case order:
# each case = one warm-up call + --reps calls).  Usage: tools/r3_sqcases.sh "<cases>" [lib]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CASES=$1
[ -n "$2" ] && export STS_HIP_LIB=$2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
  -d gpurun_out/sqcases${3} -o run --output-format csv -- python -u tools/kbench.py --series ${PROF_SERIES:-1000} --reps 1 --cases "$CASES" > gpurun_out/sqcases${3}.log 2>&1
