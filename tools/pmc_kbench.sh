#!/bin/bash
# SQ counter passes over tools/kbench.py (one rocprofv3 --pmc pass per group; per-dispatch
# rows in gpurun_out/pmck_<i>/).  Usage: tools/pmc_kbench.sh "<cases>" "<grp1>" "<grp2>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CASES=$1; shift
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $grp" >&2
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmck_$i -o run --output-format csv -- \
      python -u tools/kbench.py --series ${PROF_SERIES:-1000} --reps 1 --cases "$CASES" > gpurun_out/pmck_$i.log 2>&1
  rc=$?
  echo "=== pass $i rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmck_$i.log >&2; exit $rc; fi
done
