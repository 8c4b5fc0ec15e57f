#!/bin/bash
# SQ / TCC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${PROF_SERIES:-500}
WL=${WORKLOAD:-c3}
i=0
for grp in "${@}"; do
  i=$((i+1))
  echo "=== pass $i: $grp" >&2
  timeout -s KILL 120 rocprofv3 --pmc $grp -T -d gpurun_out/pmc_$i -o run --output-format csv -- \
      python -u bench.py --workload $WL --series $N --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$i.log 2>&1
  rc=$?
  echo "=== pass $i rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$i.log >&2; exit $rc; fi
done
