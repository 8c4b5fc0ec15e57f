#!/bin/bash
# Same-box A/B of library builds on one bench workload: tools/ab_bench.sh WORKLOAD lib1 lib2 ...
# (base = the product library, ab:ENV=VAL = the A/B-knob build with that knob, anything else =
# build/var_<name>); two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL=$1; shift
for rep in 1 2; do
  for L in "$@"; do
    E=""
    case $L in base) P=spark-timeseries_amd/build/libsts_hip.so ;;
      ab:*) P=spark-timeseries_amd/build/libsts_hip_ab.so; E=${L#ab:} ;;
      *) P=spark-timeseries_amd/build/var_$L/libsts_hip.so ;; esac
    env $E STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null \
      | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'workload': '$WL', 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" || exit 1
  done
done
