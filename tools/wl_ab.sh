#!/bin/bash
# A/B of library variants on bench.py workloads, interleaved rounds in one box session:
#   tools/wl_ab.sh "c3 c2" main var1 var2 ...   (main = spark-timeseries_amd/build/libsts_hip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WLS=$1; shift
for r in 1 2; do for w in $WLS; do for v in "$@"; do
  if [ "$v" = main ]; then lib=spark-timeseries_amd/build/libsts_hip.so; else lib=spark-timeseries_amd/build/var_$v/libsts_hip.so; fi
  STS_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline ${WL_ARGS:-} | sed "s/^/$v $w /" || exit 1
done; done; done
