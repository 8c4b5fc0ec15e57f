#!/bin/bash
# A/B kernel timing in ONE process per variant, interleaved R rounds (box-to-box variance
# is ~15 %, so only same-run comparisons count).  Usage: tools/ab.sh "cases" var1 var2 ...
# (variant "main" = spark-timeseries_amd/build/libsts_hip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CASES=$1; shift
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=spark-timeseries_amd/build/libsts_hip.so; else lib=spark-timeseries_amd/build/var_$v/libsts_hip.so; fi
    STS_HIP_LIB=$lib timeout -k 10 300 python -u tools/kbench.py --series ${AB_SERIES:-2000} --cases "$CASES" 2>/dev/null |
      sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" || exit 1
  done
done
