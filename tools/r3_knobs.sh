#!/bin/bash
# Same-box timing of A/B-knob settings (libsts_hip_ab.so) and library builds on the C3 shape.
# Usage: tools/r3_knobs.sh "<cases>" "ENV=VAL ..." ... ; a spec "lib:<var>" runs that build instead
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CASES=$1; shift
for rep in 1 2; do
  for spec in "$@"; do
    case $spec in
      lib:base) L=spark-timeseries_amd/build/libsts_hip.so; E="" ;;
      lib:*) L=spark-timeseries_amd/build/var_${spec#lib:}/libsts_hip.so; E="" ;;
      *) L=spark-timeseries_amd/build/libsts_hip_ab.so; E="$spec" ;;
    esac
    env $E STS_HIP_LIB=$L timeout -k 10 120 python -u tools/kbench.py --series ${AB_SERIES:-2000} --reps 5 --cases "$CASES" 2>/dev/null \
      | grep case | sed "s|^|{\"spec\": \"$spec\", \"rep\": $rep, \"r\": |; s|\$|}|" || exit 1
  done
done
