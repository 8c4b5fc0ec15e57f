#!/bin/bash
# Same-box A/B of library builds: tools/ab_libs.sh "CASES" lib1 lib2 ... (paths or var names)
# -> one kbench JSON line per (lib, case), twice in alternating order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CASES=$1; shift
SER=${AB_SERIES:-2000}
for rep in 1 2; do
  for L in "$@"; do
    case $L in
      base) P=spark-timeseries_amd/build/libsts_hip.so ;;
      ab) P=spark-timeseries_amd/build/libsts_hip_ab.so ;;
      *) P=spark-timeseries_amd/build/var_$L/libsts_hip.so ;;
    esac
    STS_HIP_LIB=$P timeout -k 10 120 python -u tools/kbench.py --series $SER --reps 5 --cases "$CASES" 2>/dev/null \
      | grep -v amdgpu.ids | sed "s/^/{\"lib\": \"$L\", \"rep\": $rep, \"r\": /; s/\$/}/" || exit $?
  done
done
