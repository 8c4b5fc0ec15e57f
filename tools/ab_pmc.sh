#!/bin/bash
# Same-box A/B of library variants on bench workloads + one SQ instruction-count PMC pass per
# variant.  AB_WLS="c3 c1" AB_VARS="main r01 ..." PMC_VARS="main r01" tools/ab_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
libof() { if [ "$1" = main ]; then echo spark-timeseries_amd/build/libsts_hip.so; else echo spark-timeseries_amd/build/var_$1/libsts_hip.so; fi; }
for r in 1 2; do for w in ${AB_WLS:-c3}; do for v in ${AB_VARS:-main}; do
  STS_HIP_LIB=$(libof $v) timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps ${AB_STEPS:-10} --warmup 3 \
    ${AB_SERIES:+--series $AB_SERIES} | sed "s/^/$v $w /" >> gpurun_out/ab.txt || exit 1
done; done; done
CTRS=${PMC_CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"}
for v in ${PMC_VARS:-}; do
  STS_HIP_LIB=$(libof $v) timeout -s KILL 120 rocprofv3 --pmc $CTRS -T -d gpurun_out/pmc_$v -o run --output-format csv -- \
      python -u bench.py --workload ${PMC_WL:-c3} --series ${PMC_SERIES:-1000} --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc" >> gpurun_out/ab.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
