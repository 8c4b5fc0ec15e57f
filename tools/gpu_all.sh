#!/bin/bash
# One GPU session: every workload's bench line, the rocprof stats of the default bench
# command, and FETCH_SIZE / WRITE_SIZE passes.  Every GPU step has its own time limit; a
# step that dies by signal/timeout (rc >= 124) or fails ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc" >&2; exit $rc; fi
}
for s in ${STEPS:-c1 c2 c4 c5 prof fetch write}; do
  case $s in
    c1|c2|c3|c4|c5|stage_c2|ewma_fit|garch_fit|stats|nan_instants|to_instants|wire_decode) step bench_$s 300 python -u bench.py --workload $s ;;
    prof) step prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o bench --output-format csv -- python -u bench.py ;;
    prof_*) W=${s#prof_}; step prof_$W 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$W -o bench --output-format csv -- python -u bench.py --workload $W --no-cpu-baseline ;;
    fetch) step pmc_fetch_c3 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c3 -o bench --output-format csv -- python -u bench.py --steps 2 --warmup 0 --no-cpu-baseline ;;
    write) step pmc_write_c3 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c3 -o bench --output-format csv -- python -u bench.py --steps 2 --warmup 0 --no-cpu-baseline ;;
    fetch_*) W=${s#fetch_}; step pmc_fetch_$W 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$W -o bench --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    write_*) W=${s#write_}; step pmc_write_$W 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$W -o bench --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    fp64_c3|fp64_c4) W=${s#fp64_}; step pmc_$s 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_$s -o bench --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    tests) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    custom) step custom ${CUSTOM_SECS:-300} bash -c "$CUSTOM_CMD" ;;
    pytest) step pytest_sel ${TEST_SECS:-900} python -u -m pytest $TEST_FILES -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    ab) step ab_libs ${AB_SECS:-600} bash tools/ab_libs.sh "$AB_CASES" $AB_LIBS ;;
  esac
done
