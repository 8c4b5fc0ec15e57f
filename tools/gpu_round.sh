#!/bin/bash
# One GPU session: parity tests, then a small bench, then smoke. Every GPU step has its
# own time limit; a step that dies by signal/timeout (rc >= 124) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc" >&2; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests bench smoke"}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    bench) run bench_small 400 python -u bench.py --series ${BENCH_SERIES:-1000} --steps 3 --warmup 1 --cpu-seconds 3 ;;
    benchfull) run bench_full 600 python -u bench.py ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    prof) export TMPDIR=/tmp; run rocprof_stats 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof -o bench --output-format csv -- python -u bench.py --series ${PROF_SERIES:-2000} --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmcfetch) export TMPDIR=/tmp; run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/pmc_fetch -o bench --output-format csv -- python -u bench.py --series ${PROF_SERIES:-2000} --steps 2 --warmup 0 --no-cpu-baseline ;;
    pmcwrite) export TMPDIR=/tmp; run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/pmc_write -o bench --output-format csv -- python -u bench.py --series ${PROF_SERIES:-2000} --steps 2 --warmup 0 --no-cpu-baseline ;;
    custom) run custom ${CUSTOM_SECS:-300} bash -c "$CUSTOM_CMD" ;;
  esac
done
