#!/bin/bash
# Round-5 GPU session driver: STEPS="..." picks the steps, each under its own time limit;
# a failing or killed step ends the session (no retries).  Outputs under gpurun_out/r5/.
#   artests        AR rule / QR parity tests (tests/test_ar_price_levels.py + the AR rows of test_parity_gpu.py)
#   tests          the whole GPU suite
#   c1 c2 c3 c4 c5 bench lines (bench.py --workload ..)
#   prof_<wl>      rocprofv3 --kernel-trace --stats of the bench command
#   fetch_<wl> write_<wl>  FETCH_SIZE / WRITE_SIZE passes
#   c5diag         three consecutive C5 processes under clock + UTCL1 counters, then a plain line
#   smoke          __graft_entry__.smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r5}
mkdir -p $O
export TMPDIR=/tmp
sha256sum spark-timeseries_amd/build/libsts_hip.so > $O/libsha.txt
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)" >&2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -4 "$O/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc" >&2; exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
for s in ${STEPS:-artests}; do
  case $s in
    artests) step artests 900 $PYT -m gpu tests/test_ar_price_levels.py tests/test_parity_gpu.py -k "ar_ or arima or argarch or AR" ;;
    tests) step tests 1100 $PYT -m gpu tests ;;
    pytest) step pytest_sel ${TEST_SECS:-900} $PYT -m gpu $TEST_FILES ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    c1|c2|c3|c4|c5|c4_levels|c1_rule3|c3_rule3|ewma_fit|garch_fit|stats|nan_instants|to_instants|wire_decode|stage_c2|spline) step bench_$s 300 python -u bench.py --workload $s ;;
    percall) step percall 300 python -u bench.py --percall ;;
    prof_*) W=${s#prof_}; step prof_$W 400 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python -u bench.py --workload $W --no-cpu-baseline ;;
    fetch_*) W=${s#fetch_}; step pmc_fetch_$W 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$W -o run --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    write_*) W=${s#write_}; step pmc_write_$W 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$W -o run --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    fp64_*) W=${s#fp64_}; step pmc_fp64_$W 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_fp64_$W -o run --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline ;;
    c5diag)
      timeout -k 5 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
      for rep in 1 2 3; do
        step c5diag_p$rep 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
          -d $O/c5diag_p$rep -o run --output-format csv -- python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
      done
      step bench_c5_after 300 python -u bench.py --workload c5 --no-cpu-baseline ;;
    c5diag2)
      # second set: DRAM-side credit stalls, UTCL2 busy / out-of-credit stalls, per process
      for rep in 1 2 3; do
        step c5diag2_p$rep 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY TCP_UTCL1_TRANSLATION_MISS_sum \
          TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
          -d $O/c5diag2_p$rep -o run --output-format csv -- python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
      done ;;
    c5diag3)
      # third set: is one L2 channel hot?  max-over-instances write stalls, tag stalls
      for rep in 1 2 3; do
        step c5diag3_p$rep 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCC_WRREQ_STALL_max TCC_TAG_STALL_sum \
          TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_STALL_sum \
          -d $O/c5diag3_p$rep -o run --output-format csv -- python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
      done ;;
    sq_*) W=${s#sq_}; step pmc_sq_$W 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
          -d $O/pmc_sq_$W -o run --output-format csv -- python -u bench.py --workload $W --series ${SQ_SERIES:-0} --steps 2 --warmup 0 --no-cpu-baseline ;;
    kbench) step kbench 600 env STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so python -u tools/kbench.py --series ${KB_SERIES:-12500} --reps 3 --cases ${KB_CASES:-tile:linear:60,seg:linear:60} ;;
    ablibs) step ablibs ${AB_SECS:-900} env AB_SERIES=${AB_SERIES:-4000} bash tools/ab_libs.sh "${AB_CASES:-tile:linear:60}" $AB_LIBS ;;
    custom) step custom ${CUSTOM_SECS:-300} bash -c "$CUSTOM_CMD" ;;
  esac
done
