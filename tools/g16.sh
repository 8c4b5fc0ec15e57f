cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
STS_HIP_LIB=spark-timeseries_amd/build/var_rv2/libsts_hip.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_mapseries.py tests/test_staging.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "fill_diff or pipeline or stag" > gpurun_out/t16.log 2>&1; rc=$?; tail -2 gpurun_out/t16.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for L in base rv2; do
  if [ $L = rv2 ]; then P=spark-timeseries_amd/build/var_rv2/libsts_hip.so; else P=spark-timeseries_amd/build/libsts_hip.so; fi
  STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$L', d['roofline']['avg_kernel_ms'], d['roofline']['achieved'])" || exit 1
done; done
