cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
STS_HIP_LIB=spark-timeseries_amd/build/var_arstg/libsts_hip.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_ar_price_levels.py tests/test_garch.py tests/test_mapseries.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "ar or garch or pipeline" > gpurun_out/t18.log 2>&1; rc=$?; tail -2 gpurun_out/t18.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh c4 base arstg
