cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t19_all.log 2>&1; rc=$?; tail -3 gpurun_out/t19_all.log; [ $rc -ne 0 ] && exit $rc
STS_HIP_LIB=spark-timeseries_amd/build/var_arstg/libsts_hip.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_ar_price_levels.py tests/test_garch.py tests/test_mapseries.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "ar or garch or pipeline" > gpurun_out/t19_arstg.log 2>&1; rc=$?; tail -2 gpurun_out/t19_arstg.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh c4 base arstg || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/b19_c3.log 2>&1; rc=$?; tail -1 gpurun_out/b19_c3.log; exit $rc
