cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
STS_HIP_LIB=spark-timeseries_amd/build/var_db/libsts_hip.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_acf_robust.py tests/test_acf_wide.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x > gpurun_out/t15.log 2>&1; rc=$?; tail -3 gpurun_out/t15.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh tile:linear:60,tile:previous:60,tile:linear:20 base db > gpurun_out/ab_db.jsonl; cat gpurun_out/ab_db.jsonl
