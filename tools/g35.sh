cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t35.log 2>&1; rc=$?; tail -1 gpurun_out/t35.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t35.log | head -10; exit $rc; }
bash tools/ab_bench.sh c1 base novtab
