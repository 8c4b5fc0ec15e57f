cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t28_all.log 2>&1; rc=$?; tail -3 gpurun_out/t28_all.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh c2 base norows || exit 1
bash tools/ab_bench.sh c4 base nodma
