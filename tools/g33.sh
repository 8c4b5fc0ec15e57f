cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_staging.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
for rep in 1 2; do for L in l0s3 l1s4 l0s4 l1s5 l0s5 l1s6; do
  case $L in base) P=spark-timeseries_amd/build/libsts_hip.so ;; *) P=spark-timeseries_amd/build/var_$L/libsts_hip.so ;; esac
  STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload stage_c2 --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['staging']; print(json.dumps({'lib': '$L', 'rep': $rep, 'pinned_ms': st['pinned']['wall_ms'], 'pinned_both_GBps': st['pinned']['pcie_both_ways_GBps'], 'h2d': st['pinned']['h2d_GBps'], 'd2h': st['pinned']['d2h_GBps'], 'pageable_ms': st['pageable']['wall_ms']}))" || exit 1
done; done
