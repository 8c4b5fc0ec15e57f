#!/bin/bash
# Round-4 session 3: the C2 rows kernel (v2) against the round-3 tree, C5 run-to-run drift (three
# consecutive runs per library), and the C3 kernel's sensitivity to the NaN rate (how much of the
# fused time the imputation phases hold).  The first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 200 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider --sts-lib spark-timeseries_amd/build/var_rows/libsts_hip.so > gpurun_out/pytest_rows.log 2>&1
bash tools/ab_bench.sh c2 base rows r3 > gpurun_out/ab_c2.jsonl
for L in base r3; do
  P=spark-timeseries_amd/build/libsts_hip.so; [ $L != base ] && P=spark-timeseries_amd/build/var_$L/libsts_hip.so
  for rep in 1 2 3; do
    STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/c5_drift.jsonl
  done
done
for NAN in 0.0 0.05 0.3; do
  timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --nan $NAN --cases tile:linear:60,tile:linear:0 \
    | sed "s/^{/{\"nan\": $NAN, /" >> gpurun_out/kb_nan.jsonl
done
