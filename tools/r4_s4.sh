#!/bin/bash
# Round-4 session 4: the per-wave scan variant (WSCAN) parity + C3 A/B; C2 stride fix; C5 store forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    --sts-lib spark-timeseries_amd/build/var_wscan/libsts_hip.so > gpurun_out/pytest_wscan.log 2>&1
for rep in 1 2; do
  for V in base wscan; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    for NAN in 0.05 0.3; do
      STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --nan $NAN \
          --cases tile:linear:60,tile:linear:0 | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, \"nan\": $NAN, /" >> gpurun_out/kb_wscan.jsonl
    done
  done
done
bash tools/ab_bench.sh c2 base ch128 r3 > gpurun_out/ab_c2.jsonl
for rep in 1 2 3; do
  for L in base c5plain r3; do
    P=spark-timeseries_amd/build/libsts_hip.so; [ $L != base ] && P=spark-timeseries_amd/build/var_$L/libsts_hip.so
    STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/c5_forms.jsonl
  done
done
for rep in 1 2; do
  for V in base wscanab; do
    L=spark-timeseries_amd/build/libsts_hip.so; E=""; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so && E="STS_TILE_W=2048"
    env $E STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_wscan2w.jsonl
  done
done
