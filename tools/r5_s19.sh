#!/bin/bash
# Round-5 session 19: non-temporal prefetch loads (var_ntl) against the product, three more
# alternating rounds on C3 (kernel A/B) and on C5 (bench, after one warm-up C5 process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
for rep in 3 4 5; do
  for V in ntl base; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 300 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
      | grep -v amdgpu.ids | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> $O/rs_ab.jsonl
  done
done
timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
bash tools/ab_bench.sh c5 base ntl >> $O/ab_c5_ntl.jsonl
bash tools/ab_bench.sh c5 ntl base >> $O/ab_c5_ntl.jsonl
