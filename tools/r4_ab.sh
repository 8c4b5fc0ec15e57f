#!/bin/bash
# Round-4 A/B session steps (after tools/gpu_all.sh's own steps): variant parity, kernel-level
# C3 A/B of the product and the LDS-DMA variant on the full C3 shard, C2 / C5 against the
# round-3 tree, phase stamps.  Every GPU step has its own limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
for V in ${VARS:-dma}; do
  timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
done
for rep in 1 2; do
  for V in base ${VARS:-dma}; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series ${KB_SERIES:-12500} --reps 3 \
        --cases ${KB_CASES:-tile:linear:60,tile:linear:0} | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_c3.jsonl
  done
done
[ -n "$NO_C2C5" ] || bash tools/ab_bench.sh c2 base r3 > gpurun_out/ab_c2.jsonl
[ -n "$NO_C2C5" ] || bash tools/ab_bench.sh c5 base r3 > gpurun_out/ab_c5.jsonl
STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_stamps.so timeout -k 10 120 python tools/stamps.py 2000 60 0 > gpurun_out/stamps.json
