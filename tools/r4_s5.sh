#!/bin/bash
# Round-4 session 5: the fill method as a template parameter (+ the SGPR-spill cut of 7b06d88)
# against 7b06d88 (var_s5) and the round-3 tree (var_r3) on C3 / C2 / C5, and SQ counters of the
# product and the measured-negative variants (LDS-DMA 2048-step tiles, per-wave scans).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
for rep in 1 2; do
  for V in base s5 r3; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60,tile:linear:0 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_s5.jsonl
  done
done
bash tools/ab_bench.sh c5 base r3 > gpurun_out/ab_c5.jsonl
bash tools/ab_bench.sh c2 base r3 > gpurun_out/ab_c2.jsonl
for V in base r3 dma wscan; do
  L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
  bash tools/r3_sqcases.sh tile:linear:60,tile:linear:0 $L _$V
done
