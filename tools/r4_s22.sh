#!/bin/bash
# Round-4 session 22: tiles per tile-kernel workgroup for fill + ACF(60) on the C3 shard (A/B
# build knob): 8 / 12 / 16 (product) / 24 / 32, two alternating rounds through tools/kbench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for N in 16 8 12 24 32; do
    STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
      | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> gpurun_out/kb_c3_tpc.jsonl || exit 1
  done
done
