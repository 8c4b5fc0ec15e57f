#!/bin/bash
# Round-5 session 24: tiles per tile-kernel workgroup for fill + ACF(60) on the C3 shard with the
# non-temporal prefetch loads (A/B build knob STS_TILES_PER_CHUNK): 12 / 16 (product) / 24 / 32, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
for rep in 1 2; do
  for N in 16 12 24 32; do
    STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 300 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
      | grep -v amdgpu.ids | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> $O/kb_c3_tpc_nt.jsonl
  done
done
