#!/bin/bash
# Tiles per tile-kernel workgroup on the C3 shard (A/B build, STS_TILES_PER_CHUNK), fill only and
# fill + ACF(60): does a denser sweep of the panel by the resident workgroups (fewer tiles each)
# move the fill path's memory rate?  Two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
for rep in 1 2; do
  for N in ${TPCS:-1 2 4 16 64}; do
    STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 200 python -u tools/kbench.py \
        --series ${KB_SERIES:-12500} --reps 3 --cases ${KB_CASES:-tile:linear:0,tile:linear:60} \
        | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> gpurun_out/kb_tpc.jsonl
  done
done
