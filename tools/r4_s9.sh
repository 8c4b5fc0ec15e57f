#!/bin/bash
# Round-4 session 9: phase-graded wave priorities in the C3 tile kernel (priority 3 for wave 0's
# word scan (pscan), the imputation (pimp), both (pscanimp), or the store pass (pstore); 2
# elsewhere, 0 in the MFMA phase) against the product, three alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
for rep in 1 2 3; do
  for V in base pscan pimp pscanimp pstore; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio4.jsonl
  done
done
