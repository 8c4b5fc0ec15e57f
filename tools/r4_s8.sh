#!/bin/bash
# Round-4 session 8 (second call: prio_0 = no priority change, same box as base and prio_s): wave priority around the C3 MFMA phase -- the product (STS_FILL_PRIO=2) on
# the full GPU suite, then C3 kernel A/B against priority 1 / 3 and against raising it from the
# first tile on (prio_s), three alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tile or acf or fill" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_prio.log 2>&1
for rep in 1 2 3; do
  for V in prio_0 base prio_s; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio3.jsonl
  done
done
