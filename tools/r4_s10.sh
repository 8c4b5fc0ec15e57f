#!/bin/bash
# Round-4 session 10: recur_row_kernel (one wave per series, affine-scan guess verified lane by
# lane) -- recurrence parity, then C2 A/B against the 16 x 128 chunk kernel (var_chunk), and the
# C3 priority-in-scan A/B (pscan / pscanimp) once more.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "recur or ewma or fill_diff" > gpurun_out/pytest_rowscan.log 2>&1
bash tools/ab_bench.sh c2 base chunk > gpurun_out/ab_c2_rowscan.jsonl
for rep in 1 2; do
  for V in base pscan pscanimp; do
    L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
    STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
        | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio5.jsonl
  done
done
