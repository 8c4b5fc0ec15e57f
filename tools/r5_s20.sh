#!/bin/bash
# Round-5 session 20: cache policy of the staged-series kernels (C1 short kernel, C4 AR kernel, C2
# row kernel): non-temporal LDS-DMA loads (var_dmant), non-temporal 16-B result stores (var_stnt),
# both (var_ntboth) -- parity of the short / AR / recurrence rows on ntboth, then bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py \
    -k "short or fill_acf or ar_ or fill_diff or ewma" --sts-lib spark-timeseries_amd/build/var_ntboth/libsts_hip.so > $O/ntboth_parity.log 2>&1
for W in c1 c4 c2; do
  bash tools/ab_bench.sh $W base dmant stnt ntboth >> $O/ab_policy.jsonl
done
