#!/bin/bash
# Round-5 session 25: the C1 short kernel's finalize with DPP suffix sums (var_c1dpp) -- its parity
# rows, then C1 bench A/B; and the C3 tiles-per-workgroup sweep with non-temporal loads (tools/r5_s24.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py tests/test_acf_robust.py \
    -k "short or fill_acf or product or returns" --sts-lib spark-timeseries_amd/build/var_c1dpp/libsts_hip.so > $O/c1dpp_parity.log 2>&1
bash tools/ab_bench.sh c1 base c1dpp > $O/ab_c1dpp.jsonl
bash tools/ab_bench.sh c1 c1dpp base >> $O/ab_c1dpp.jsonl
bash tools/r5_s24.sh
