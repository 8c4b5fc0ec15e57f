#!/bin/bash
# Round-5 session 22: cache-policy modifiers of the C1 short kernel (result stores: nt = product,
# sc0 sc1 nt, sc1 nt, sc1; DMA loads: sc1, sc0 sc1) -- parity on two variants, C1 bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
for V in st2 ld3; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py \
      -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > $O/pol_parity_$V.log 2>&1
done
bash tools/ab_bench.sh c1 base st2 st3 st4 ld2 ld3 > $O/ab_c1_pol.jsonl
