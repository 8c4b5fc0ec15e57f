#!/bin/bash
# Round-5 session 23: timing-only cost models of the C1 short kernel on the final tree
# (STS_SHORT_DIAG 1 no ACF, 2 no fill, 3 no per-lag finalize, 4 no robust shift, 5 no lag FMAs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
O=gpurun_out/r5; mkdir -p $O
bash tools/ab_bench.sh c1 base sd1 sd2 sd3 sd4 sd5 > $O/ab_c1_diag.jsonl
