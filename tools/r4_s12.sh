#!/bin/bash
# Round-4 session 12: the tree with the C2 row kernel and the C3 scan priority -- full GPU suite,
# C2 bench + rocprof stats + FETCH / WRITE passes, C3 bench + rocprof stats; then the wave-0
# scan priority for the fill-only (C5) instantiation as an A/B variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="tests c2 prof_c2 fetch_c2 write_c2 c3 prof" bash tools/gpu_all.sh || exit 1
bash tools/ab_bench.sh c5 base c5prio > gpurun_out/ab_c5_prio.jsonl
