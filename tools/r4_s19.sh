#!/bin/bash
# Round-4 session 19: tiles per tile-kernel workgroup for the fill-only + lag-matrix instantiation
# (C5) through the A/B build's STS_TILES_PER_CHUNK knob, two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_bench.sh c5 ab:STS_TILES_PER_CHUNK=16 ab:STS_TILES_PER_CHUNK=2 ab:STS_TILES_PER_CHUNK=1 ab:STS_TILES_PER_CHUNK=4 > gpurun_out/ab_c5_tpc.jsonl
