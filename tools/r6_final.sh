#!/bin/bash
# Round-6 final-tree evidence, in three calls (each within gpurun's 20-minute limit), on the driver
# of tools/r5_session.sh:
#   bash tools/r6_final.sh A   -> the whole GPU suite, smoke(), C3 bench + rocprof stats + FETCH / WRITE / FP64 passes
#   bash tools/r6_final.sh B   -> C1 / C2 / C4 / C5 lines, rocprof stats and PMC passes, the worst cases, spline, per-call
#   bash tools/r6_final.sh F   -> the f rows
# Outputs under gpurun_out/r6f (then: python tools/collect.py r06_final gpurun_out/r6f).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT_DIR=gpurun_out/r6f
case "$1" in
  A) STEPS="tests smoke c3 prof_c3 fetch_c3 write_c3 fp64_c3" bash tools/r5_session.sh ;;
  B) STEPS="c1 prof_c1 fetch_c1 write_c1 c2 prof_c2 fetch_c2 write_c2 c4 prof_c4 fetch_c4 write_c4 fp64_c4 c5 prof_c5 fetch_c5 write_c5 c4_levels c1_rule3 c3_rule3 spline prof_spline fetch_spline write_spline percall" bash tools/r5_session.sh ;;
  F) STEPS="stats prof_stats fetch_stats write_stats nan_instants prof_nan_instants fetch_nan_instants write_nan_instants to_instants prof_to_instants fetch_to_instants write_to_instants wire_decode prof_wire_decode fetch_wire_decode write_wire_decode ewma_fit prof_ewma_fit fetch_ewma_fit write_ewma_fit fp64_ewma_fit stage_c2 prof_stage_c2 garch_fit prof_garch_fit fp64_garch_fit" bash tools/r5_session.sh ;;
  *) echo "usage: $0 A|B|F" >&2; exit 2 ;;
esac
