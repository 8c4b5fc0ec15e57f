#!/bin/bash
# Round-4 closing session: the C2 shape A/B with XCD remap on (tools/r4_s17.sh), then the
# final-tree evidence (tools/r4_final3.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r4_s17.sh || exit 1
bash tools/r4_final3.sh
