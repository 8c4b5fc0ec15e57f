#!/bin/bash
# Full GPU parity of the in-tree build, then tools/ab.sh of main against the given variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_main.log 2>&1
rc=$?; echo "parity main rc=$rc $(tail -1 gpurun_out/parity_main.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "${AB_CASES:-tile:linear:60}" main "$@" > gpurun_out/ab_main.jsonl; rc=$?
cat gpurun_out/ab_main.jsonl; exit $rc
