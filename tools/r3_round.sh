#!/bin/bash
# r3 GPU session: full GPU tests, then same-box A/B of library builds on C3 shapes, then
# one SQ instruction-count pass.  Env: AB_LIBS (var names / base), AB_CASES, SQ_CASES.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
bash tools/ab_libs.sh "${AB_CASES:-tile:linear:60,tile:linear:0}" ${AB_LIBS:-base} > gpurun_out/ab.jsonl 2>&1 || exit 1
cat gpurun_out/ab.jsonl
if [ -n "$SQ_CASES" ]; then bash tools/r3_sqcases.sh "$SQ_CASES" "" _new || exit 1; fi
