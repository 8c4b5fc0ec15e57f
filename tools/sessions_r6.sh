#!/bin/bash
# Round-6 GPU sessions, one per case: `bash tools/sessions_r6.sh s1` re-runs what the round-6 rows
# of profiles/INDEX.md name as session s1.  Each step keeps its own time limit and the session stops at
# its first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SESSION=$1; shift
O=${OUT_DIR:-gpurun_out/r6}
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
case "$SESSION" in
  spline)
    # fill("spline") on the device, the fixed fill -> diff -> EWMA composition, then the
    # per-call latency table (bench.py --percall)
    timeout -k 10 600 $PYT tests/test_spline.py tests/test_parity_gpu.py -k "spline or unsupported or fill_diff_ewma" \
        > $O/spline_pytest.log 2>&1 || { tail -30 $O/spline_pytest.log; exit 1; }
    tail -2 $O/spline_pytest.log
    timeout -k 10 600 python -u bench.py --percall > $O/percall.json 2> $O/percall.err || { tail -20 $O/percall.err; exit 1; }
    cat $O/percall.json
    ;;
  arfilled)
    # AR fit on filled series + the near-threshold rows
    timeout -k 10 900 $PYT tests/test_ar_filled.py > $O/arfilled_pytest.log 2>&1 || { tail -40 $O/arfilled_pytest.log; exit 1; }
    tail -2 $O/arfilled_pytest.log
    ;;
  *)
    echo "unknown session $SESSION"; exit 2 ;;
esac
