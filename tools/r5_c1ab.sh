#!/bin/bash
# C1 A/B of the half-block short kernel (var_short2) against the product: parity first (the short
# kernel's GPU tests bound to the variant), then bench.py --workload c1 alternating libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r5}
mkdir -p $O
V=spark-timeseries_amd/build/var_${C1_VAR:-short2}/libsts_hip.so
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $PYT --sts-lib $V tests/test_parity_gpu.py -k "short or fused or c1" > $O/c1ab_parity1.log 2>&1 || { tail -20 $O/c1ab_parity1.log; exit 1; }
timeout -k 10 600 $PYT --sts-lib $V tests/test_acf_robust.py -k "product or returns" > $O/c1ab_parity2.log 2>&1 || { tail -20 $O/c1ab_parity2.log; exit 1; }
tail -1 $O/c1ab_parity1.log $O/c1ab_parity2.log
for rep in 1 2 3; do
  for L in base var; do
    if [ $L = var ]; then E="STS_HIP_LIB=$V"; else E=""; fi
    env $E timeout -k 10 200 python -u bench.py --workload c1 --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{' \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'ms_per_step': d['ms_per_step']}))" >> $O/c1ab.jsonl || exit 1
  done
done
cat $O/c1ab.jsonl
