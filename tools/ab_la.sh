#!/bin/bash
# Same-box alternating A/B of the product library against build/var_$VAR (default laoff:
# STS_STATS_LA=0) on the workloads $WLS (default stats) -> gpurun_out/r5la/ab.jsonl
#   VAR=trxcd0 WLS=to_instants bash tools/ab_la.sh   (the XCD-contiguous transpose tiles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5la; mkdir -p $O
for rep in 1 2 3; do
  for lib in product ${VAR:-laoff}; do
    for wl in ${WLS:-stats}; do
      if [ $lib = product ]; then E=""; else E="STS_HIP_LIB=spark-timeseries_amd/build/var_$lib/libsts_hip.so"; fi
      env $E timeout -k 10 240 python -u bench.py --workload $wl --no-cpu-baseline > $O/$lib.$wl.$rep.log 2>&1 || exit 1
      python - "$lib" "$wl" "$rep" "$O/$lib.$wl.$rep.log" >> $O/ab.jsonl <<'PY'
import json, sys
ln = [l for l in open(sys.argv[4]) if l.startswith("{")][-1]
d = json.loads(ln)
print(json.dumps({"lib": sys.argv[1], "workload": sys.argv[2], "rep": int(sys.argv[3]),
                  "kernel_ms": d["roofline"]["avg_kernel_ms"], "frac": d["roofline"]["frac"], "lib_sha16": d["roofline"]["lib_sha16"]}))
PY
    done
  done
done
cat $O/ab.jsonl
