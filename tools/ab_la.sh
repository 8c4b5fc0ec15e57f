#!/bin/bash
# A/B of the line-aligned seriesStats chunks: the product library against
# build/var_laoff (STS_STATS_LA=0), alternating, same box -> gpurun_out/r5la/ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5la; mkdir -p $O
for rep in 1 2 3; do
  for lib in product laoff; do
    for wl in stats; do
      if [ $lib = product ]; then E=""; else E="STS_HIP_LIB=spark-timeseries_amd/build/var_laoff/libsts_hip.so"; fi
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
