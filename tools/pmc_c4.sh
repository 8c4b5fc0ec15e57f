#!/bin/bash
# L1 -> L2 read requests and HBM fetch of the C4 (AR fit + remove) kernel: separate passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_c4_tcp -o c4 --output-format csv -- python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c4_tcp.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c4_fetch -o c4 --output-format csv -- python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c4_fetch.log 2>&1 || exit $?
for f in gpurun_out/pmc_c4_tcp/*counter_collection.csv gpurun_out/pmc_c4_fetch/*counter_collection.csv; do
  python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "ar_fit" in r["Kernel_Name"]:
        acc[(r["Kernel_Name"][:60], r["Counter_Name"])] += float(r["Counter_Value"])
for k, v in acc.items(): print(k, "%.4g" % v)
PY
done
