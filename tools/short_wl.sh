cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in c1 stats c2; do
  timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/short_$w.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/short_$w.json')); print('$w', '%.4g'%d['value'], round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'])"
done
