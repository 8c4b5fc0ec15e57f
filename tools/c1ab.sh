for r in 1 2; do for v in main ntst; do
  if [ $v = main ]; then lib=spark-timeseries_amd/build/libsts_hip.so; else lib=spark-timeseries_amd/build/var_$v/libsts_hip.so; fi
  STS_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --workload c1 --no-cpu-baseline --steps 50 --warmup 5 | sed "s/^/$v /" || exit 1
done; done
