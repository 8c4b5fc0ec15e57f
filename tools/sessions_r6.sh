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
  rule3)
    # rule 3's fallback streamed through LDS: parity first, then the worst-case
    # bench lines c1_rule3 / c3_rule3 and the normal c1 / c3 lines (the fallback must not cost them)
    timeout -k 10 900 $PYT tests/test_acf_robust.py tests/test_acf_wide.py > $O/rule3_pytest1.log 2>&1 || { tail -40 $O/rule3_pytest1.log; exit 1; }
    tail -2 $O/rule3_pytest1.log
    timeout -k 10 900 $PYT tests/test_parity_gpu.py -k "acf or autocorr or rule3 or short or constant" > $O/rule3_pytest2.log 2>&1 || { tail -40 $O/rule3_pytest2.log; exit 1; }
    tail -2 $O/rule3_pytest2.log
    for w in c1_rule3 c3_rule3 c1; do
      timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 4 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', round(d['ms_per_step'],3), r['avg_kernel_ms'], r['frac'], d['cpu_baseline']['sample_check'])"
    done
    ;;
  latency)
    # dependent-chain latency of FP64 VALU ops (the floor of the bit-exact sequential recurrences)
    timeout -k 10 120 ./tools/ubench_latency > $O/ubench_latency.jsonl && cat $O/ubench_latency.jsonl
    ;;
  ewmares)
    # EWMA.fitModel: series block re-streamed per optimizer request (product) against the block held
    # in LDS (A/B build, STS_EWMA_RES=16 | 32 rows per wave); same box, alternating, with the
    # bench's sample check (smoothing bit-identical to the commons-math3 restatement)
    AB=spark-timeseries_amd/build/libsts_hip_ab.so
    for rep in 1 2; do
      for V in base res16 res32; do
        case $V in
          base) E="" ;;
          res16) E="STS_HIP_LIB=$AB STS_EWMA_RES=16" ;;
          res32) E="STS_HIP_LIB=$AB STS_EWMA_RES=32" ;;
        esac
        env $E timeout -k 10 300 python -u bench.py --workload ewma_fit --steps 3 --warmup 1 --cpu-seconds 2 > $O/ewmares_$V.json 2> $O/ewmares_$V.err || { tail -20 $O/ewmares_$V.err; exit 1; }
        python -c "import json; d=json.load(open('$O/ewmares_$V.json')); r=d['roofline']; print(json.dumps({'variant': '$V', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'ms_per_step': d['ms_per_step'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/ewmares.jsonl
      done
    done
    ;;
  arskip)
    # C4: the register AR kernel skipping its refinement pass on nearly orthogonal lags (product)
    # against the same sources with -DSTS_AR_SKIP_REFINE=0 (var_norefskip); AR parity first
    timeout -k 10 900 $PYT tests/test_ar_price_levels.py tests/test_ar_filled.py > $O/arskip_pytest1.log 2>&1 || { tail -40 $O/arskip_pytest1.log; exit 1; }
    tail -1 $O/arskip_pytest1.log
    timeout -k 10 900 $PYT tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_garch.py -k "ar or AR or arima or argarch" > $O/arskip_pytest2.log 2>&1 || { tail -40 $O/arskip_pytest2.log; exit 1; }
    tail -1 $O/arskip_pytest2.log
    V=spark-timeseries_amd/build/var_norefskip/libsts_hip.so
    for rep in 1 2 3; do
      for L in skip norefskip; do
        if [ $L = norefskip ]; then E="STS_HIP_LIB=$V"; else E=""; fi
        env $E timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --cpu-seconds 2 > $O/arskip_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/arskip_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/arskip.jsonl
      done
    done
    ;;
  pair)
    # C1: the short kernel with two series per LDS block (STS_SHORT_PAIR on the A/B
    # build): parity through the pair form first, then C1 / c1_rule3 alternating the two forms
    AB=spark-timeseries_amd/build/libsts_hip_ab.so
    timeout -k 10 900 $PYT tests/test_parity_gpu.py -k "short or fused or both_kernels" > $O/pair_pytest1.log 2>&1 || { tail -40 $O/pair_pytest1.log; exit 1; }
    tail -1 $O/pair_pytest1.log
    STS_SHORT_PAIR=1 timeout -k 10 900 $PYT --sts-lib $AB tests/test_acf_robust.py tests/test_parity_gpu.py -k "product or returns or short or autocorr or acf" > $O/pair_pytest2.log 2>&1 || { tail -40 $O/pair_pytest2.log; exit 1; }
    tail -1 $O/pair_pytest2.log
    # forms: 0 / 1 = STS_SHORT_PAIR on the A/B build; any other name = build/var_<name> (tools/variant.sh
    # with -DSTS_AB) under STS_SHORT_PAIR=1
    for rep in 1 2 3; do
      for P in 0 1 $PAIR_VARS; do
        L=$AB; PP=$P
        case $P in 0|1) ;; *) L=spark-timeseries_amd/build/var_$P/libsts_hip.so; PP=1 ;; esac
        for w in c1 ${PAIR_WL-c1_rule3}; do
          STS_SHORT_PAIR=$PP STS_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 2 > $O/pair_${w}_$P.json 2>/dev/null || exit 1
          python -c "import json; d=json.load(open('$O/pair_${w}_$P.json')); r=d['roofline']; print(json.dumps({'workload': '$w', 'form': '$P', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'ms_per_step': d['ms_per_step'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/pair.jsonl
        done
      done
    done
    ;;
  c1sq)
    # SQ counters of the C1 short kernel, both forms (STS_SHORT_PAIR on the A/B build), two passes each
    AB=spark-timeseries_amd/build/libsts_hip_ab.so
    export TMPDIR=/tmp
    for P in 0 1; do
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
                 "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        STS_SHORT_PAIR=$P STS_HIP_LIB=$AB timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/c1sq_${P}_$i -o run --output-format csv -- \
            python -u bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline > $O/c1sq_${P}_$i.out 2>&1 || { tail -5 $O/c1sq_${P}_$i.out; exit 1; }
      done
    done
    python tools/c1_sq.py $O/c1_sq.json $O
    ;;
  trim)
    # C1: the one-wave short kernel with fewer VALU per series (STS_SHORT_TRIM, product) against
    # var_notrim (-DSTS_SHORT_TRIM=0); the short-kernel parity first
    timeout -k 10 900 $PYT tests/test_parity_gpu.py -k "short or fused or both_kernels or c1" > $O/trim_pytest.log 2>&1 || { tail -40 $O/trim_pytest.log; exit 1; }
    tail -1 $O/trim_pytest.log
    timeout -k 10 900 $PYT tests/test_acf_robust.py -k "product or returns or short" > $O/trim_pytest2.log 2>&1 || { tail -40 $O/trim_pytest2.log; exit 1; }
    tail -1 $O/trim_pytest2.log
    V=spark-timeseries_amd/build/var_notrim/libsts_hip.so
    for rep in 1 2 3; do
      for L in trim notrim; do
        if [ $L = notrim ]; then E="STS_HIP_LIB=$V"; else E=""; fi
        env $E timeout -k 10 200 python -u bench.py --workload c1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/trim_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/trim_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/trim.jsonl
      done
    done
    ;;
  dpp)
    # DPP moves without an old value (bound_ctrl): the whole GPU suite, then same-box A/B of the
    # product against var_head (the previous tree) on the workloads whose kernels use the helpers
    timeout -k 10 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > $O/dpp_pytest.log 2>&1 || { tail -40 $O/dpp_pytest.log; exit 1; }
    tail -1 $O/dpp_pytest.log
    for rep in 1 2 3; do
      for w in ${DPP_WL:-c1 c2 c4}; do
        for L in new ${DPP_LIBS:-head}; do
          if [ $L = new ]; then E=""; else E="STS_HIP_LIB=spark-timeseries_amd/build/var_$L/libsts_hip.so"; fi
          env $E timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 2 > $O/dpp_${w}_$L.json 2>/dev/null || exit 1
          python -c "import json; d=json.load(open('$O/dpp_${w}_$L.json')); r=d['roofline']; print(json.dumps({'workload': '$w', 'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/dpp.jsonl
        done
      done
    done
    ;;
  splds)
    # fill("spline") with the rows and the (mu, z) scratch through LDS (STS_SPLINE_LDS, product) against
    # var_splold (-DSTS_SPLINE_LDS=0); the spline tests first
    timeout -k 10 900 $PYT tests/test_spline.py tests/test_fuzz_gpu.py tests/test_parity_gpu.py -k "spline or unsupported or fill_diff_ewma" > $O/splds_pytest.log 2>&1 || { tail -40 $O/splds_pytest.log; exit 1; }
    tail -1 $O/splds_pytest.log
    V=spark-timeseries_amd/build/var_splold/libsts_hip.so
    for rep in 1 2 3; do
      for L in lds old; do
        if [ $L = old ]; then E="STS_HIP_LIB=$V"; else E=""; fi
        env $E timeout -k 10 300 python -u bench.py --workload spline --steps 5 --warmup 2 --cpu-seconds 2 > $O/splds_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/splds_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/splds.jsonl
      done
    done
    ;;
  splsq)
    # SQ counters of the spline kernel (one pass of 8 SQ counters)
    export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        -d $O/splsq_1 -o run --output-format csv -- python -u bench.py --workload spline --steps 1 --warmup 0 --no-cpu-baseline > $O/splsq_1.out 2>&1 || { tail -5 $O/splsq_1.out; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE \
        -d $O/splsq_2 -o run --output-format csv -- python -u bench.py --workload spline --steps 1 --warmup 0 --no-cpu-baseline > $O/splsq_2.out 2>&1 || { tail -5 $O/splsq_2.out; exit 1; }
    python - <<'PY'
import csv, glob, collections, json
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6/splsq_*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "spline" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"]); per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for c in per.values():
        for k, v in c.items():
            d[k].append(v)
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(d.items())}, indent=1))
PY
    ;;
  overlap)
    # the fill's HBM stream and the lag products' FP64 MFMAs from different waves: alone and together
    timeout -k 10 120 ./tools/ubench_overlap 8 4 12288 2048 > $O/overlap.jsonl && cat $O/overlap.jsonl
    timeout -k 10 120 ./tools/ubench_overlap 8 4 12288 512 > $O/overlap_fewB.jsonl && cat $O/overlap_fewB.jsonl
    ;;
  overlap2)
    # the C3 proportions: an HBM stream of ~20 ms beside MFMA work of ~15-20 ms, MFMA from 2 / 4 waves per SIMD
    timeout -k 10 200 ./tools/ubench_overlap 8 8 49152 512 > $O/overlap2_w2.jsonl && cat $O/overlap2_w2.jsonl
    timeout -k 10 200 ./tools/ubench_overlap 8 8 24576 1024 > $O/overlap2_w4.jsonl && cat $O/overlap2_w4.jsonl
    ;;
  overlap3)
    # the same with the MFMA waves' shader clock recorded (s_memtime against the 100-MHz wall clock)
    timeout -k 10 200 ./tools/ubench_overlap 8 8 49152 512 > $O/overlap3_w2.jsonl && cat $O/overlap3_w2.jsonl
    timeout -k 10 200 ./tools/ubench_overlap 8 8 24576 1024 > $O/overlap3_w4.jsonl && cat $O/overlap3_w4.jsonl
    timeout -k 10 200 ./tools/ubench_overlap 8 8 12288 2048 > $O/overlap3_w8.jsonl && cat $O/overlap3_w8.jsonl
    ;;
  overlap4)
    # launch order swapped (the copy's waves resident first), and a lighter MFMA load
    timeout -k 10 200 ./tools/ubench_overlap 8 8 49152 512 1 > $O/overlap4_w2_copyfirst.jsonl && cat $O/overlap4_w2_copyfirst.jsonl
    timeout -k 10 200 ./tools/ubench_overlap 8 8 12288 512 1 > $O/overlap4_w2_light_copyfirst.jsonl && cat $O/overlap4_w2_light_copyfirst.jsonl
    ;;
  ew)
    # EWMA.fitModel with 64 series per wave in 32-step chunks (var_ew6432) against the product's 32 x 64;
    # the EWMA parity first, on the variant
    V=spark-timeseries_amd/build/var_ew6432/libsts_hip.so
    timeout -k 10 900 $PYT --sts-lib $V tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_ewma_state_machine.py -k "ewma or EWMA" > $O/ew_pytest.log 2>&1 || { tail -40 $O/ew_pytest.log; exit 1; }
    tail -1 $O/ew_pytest.log
    for rep in 1 2 3; do
      for L in prod ew6432; do
        if [ $L = prod ]; then E=""; else E="STS_HIP_LIB=$V"; fi
        env $E timeout -k 10 200 python -u bench.py --workload ewma_fit --steps 5 --warmup 2 --cpu-seconds 2 > $O/ew_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/ew_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/ew.jsonl
      done
    done
    ;;
  c3sleep)
    # C3: the MFMA phase with an s_sleep after each chunk's MFMAs (lower MFMA duty per wave) against the product
    for rep in 1 2 3; do
      for L in prod ${C3_VARS:-sleep1 sleep2}; do
        if [ $L = prod ]; then E=""; else E="STS_HIP_LIB=spark-timeseries_amd/build/var_$L/libsts_hip.so"; fi
        env $E timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > $O/c3s_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/c3s_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac']}))" | tee -a $O/c3s.jsonl
      done
    done
    ;;
  compact)
    # C1: the fill's in-block runs as one wave-wide list (var_compact, -DSTS_SHORT_COMPACT=1) against the product
    V=spark-timeseries_amd/build/var_compact/libsts_hip.so
    timeout -k 10 900 $PYT --sts-lib $V tests/test_parity_gpu.py tests/test_acf_robust.py tests/test_fuzz_gpu.py -k "short or fused or autocorr or acf or fill" > $O/compact_pytest.log 2>&1 || { tail -40 $O/compact_pytest.log; exit 1; }
    tail -1 $O/compact_pytest.log
    for rep in 1 2 3; do
      for L in prod compact; do
        if [ $L = prod ]; then E=""; else E="STS_HIP_LIB=$V"; fi
        env $E timeout -k 10 200 python -u bench.py --workload c1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/compact_$L.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/compact_$L.json')); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'frac': r['frac'], 'check': d['cpu_baseline']['sample_check']}))" | tee -a $O/compact.jsonl
      done
    done
    ;;
  splsq2)
    # the spline kernel's waiting time: instruction fetch and the I-cache
    export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY \
        -d $O/splsq2_1 -o run --output-format csv -- python -u bench.py --workload spline --steps 1 --warmup 0 --no-cpu-baseline > $O/splsq2_1.out 2>&1 || { tail -5 $O/splsq2_1.out; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ GRBM_GUI_ACTIVE \
        -d $O/splsq2_2 -o run --output-format csv -- python -u bench.py --workload spline --steps 1 --warmup 0 --no-cpu-baseline > $O/splsq2_2.out 2>&1 || { tail -5 $O/splsq2_2.out; exit 1; }
    python - <<'PY'
import csv, glob, collections, json
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6/splsq2_*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "spline" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"]); per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for c in per.values():
        for k, v in c.items():
            d[k].append(v)
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(d.items())}, indent=1))
PY
    ;;
  *)
    echo "unknown session $SESSION"; exit 2 ;;
esac
