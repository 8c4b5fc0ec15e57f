#!/bin/bash
# Round-4 GPU evidence sessions, one per case: `bash tools/sessions_r4.sh s21` re-runs what the
# round-4 rows of profiles/INDEX.md name as session s21 (formerly tools/r4_s21.sh).  Each session
# keeps its own time limits and stops at its first failure.  New sessions use tools/r5_session.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case "$1" in
  s3)
    # Round-4 session 3: the C2 rows kernel (v2) against the round-3 tree, C5 run-to-run drift (three
    # consecutive runs per library), and the C3 kernel's sensitivity to the NaN rate (how much of the
    # fused time the imputation phases hold).  The first failure ends the session.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 200 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 \
        --timeout-method thread -p no:cacheprovider --sts-lib spark-timeseries_amd/build/var_rows/libsts_hip.so > gpurun_out/pytest_rows.log 2>&1
    bash tools/ab_bench.sh c2 base rows r3 > gpurun_out/ab_c2.jsonl
    for L in base r3; do
      P=spark-timeseries_amd/build/libsts_hip.so; [ $L != base ] && P=spark-timeseries_amd/build/var_$L/libsts_hip.so
      for rep in 1 2 3; do
        STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
          | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/c5_drift.jsonl
      done
    done
    for NAN in 0.0 0.05 0.3; do
      timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --nan $NAN --cases tile:linear:60,tile:linear:0 \
        | sed "s/^{/{\"nan\": $NAN, /" >> gpurun_out/kb_nan.jsonl
    done
    ;;
  s4)
    # Round-4 session 4: the per-wave scan variant (WSCAN) parity + C3 A/B; C2 stride fix; C5 store forms.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        --sts-lib spark-timeseries_amd/build/var_wscan/libsts_hip.so > gpurun_out/pytest_wscan.log 2>&1
    for rep in 1 2; do
      for V in base wscan; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        for NAN in 0.05 0.3; do
          STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --nan $NAN \
              --cases tile:linear:60,tile:linear:0 | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, \"nan\": $NAN, /" >> gpurun_out/kb_wscan.jsonl
        done
      done
    done
    bash tools/ab_bench.sh c2 base ch128 r3 > gpurun_out/ab_c2.jsonl
    for rep in 1 2 3; do
      for L in base c5plain r3; do
        P=spark-timeseries_amd/build/libsts_hip.so; [ $L != base ] && P=spark-timeseries_amd/build/var_$L/libsts_hip.so
        STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
          | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/c5_forms.jsonl
      done
    done
    for rep in 1 2; do
      for V in base wscanab; do
        L=spark-timeseries_amd/build/libsts_hip.so; E=""; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so && E="STS_TILE_W=2048"
        env $E STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_wscan2w.jsonl
      done
    done
    ;;
  s5)
    # Round-4 session 5: the fill method as a template parameter (+ the SGPR-spill cut of 7b06d88)
    # against 7b06d88 (var_s5) and the round-3 tree (var_r3) on C3 / C2 / C5, and SQ counters of the
    # product and the measured-negative variants (LDS-DMA 2048-step tiles, per-wave scans).
    mkdir -p gpurun_out
    set -e
    for rep in 1 2; do
      for V in base s5 r3; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60,tile:linear:0 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_s5.jsonl
      done
    done
    bash tools/ab_bench.sh c5 base r3 > gpurun_out/ab_c5.jsonl
    bash tools/ab_bench.sh c2 base r3 > gpurun_out/ab_c2.jsonl
    for V in base r3 dma wscan; do
      L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
      bash tools/r3_sqcases.sh tile:linear:60,tile:linear:0 $L _$V
    done
    ;;
  s6)
    # Round-4 session 6: early raw stores from the prefetch registers (STS_EARLY_ST) -- parity, C3
    # kernel A/B (fill + ACF, fill only), C5 A/B.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        --sts-lib spark-timeseries_amd/build/var_est/libsts_hip.so > gpurun_out/pytest_est.log 2>&1
    for rep in 1 2; do
      for V in base est; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60,tile:linear:0 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_est.jsonl
      done
    done
    bash tools/ab_bench.sh c5 base est > gpurun_out/ab_c5_est.jsonl
    ;;
  s7)
    # Round-4 session 7: the AR(p) Gram's lag products on FP64 MFMA inside the C4 register kernel
    # (STS_AR_MFMA variant) -- AR parity, C4 A/B, FP64 / MFMA counters of the variant; s_setprio
    # around the C3 MFMA phase (var_prio_m) or the fill phase (var_prio_f) -- C3 kernel A/B.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "ar_ or arima" --sts-lib spark-timeseries_amd/build/var_ar_mfma/libsts_hip.so > gpurun_out/pytest_ar_mfma.log 2>&1
    bash tools/ab_bench.sh c4 base ar_mfma > gpurun_out/ab_c4_ar_mfma.jsonl
    STS_HIP_LIB=spark-timeseries_amd/build/var_ar_mfma/libsts_hip.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/pmc_c4_ar_mfma -o bench --output-format csv -- python -u bench.py --workload c4 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c4_ar_mfma.log 2>&1
    for rep in 1 2; do
      for V in base prio_m prio_f; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio.jsonl
      done
    done
    ;;
  s8)
    # Round-4 session 8 (second call: prio_0 = no priority change, same box as base and prio_s): wave priority around the C3 MFMA phase -- the product (STS_FILL_PRIO=2) on
    # the full GPU suite, then C3 kernel A/B against priority 1 / 3 and against raising it from the
    # first tile on (prio_s), three alternating rounds.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tile or acf or fill" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_prio.log 2>&1
    for rep in 1 2 3; do
      for V in prio_0 base prio_s; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio3.jsonl
      done
    done
    ;;
  s9)
    # Round-4 session 9: phase-graded wave priorities in the C3 tile kernel (priority 3 for wave 0's
    # word scan (pscan), the imputation (pimp), both (pscanimp), or the store pass (pstore); 2
    # elsewhere, 0 in the MFMA phase) against the product, three alternating rounds.
    mkdir -p gpurun_out
    set -e
    for rep in 1 2 3; do
      for V in base pscan pimp pscanimp pstore; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio4.jsonl
      done
    done
    ;;
  s10)
    # Round-4 session 10: recur_row_kernel (one wave per series, affine-scan guess verified lane by
    # lane) -- recurrence parity, then C2 A/B against the 16 x 128 chunk kernel (var_chunk), and the
    # C3 priority-in-scan A/B (pscan / pscanimp) once more.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "recur or ewma or fill_diff" > gpurun_out/pytest_rowscan.log 2>&1
    bash tools/ab_bench.sh c2 base chunk > gpurun_out/ab_c2_rowscan.jsonl
    for rep in 1 2; do
      for V in base pscan pscanimp; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
            | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_prio5.jsonl
      done
    done
    ;;
  s11)
    # Round-4 session 11: recur_row_kernel with 16 lanes per series (4 series per wave, lane blocks of
    # B = 26 steps for C2), rows through a per-wave LDS span (IO) or direct (noio) -- recurrence parity, then C2 A/B against the chunk kernel.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "recur or ewma or fill_diff" > gpurun_out/pytest_rowscan3.log 2>&1
    bash tools/ab_bench.sh c2 base noio chunk > gpurun_out/ab_c2_rowscan3.jsonl
    ;;
  s12)
    # Round-4 session 12: the tree with the C2 row kernel and the C3 scan priority -- full GPU suite,
    # C2 bench + rocprof stats + FETCH / WRITE passes, C3 bench + rocprof stats; then the wave-0
    # scan priority for the fill-only (C5) instantiation as an A/B variant.
    STEPS="tests c2 prof_c2 fetch_c2 write_c2 c3 prof" bash tools/gpu_all.sh || exit 1
    bash tools/ab_bench.sh c5 base c5prio > gpurun_out/ab_c5_prio.jsonl
    ;;
  s13)
    # Round-4 session 13: recur_row_kernel with 32 lanes per series (2 series per wave, B = 14 for C2,
    # 5 workgroups per CU) -- its recurrence parity, C2 A/B against the 16-lane product, and the SQ
    # counters of the product's C2 kernel.
    mkdir -p gpurun_out
    export TMPDIR=/tmp
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "recur or ewma or fill_diff" --sts-lib spark-timeseries_amd/build/var_lps32/libsts_hip.so > gpurun_out/pytest_lps32.log 2>&1
    bash tools/ab_bench.sh c2 base lps32 > gpurun_out/ab_c2_lps32.jsonl
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        -d gpurun_out/c2sq_row -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_row.log 2>&1
    ;;
  s14)
    # Round-4 session 14: lanes per series in recur_row_kernel -- parity of the 32- and 64-lane forms
    # and C2 A/B of 16 (product) / 32 / 64 lanes, two alternating rounds.
    mkdir -p gpurun_out
    set -e
    for V in lps32 lps64; do
      timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
          -k "recur or ewma or fill_diff" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
    done
    bash tools/ab_bench.sh c2 base lps32 lps64 > gpurun_out/ab_c2_lps.jsonl
    ;;
  s15)
    # Round-4 session 15: recur_row_kernel launch shape on C2 -- 1 / 2 / 4 (product) waves per
    # workgroup, XCD-contiguous span ranges; parity of the 1-wave form.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "fill_diff or ewma or row_scan" --sts-lib spark-timeseries_amd/build/var_wpg1/libsts_hip.so > gpurun_out/pytest_wpg1.log 2>&1
    bash tools/ab_bench.sh c2 base wpg1 wpg2 xcd > gpurun_out/ab_c2_shape.jsonl
    ;;
  s16)
    # Round-4 session 16: XCD-contiguous workgroup ranges -- the row kernel's product (remap on) on
    # the recurrence tests and against noxcd on C2; the same remap as variants of the C1 short kernel
    # and the C4 AR kernel (parity, then A/B).
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_xcd_recur.log 2>&1
    timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_short_xcd/libsts_hip.so > gpurun_out/pytest_short_xcd.log 2>&1
    timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "ar_" --sts-lib spark-timeseries_amd/build/var_ar_xcd/libsts_hip.so > gpurun_out/pytest_ar_xcd.log 2>&1
    bash tools/ab_bench.sh c2 base noxcd > gpurun_out/ab_c2_xcd.jsonl
    bash tools/ab_bench.sh c1 base short_xcd > gpurun_out/ab_c1_xcd.jsonl
    bash tools/ab_bench.sh c4 base ar_xcd > gpurun_out/ab_c4_xcd.jsonl
    ;;
  s17)
    # Round-4 session 17: with XCD-contiguous spans, lanes per series (16 / 32 product / 64) and
    # 2-wave workgroups once more on C2; the product's recurrence tests.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s17.log 2>&1
    bash tools/ab_bench.sh c2 base l16 l64 w2 > gpurun_out/ab_c2_s17.jsonl
    ;;
  s18)
    # Round-4 session 18: wave priorities in the C4 AR kernel (remove + store phase at 2) and the C1
    # short kernel (stores, or fill + stores, at 2; the ACF at 0) -- parity, then same-box A/B.
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "ar_" --sts-lib spark-timeseries_amd/build/var_ar_prio/libsts_hip.so > gpurun_out/pytest_ar_prio.log 2>&1
    for V in sh_prio_st sh_prio_fill; do
      timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
          -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
    done
    bash tools/ab_bench.sh c4 base ar_prio > gpurun_out/ab_c4_prio.jsonl
    bash tools/ab_bench.sh c1 base sh_prio_st sh_prio_fill > gpurun_out/ab_c1_prio.jsonl
    ;;
  s19)
    # Round-4 session 19: tiles per tile-kernel workgroup for the fill-only + lag-matrix instantiation
    # (C5) through the A/B build's STS_TILES_PER_CHUNK knob, two alternating rounds.
    mkdir -p gpurun_out
    bash tools/ab_bench.sh c5 ab:STS_TILES_PER_CHUNK=16 ab:STS_TILES_PER_CHUNK=2 ab:STS_TILES_PER_CHUNK=1 ab:STS_TILES_PER_CHUNK=4 > gpurun_out/ab_c5_tpc.jsonl
    ;;
  s20)
    # Round-4 session 20: C5 tiles per workgroup 1 vs 16 (A/B build knob), alternating three times,
    # after one warm-up C5 process (the first C5 process on a box runs fast).
    mkdir -p gpurun_out
    STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip.so timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
    for rep in 1 2 3; do
      for L in ab:STS_TILES_PER_CHUNK=1 ab:STS_TILES_PER_CHUNK=16 base; do
        E=""; P=spark-timeseries_amd/build/libsts_hip.so
        case $L in ab:*) P=spark-timeseries_amd/build/libsts_hip_ab.so; E=${L#ab:} ;; esac
        env $E STS_HIP_LIB=$P timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null \
          | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'lib': '$L', 'rep': $rep, 'workload': 'c5', 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved']}))" >> gpurun_out/ab_c5_tpc2.jsonl || exit 1
      done
    done
    ;;
  s21)
    # Round-4 session 21: one tile per workgroup for the fill-only / lag-matrix tile launches -- full
    # GPU suite, C5 bench (four processes) with rocprof stats, fill-only kbench on the C3 shard.
    STEPS="tests c5 prof_c5" bash tools/gpu_all.sh || exit 1
    for rep in 1 2 3; do
      timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
        | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs4.jsonl || exit 1
    done
    timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:0,tile:nearest:0 > gpurun_out/kb_fill_tpc1.jsonl
    ;;
  s22)
    # Round-4 session 22: tiles per tile-kernel workgroup for fill + ACF(60) on the C3 shard (A/B
    # build knob): 8 / 12 / 16 (product) / 24 / 32, two alternating rounds through tools/kbench.py.
    mkdir -p gpurun_out
    for rep in 1 2; do
      for N in 16 8 12 24 32; do
        STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 200 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
          | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> gpurun_out/kb_c3_tpc.jsonl || exit 1
      done
    done
    ;;
  s23)
    # Round-4 session 23: the row kernel's direct-access form on odd T (new test).
    mkdir -p gpurun_out
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s23.log 2>&1
    ;;
  s24)
    # Round-4 session 24: non-temporal 16-B stores for the C2 row kernel's span output (var_ntc2).
    mkdir -p gpurun_out
    set -e
    timeout -k 10 300 python -u -m pytest tests/test_recur_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        -k "fill_diff or row_scan" --sts-lib spark-timeseries_amd/build/var_ntc2/libsts_hip.so > gpurun_out/pytest_ntc2.log 2>&1
    bash tools/ab_bench.sh c2 base ntc2 > gpurun_out/ab_c2_nt.jsonl
    bash tools/ab_bench.sh c2 base ntc2 >> gpurun_out/ab_c2_nt.jsonl
    ;;
  ab)
    # Round-4 A/B session steps (after tools/gpu_all.sh's own steps): variant parity, kernel-level
    # C3 A/B of the product and the LDS-DMA variant on the full C3 shard, C2 / C5 against the
    # round-3 tree, phase stamps.  Every GPU step has its own limit; the first failure ends it.
    mkdir -p gpurun_out
    set -e
    for V in ${VARS:-dma}; do
      timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
          --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > gpurun_out/pytest_$V.log 2>&1
    done
    for rep in 1 2; do
      for V in base ${VARS:-dma}; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --series ${KB_SERIES:-12500} --reps 3 \
            --cases ${KB_CASES:-tile:linear:60,tile:linear:0} | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> gpurun_out/kb_c3.jsonl
      done
    done
    [ -n "$NO_C2C5" ] || bash tools/ab_bench.sh c2 base r3 > gpurun_out/ab_c2.jsonl
    [ -n "$NO_C2C5" ] || bash tools/ab_bench.sh c5 base r3 > gpurun_out/ab_c5.jsonl
    STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_stamps.so timeout -k 10 120 python tools/stamps.py 2000 60 0 > gpurun_out/stamps.json
    ;;
  c2sq)
    # SQ counters of the C2 pipeline for the product (recur_kernel, 16 series x 128-step chunks) and
    # the measured-negative whole-row variant (rows_kernel, built from 7b06d88 with -DSTS_ROWS).
    export TMPDIR=/tmp
    mkdir -p gpurun_out
    for V in base rows; do
      L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
      STS_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        -d gpurun_out/c2sq_$V -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_$V.log 2>&1 || exit 1
    done
    ;;
  combo)
    # Round-4 closing session: the C2 shape A/B with XCD remap on (tools/r4_s17.sh), then the
    # final-tree evidence (tools/r4_final3.sh).
    bash tools/sessions_r4.sh s17 || exit 1
    bash tools/sessions_r4.sh final3
    ;;
  final)
    # Round-4 final-tree evidence: GPU tests, every workload's bench line, rocprof stats of the C3
    # and C5 bench commands, C3 HBM traffic and FP64 counters, C5 three consecutive runs, smoke.
    mkdir -p gpurun_out
    STEPS="tests c3 prof fetch write fp64_c3 c1 c2 c4 c5 prof_c5" bash tools/gpu_all.sh || exit $?
    set -e
    for rep in 1 2 3; do
      timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep metric \
        | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs.jsonl
    done
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    ;;
  final2)
    # Round-4 final-tree evidence (second set, after the C2 row kernel and the C3 priorities): full GPU
    # suite, every workload's bench line, rocprof stats of C3 / C2 / C5, FETCH / WRITE of C3 and C2,
    # FP64 counters of C3, three more C5 processes, smoke().
    STEPS="tests c3 prof fetch write fp64_c3 c2 prof_c2 fetch_c2 write_c2 c1 c4 c5 prof_c5" bash tools/gpu_all.sh || exit 1
    for rep in 1 2 3; do
      timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
        | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs2.jsonl || exit 1
    done
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1
    ;;
  final3)
    # Round-4 final-tree evidence (third set: C2 row kernel with XCD-contiguous spans, C4 XCD remap): full GPU
    # suite, every workload's bench line, rocprof stats of C3 / C2 / C5, FETCH / WRITE of C3 and C2,
    # FP64 counters of C3, three more C5 processes, smoke().
    STEPS="tests c3 prof fetch write fp64_c3 c2 prof_c2 fetch_c2 write_c2 c1 c4 c5 prof_c5" bash tools/gpu_all.sh || exit 1
    for rep in 1 2 3; do
      timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
        | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs3.jsonl || exit 1
    done
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        -d gpurun_out/c2sq_final -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_final.log 2>&1
    ;;
  final4)
    # Round-4 final-tree evidence (fourth set: + one tile per workgroup for fill-only / lag-matrix launches): full GPU
    # suite, every workload's bench line, rocprof stats of C3 / C2 / C5, FETCH / WRITE of C3 and C2,
    # FP64 counters of C3, three more C5 processes, smoke().
    STEPS="tests c3 prof fetch write fp64_c3 c2 prof_c2 fetch_c2 write_c2 c1 c4 c5 prof_c5" bash tools/gpu_all.sh || exit 1
    for rep in 1 2 3; do
      timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep metric \
        | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps({'rep': $rep, 'kernel_ms': r['avg_kernel_ms'], 'GBps': r['achieved'], 'frac': r['frac']}))" >> gpurun_out/c5_runs5.jsonl || exit 1
    done
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke5.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        -d gpurun_out/c2sq_final5 -o run --output-format csv -- python -u bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c2sq_final5.log 2>&1
    ;;
  tpc)
    # Tiles per tile-kernel workgroup on the C3 shard (A/B build, STS_TILES_PER_CHUNK), fill only and
    # fill + ACF(60): does a denser sweep of the panel by the resident workgroups (fewer tiles each)
    # move the fill path's memory rate?  Two alternating rounds.
    mkdir -p gpurun_out
    set -e
    for rep in 1 2; do
      for N in ${TPCS:-1 2 4 16 64}; do
        STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 200 python -u tools/kbench.py \
            --series ${KB_SERIES:-12500} --reps 3 --cases ${KB_CASES:-tile:linear:0,tile:linear:60} \
            | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> gpurun_out/kb_tpc.jsonl
      done
    done
    ;;
  *) echo "usage: $0 {s3|s4|s5|s6|s7|s8|s9|s10|s11|s12|s13|s14|s15|s16|s17|s18|s19|s20|s21|s22|s23|s24|ab|c2sq|combo|final|final2|final3|final4|tpc}" >&2; exit 2 ;;
esac
