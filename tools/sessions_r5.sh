#!/bin/bash
# Round-5 GPU sessions, one per case: `bash tools/sessions_r5.sh s20` re-runs what the round-5 rows
# of profiles/INDEX.md name as session s20.  Each keeps its own time limits and stops at its first
# failure.  A/B libraries (build/var_*) are gpurun-ignored: drop that line from .gpurunignore for an
# A/B call.  The parameterised driver is tools/r5_session.sh; the final-tree evidence tools/r5_final.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SESSION=$1; shift
case "$SESSION" in
  c1ab)
    # C1 A/B of the half-block short kernel (var_short2) against the product: parity first (the short
    # kernel's GPU tests bound to the variant), then bench.py --workload c1 alternating libraries.
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
    ;;
  rs)
    # Round-5: the role-split tile kernel (STS_TILE_RS, fill waves + MFMA waves) -- its parity tests on
    # the A/B build, then fill + ACF(60) on the C3 shard alternating: product, A/B build with RS = 0 and
    # RS = 1, the previous tree (var_head).  The first failure ends the session.
    O=${OUT_DIR:-gpurun_out/r5}
    mkdir -p $O
    set -e
    B=spark-timeseries_amd/build
    [ "${RS_PARITY:-1}" = 0 ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
        tests/test_parity_gpu.py -k "tilers or role_split" > $O/rs_parity.log 2>&1
    for rep in 1 2; do
      for V in ${RS_ARMS:-base rs0 rs1 head}; do
        E=""
        case $V in
          base) L=$B/libsts_hip.so ;;
          rs0) L=$B/libsts_hip_ab.so; E="STS_TILE_RS=0" ;;
          rs1) L=$B/libsts_hip_ab.so; E="STS_TILE_RS=1" ;;
          rs1s) L=$B/libsts_hip_ab.so; E="STS_TILE_RS=1 STS_TILES_PER_CHUNK=${RS_TPC:-32}" ;;
          *) L=$B/var_$V/libsts_hip.so ;;
        esac
        env $E STS_HIP_LIB=$L timeout -k 10 300 python -u tools/kbench.py --series ${KB_SERIES:-12500} --reps 3 \
            --cases ${KB_CASES:-tile:linear:60} | grep -v amdgpu.ids | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> $O/rs_ab.jsonl
      done
    done
    ;;
  rs_sq)
    # Round-5: SQ counters of the tile kernel, shipped form against the role split (fill waves + MFMA
    # waves) and its diagnostics, on fill + ACF(60) over 2 000 C3-length series.  One rocprofv3 --pmc
    # pass per counter group, each under its own limit; the first failure ends the session.
    O=${OUT_DIR:-gpurun_out/r5}
    mkdir -p $O
    export TMPDIR=/tmp
    B=spark-timeseries_amd/build
    PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
    PB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"
    for V in ${SQ_ARMS:-base rs1}; do
      unset STS_TILE_RS
      case $V in
        base) export STS_HIP_LIB=$B/libsts_hip.so ;;
        rs1) export STS_HIP_LIB=$B/libsts_hip_ab.so STS_TILE_RS=1 ;;
        *) export STS_HIP_LIB=$B/var_$V/libsts_hip.so ;;
      esac
      for G in A B; do
        [ $G = A ] && P=$PA || P=$PB
        timeout -s KILL 90 rocprofv3 --pmc $P -d $O/sq_${V}_$G -o run --output-format csv -- \
            python -u tools/kbench.py --series 2000 --reps 1 --cases tile:linear:60 > $O/sq_${V}_$G.log 2>&1 || exit 1
      done
    done
    ;;
  s18)
    # Round-5 session 18: RCCL collectives on one GPU (tests/test_rccl_gpu.py); non-temporal prefetch loads in the
    # tile kernel (var_ntl): parity, C3 kernel A/B, C5 bench A/B.
    set -e
    O=gpurun_out/r5; mkdir -p $O
    timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rccl_gpu.py > $O/rccl.log 2>&1
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py -k "tile or fill_acf or c5 or lag" --sts-lib spark-timeseries_amd/build/var_ntl/libsts_hip.so > $O/ntl_parity.log 2>&1
    RS_PARITY=0 RS_ARMS="base ntl" bash tools/sessions_r5.sh rs
    bash tools/ab_bench.sh c5 base ntl > $O/ab_c5_ntl.jsonl
    ;;
  s19)
    # Round-5 session 19: non-temporal prefetch loads (var_ntl) against the product, three more
    # alternating rounds on C3 (kernel A/B) and on C5 (bench, after one warm-up C5 process).
    set -e
    O=gpurun_out/r5; mkdir -p $O
    for rep in 3 4 5; do
      for V in ntl base; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 300 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
          | grep -v amdgpu.ids | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> $O/rs_ab.jsonl
      done
    done
    timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
    bash tools/ab_bench.sh c5 base ntl >> $O/ab_c5_ntl.jsonl
    bash tools/ab_bench.sh c5 ntl base >> $O/ab_c5_ntl.jsonl
    ;;
  s20)
    # Round-5 session 20: cache policy of the staged-series kernels (C1 short kernel, C4 AR kernel, C2
    # row kernel): non-temporal LDS-DMA loads (var_dmant), non-temporal 16-B result stores (var_stnt),
    # both (var_ntboth) -- parity of the short / AR / recurrence rows on ntboth, then bench A/B.
    set -e
    O=gpurun_out/r5; mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py \
        -k "short or fill_acf or ar_ or fill_diff or ewma" --sts-lib spark-timeseries_amd/build/var_ntboth/libsts_hip.so > $O/ntboth_parity.log 2>&1
    for W in c1 c4 c2; do
      bash tools/ab_bench.sh $W base dmant stnt ntboth >> $O/ab_policy.jsonl
    done
    ;;
  s21)
    # Round-5 session 21: C5 with plain instead of non-temporal filled-output stores in the fill-only
    # tile kernel (var_c5plain): parity of the fill / lag rows, then three alternating C5 rounds after one warm-up process.
    set -e
    O=gpurun_out/r5; mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py tests/test_c5_length.py \
        -k "fill or lag or c5" --sts-lib spark-timeseries_amd/build/var_c5plain/libsts_hip.so > $O/c5plain_parity.log 2>&1
    timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
    bash tools/ab_bench.sh c5 base c5plain > $O/ab_c5plain.jsonl
    bash tools/ab_bench.sh c5 c5plain base >> $O/ab_c5plain.jsonl
    ;;
  s22)
    # Round-5 session 22: cache-policy modifiers of the C1 short kernel (result stores: nt = product,
    # sc0 sc1 nt, sc1 nt, sc1; DMA loads: sc1, sc0 sc1) -- parity on two variants, C1 bench A/B.
    set -e
    O=gpurun_out/r5; mkdir -p $O
    for V in st2 ld3; do
      timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py \
          -k "short or fill_acf" --sts-lib spark-timeseries_amd/build/var_$V/libsts_hip.so > $O/pol_parity_$V.log 2>&1
    done
    bash tools/ab_bench.sh c1 base st2 st3 st4 ld2 ld3 > $O/ab_c1_pol.jsonl
    ;;
  s23)
    # Round-5 session 23: timing-only cost models of the C1 short kernel on the final tree
    # (STS_SHORT_DIAG 1 no ACF, 2 no fill, 3 no per-lag finalize, 4 no robust shift, 5 no lag FMAs).
    set -e
    O=gpurun_out/r5; mkdir -p $O
    bash tools/ab_bench.sh c1 base sd1 sd2 sd3 sd4 sd5 > $O/ab_c1_diag.jsonl
    ;;
  s24)
    # Round-5 session 24: tiles per tile-kernel workgroup for fill + ACF(60) on the C3 shard with the
    # non-temporal prefetch loads (A/B build knob STS_TILES_PER_CHUNK): 12 / 16 (product) / 24 / 32, two rounds.
    set -e
    O=gpurun_out/r5; mkdir -p $O
    for rep in 1 2; do
      for N in 16 12 24 32; do
        STS_TILES_PER_CHUNK=$N STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_ab.so timeout -k 10 300 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
          | grep -v amdgpu.ids | sed "s/^{/{\"tpc\": $N, \"rep\": $rep, /" >> $O/kb_c3_tpc_nt.jsonl
      done
    done
    ;;
  s25)
    # Round-5 session 25: the C1 short kernel's finalize with DPP suffix sums (var_c1dpp) -- its parity
    # rows, then C1 bench A/B; and the C3 tiles-per-workgroup sweep with non-temporal loads (tools/r5_s24.sh).
    set -e
    O=gpurun_out/r5; mkdir -p $O
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py tests/test_acf_robust.py \
        -k "short or fill_acf or product or returns" --sts-lib spark-timeseries_amd/build/var_c1dpp/libsts_hip.so > $O/c1dpp_parity.log 2>&1
    bash tools/ab_bench.sh c1 base c1dpp > $O/ab_c1dpp.jsonl
    bash tools/ab_bench.sh c1 c1dpp base >> $O/ab_c1dpp.jsonl
    bash tools/sessions_r5.sh s24
    ;;
  s27)
    # the tile kernel with y formed in registers by the MFMA phase (var_yreg, STS_TILE_YREG=1): parity of
    # the tile / fill + ACF / robust-ACF rows, then C3 kernel A/B, three alternating rounds
    set -e
    O=gpurun_out/r5; mkdir -p $O
    timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_parity_gpu.py tests/test_acf_robust.py \
        -k "tile or fill_acf or autocorr or c3" --sts-lib spark-timeseries_amd/build/var_yreg/libsts_hip.so > $O/yreg_parity.log 2>&1
    for rep in 1 2 3; do
      for V in base yreg; do
        L=spark-timeseries_amd/build/libsts_hip.so; [ $V != base ] && L=spark-timeseries_amd/build/var_$V/libsts_hip.so
        STS_HIP_LIB=$L timeout -k 10 300 python -u tools/kbench.py --series 12500 --reps 3 --cases tile:linear:60 \
          | grep -v amdgpu.ids | sed "s/^{/{\"lib\": \"$V\", \"rep\": $rep, /" >> $O/ab_c3_yreg.jsonl
      done
    done
    ;;
  *) echo "usage: $0 {c1ab|rs|rs_sq|s18|s19|s20|s21|s22|s23|s24|s25|s27}" >&2; exit 2 ;;
esac
