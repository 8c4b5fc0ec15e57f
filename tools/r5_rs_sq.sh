#!/bin/bash
# Round-5: SQ counters of the tile kernel, shipped form against the role split (fill waves + MFMA
# waves) and its diagnostics, on fill + ACF(60) over 2 000 C3-length series.  One rocprofv3 --pmc
# pass per counter group, each under its own limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
