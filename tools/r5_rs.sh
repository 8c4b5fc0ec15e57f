#!/bin/bash
# Round-5: the role-split tile kernel (STS_TILE_RS, fill waves + MFMA waves) -- its parity tests on
# the A/B build, then fill + ACF(60) on the C3 shard alternating: product, A/B build with RS = 0 and
# RS = 1, the previous tree (var_head).  The first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
