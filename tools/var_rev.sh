#!/bin/bash
# Build spark-timeseries_amd/build/var_NAME/libsts_hip.so from the csrc/ of git revision REV
# (same-box A/B against an earlier tree): tools/var_rev.sh NAME REV
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2
W=/tmp/varrev_$NAME; rm -rf $W; mkdir -p $W/csrc $W/include
git -C $ROOT archive $REV spark-timeseries_amd/csrc include | tar -x -C $W
cd $W/spark-timeseries_amd/csrc
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$W/include -I. -c $f -o $W/$f.o 2>/dev/null &
done
wait
mkdir -p $ROOT/spark-timeseries_amd/build/var_$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/spark-timeseries_amd/build/var_$NAME/libsts_hip.so $W/*.o
echo "built var_$NAME from $REV"
