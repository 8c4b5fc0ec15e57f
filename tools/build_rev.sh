#!/bin/bash
# Build libsts_hip.so from the csrc/ of a git revision, for same-box A/B against HEAD:
#   tools/build_rev.sh REV NAME -> spark-timeseries_amd/build/var_NAME/libsts_hip.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2; XFLAGS=$3
W=/tmp/rev_$NAME; rm -rf $W; mkdir -p $W
git -C $ROOT archive $REV spark-timeseries_amd/csrc include | tar -x -C $W
cd $W/spark-timeseries_amd/csrc
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $XFLAGS -I$W/include -I. -c $f -o $W/$f.o &
done
wait
mkdir -p $ROOT/spark-timeseries_amd/build/var_$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/spark-timeseries_amd/build/var_$NAME/libsts_hip.so $W/*.o
echo "built var_$NAME from $REV"
