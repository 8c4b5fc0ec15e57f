#!/bin/bash
# Build an A/B variant of libsts_hip.so: tools/variant.sh NAME 'sed-expr' [file] [extra hipcc flags]
# (VARIANT_SRC=path: replace FILE by that source first)
# -> spark-timeseries_amd/build/var_NAME/libsts_hip.so (select with STS_HIP_LIB=...).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXPR=$2; FILE=${3:-sts_tile.hip}; XFLAGS=$4
W=/tmp/var_$NAME; rm -rf $W; mkdir -p $W; cp -r $ROOT/spark-timeseries_amd/csrc $W/
[ -n "$VARIANT_SRC" ] && cp "$VARIANT_SRC" $W/csrc/$FILE   # a whole replacement source for FILE
[ -n "$EXPR" ] && sed -i "$EXPR" $W/csrc/$FILE
if [ -n "$EXPR" ] && cmp -s $W/csrc/$FILE $ROOT/spark-timeseries_amd/csrc/$FILE; then echo "variant $NAME: sed changed nothing" >&2; exit 1; fi
cd $W/csrc
rm -f $W/*.o
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $XFLAGS -I$ROOT/include -I. -c $f -o $W/$f.o &
done
wait
for f in *.hip *.cpp; do [ -f $W/$f.o ] || { echo "variant $NAME: $f did not compile" >&2; exit 1; }; done
mkdir -p $ROOT/spark-timeseries_amd/build/var_$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/spark-timeseries_amd/build/var_$NAME/libsts_hip.so $W/*.o
echo "built var_$NAME"
