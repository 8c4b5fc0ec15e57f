#!/bin/bash
# Register / scratch / LDS usage of every kernel in one HIP source (build-time check).
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/root/repo/include \
  -I/root/repo/spark-timeseries_amd/csrc -c "$f" -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "error|Function Name|VGPRs:|ScratchSize|LDS Size" |
  sed -E 's/.*remark: +//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' | paste - - - - | cut -c1-200
