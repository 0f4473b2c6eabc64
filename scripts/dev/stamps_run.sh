#!/bin/bash
# soft-forward stamps with the STAMPS=1 library built into scripts/dev/stamplib (make OUT=...)
set -e
R=$(pwd)
OUT=${OUT:-gpurun_out/stamps}
mkdir -p $OUT
for f in ${STAMP_FLAGS:-0}; do
  STAMPS_FLAGS=$f KAOLIN_HIP_LIB=$R/scripts/dev/stamplib/libkaolin_hip.so STAMPS_DUMP=$R/$OUT/stamps_$f.npy \
    timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_$f.log 2>&1
done
