#!/bin/bash
# stamps of the soft forward under several dev flag settings (STAMP_FLAGS list)
set -e
R=$(pwd)
mkdir -p gpurun_out
for f in ${STAMP_FLAGS:-0}; do
  STAMPS_FLAGS=$f KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so STAMPS_DUMP=$R/gpurun_out/stamps_$f.npy timeout -k 10 120 python scripts/dev/stamps.py > gpurun_out/stamps_$f.log 2>&1
done
