#!/bin/bash
# stamps of the soft forward under several dev flag settings (STAMP_FLAGS list)
set -e
R=$(pwd)
mkdir -p gpurun_out
for f in ${STAMP_FLAGS:-0}; do
  STAMPS_FLAGS=$f KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so STAMPS_DUMP=$R/gpurun_out/stamps_$f.npy timeout -k 10 120 python scripts/dev/stamps.py > gpurun_out/stamps_$f.log 2>&1
done
# SoftSplit sweeps: STAMP_PARAMS="b4,b8,cap4,cap8 ..." (one run each)
for p in ${STAMP_PARAMS:-}; do
  STAMPS_PARAMS=$p KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > gpurun_out/stamps_p$p.log 2>&1
done
