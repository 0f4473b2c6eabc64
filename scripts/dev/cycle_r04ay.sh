#!/bin/bash
# raster_tile_kernel forced to 8 waves per SIMD (64 VGPRs, 20 spilled; build in scripts/dev/vlib_wpe)
set -e
OUT=gpurun_out/r04ay; mkdir -p $OUT; R=$(pwd)
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/base_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/vlib_wpe/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/wpe_$k.txt 2>&1
done
