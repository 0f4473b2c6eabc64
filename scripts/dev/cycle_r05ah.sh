#!/bin/bash
# r05ah: per-wave stamps of the tile rasterizer and the soft forward on this build (devlib/stamps)
set -e
R=$(pwd); OUT=gpurun_out/r05ah; mkdir -p $OUT
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 200 python scripts/dev/rstamps.py > $OUT/rstamps.log 2>&1
grep -v amdgpu.ids $OUT/rstamps.log | head -40
STAMPS_FLAGS=0 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps.log 2>&1
grep -v amdgpu.ids $OUT/stamps.log | head -30
