#!/bin/bash
# p2m A/B: staged-reciprocal division (default build) against the IEEE division build (scripts/dev/p2mlib)
set -e
OUT=gpurun_out/r04au; mkdir -p $OUT; R=$(pwd)
for k in 1 2 3; do
  timeout -k 10 120 python scripts/dev/p2m_ab.py 11=0 > $OUT/qdiv_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/p2mlib/libkaolin_hip.so timeout -k 10 120 python scripts/dev/p2m_ab.py 11=0 > $OUT/ieee_$k.txt 2>&1
done
