#!/bin/bash
# r05ak: p2m's per-chunk threshold maximum by DPP (wave_max_all) and the transpose's xor-4 stage by DPP, against devlib/head:
# distance GPU tests, then p2m_ab alternated between the builds
set -e
R=$(pwd); OUT=gpurun_out/r05ak; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "p2m or distance or point_to_mesh or sided or sharding" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
for k in 1 2 3; do
  timeout -k 10 200 python scripts/dev/p2m_ab.py 11=0 11=0 > $OUT/p2m_new_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 200 python scripts/dev/p2m_ab.py 11=0 11=0 > $OUT/p2m_head_$k.txt 2>&1
done
grep -H "ms" $OUT/p2m_*.txt | grep -v amdgpu
# + the transpose's xor-4 stage by DPP (tilewalk.h) against ds_swizzle: DIB-R tests and fwd/bwd
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "dibr or soft or raster" --timeout 120 --timeout-method thread > $OUT/tests_dibr.log 2>&1
tail -1 $OUT/tests_dibr.log
for k in 1 2 3; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_new_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_head_$k.txt 2>&1
done
grep -H dibr $OUT/ab_*.txt
