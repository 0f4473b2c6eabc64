#!/bin/bash
# r05u: branch-free bit-matrix transpose (soft / raster tile walks); hit-list raytrace -- candidate
# tile totals added by the write pass, 8-per-thread offsets scan, tail fill of the fixed entry;
# deftet Morton order off by default: GPU suite, raytrace A/B (dev param 25 = 1: the r05q form) +
# kernel trace; DIB-R fwd/bwd against the r05t transpose build and the soft forward occupancy builds
set -e
R=$(pwd); OUT=gpurun_out/r05u; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
grep -v amdgpu.ids $OUT/rt_ab.log
# soft forward occupancy: ST_EVAL_U=2 (89 VGPRs, 5 waves/SIMD) and + min 6 waves (80 VGPRs), with
# dev param 20 = 2 (2-row items, 24.7 KB of LDS) against the default (4 rows, 39.6 KB: 4 per CU)
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 2 > $OUT/soft_def_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/oldtr/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 > $OUT/soft_oldtr_$k.txt 2>&1
  for v in u2 u2w6; do
    KAOLIN_HIP_LIB=$R/devlib/$v/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 2 > $OUT/soft_${v}_$k.txt 2>&1
  done
done
grep -H dibr $OUT/soft_*.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_dibr -o run -- python3 $R/scripts/dev/param_ab.py 20 0 > $R/$OUT/dibr_prof.log 2>&1
