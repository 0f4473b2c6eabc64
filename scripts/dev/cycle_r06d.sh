#!/bin/bash
# r06d: soft-forward stamps on the current kernel (where the heavy items spend their cycles), the
# _C soft mask leg (padding-first wide stores) against the r05 build, kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r06d; mkdir -p $OUT
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so STAMPS_DUMP=$R/$OUT/stamps.npy timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
cat $OUT/stamps.log
STAMPS_PARAMS=0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1 KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_p30.log 2>&1 || { tail -20 $OUT/stamps_p30.log; exit 1; }
head -12 $OUT/stamps_p30.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "soft or dibr" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cat > $OUT/csm.py <<'PY'
import sys, torch
sys.path.insert(0, '.')
import bench
inp = bench.dibr_inputs(bench.views_for_rank(0, 1, 4), torch.device('cuda'), 512, 512)
inp['stats'] = bench.workload_stats(inp)
for _ in range(3):
    print(bench.soft_mask_c_leg(inp, 10))
PY
timeout -k 10 120 python $OUT/csm.py > $OUT/csm_new.log 2>&1
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/scripts/dev/_bin/r05lib/libkaolin_hip.so timeout -k 10 120 python $OUT/csm.py > $OUT/csm_r05.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 30 0 1 0 1 >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/r05lib/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 | sed 's/^/r05 /' >> $OUT/ab.txt 2>&1
done
for i in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 31 0 1 0 1 | sed 's/^/g2 /' >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/g2mw4/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 | sed 's/^/g2mw4 /' >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/g2b2/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 | sed 's/^/g2b2 /' >> $OUT/ab.txt 2>&1
done
grep params $OUT/ab.txt
echo new; cut -c1-200 $OUT/csm_new.log | grep -o "'ms': [0-9.]*\|'frac': [0-9.]*"
echo r05; cut -c1-200 $OUT/csm_r05.log | grep -o "'ms': [0-9.]*\|'frac': [0-9.]*"
