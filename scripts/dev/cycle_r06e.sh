#!/bin/bash
# r06e: the _C contract soft mask on the tile path: its tests (product + dev library), then the
# _C leg timed against the row kernel (dev param 30 = 1) and the r05 build
set -e
R=$(pwd); OUT=gpurun_out/r06e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "soft_mask" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "soft or dibr" > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q --timeout 200 --timeout-method thread -k "p2m" > $OUT/tests_p2m.log 2>&1 || { tail -30 $OUT/tests_p2m.log; exit 1; }
tail -2 $OUT/tests_p2m.log
for i in 1 2; do
  timeout -k 10 120 python scripts/dev/p2m_ab.py 11=0 11=5 11=0 11=5 >> $OUT/p2m_ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/p2mw4/libkaolin_hip.so timeout -k 10 120 python scripts/dev/p2m_ab.py 11=0 11=5 | sed 's/^/w4 /' >> $OUT/p2m_ab.txt 2>&1
done
grep params $OUT/p2m_ab.txt
for i in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 31 0 1 2 3 0 1 >> $OUT/prio_ab.txt 2>&1
done
grep params $OUT/prio_ab.txt
cat > $OUT/csm.py <<'PY'
import ctypes, os, sys, torch
sys.path.insert(0, '.')
import bench
from kaolin import _native as N
lib = N.lib()
inp = bench.dibr_inputs(bench.views_for_rank(0, 1, 4), torch.device('cuda'), 512, 512)
inp['stats'] = bench.workload_stats(inp)
for _ in range(2):
    for v in ((0, 1) if hasattr(lib, 'kl_dev_set_param') else (0,)):
        if hasattr(lib, 'kl_dev_set_param'):
            lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
            lib.kl_dev_set_param(30, v)
        r = bench.soft_mask_c_leg(inp, 10)
        print('30=%d' % v, r['ms'], r['roofline']['frac'], flush=True)
PY
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 120 python $OUT/csm.py > $OUT/csm_new.log 2>&1
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/scripts/dev/_bin/r05lib/libkaolin_hip.so timeout -k 10 120 python $OUT/csm.py > $OUT/csm_r05.log 2>&1
echo new; grep "30=" $OUT/csm_new.log; echo r05; grep "30=" $OUT/csm_r05.log
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/$OUT/csm.py > $R/$OUT/prof.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06e/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
