#!/bin/bash
# r06p: _C contract soft mask -- word binning + chip order kernel (soft bitmap only), both padding the first
# rows of the slot tensors; tests (product + dev library) and the A/B
set -e
R=$(pwd); OUT=gpurun_out/r06p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft_mask" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft_mask_C" --timeout 200 --timeout-method thread > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
timeout -k 10 300 python scripts/dev/csm_ab.py 28=0 31=1 28=1 28=0 31=1 28=1 > $OUT/csm_ab.txt 2>&1 || { tail $OUT/csm_ab.txt; exit 1; }
grep params $OUT/csm_ab.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/scripts/dev/csm_ab.py 28=0 > $R/$OUT/prof.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06p/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'kl::' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
timeout -k 10 100 python scripts/dev/m2s_trace.py > $OUT/m2s.txt 2>&1; cat $OUT/m2s.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/m2str -o run -- python3 $R/scripts/dev/m2s_trace.py 2 > $R/$OUT/m2str.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06p/m2str/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-40:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
