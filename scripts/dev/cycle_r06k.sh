#!/bin/bash
# r06k: the order kernel's bounded barrier wait (fallback forced by dev param 16 = 1: tests + timing);
# the current voxelgrid's kernel trace
set -e
R=$(pwd); OUT=gpurun_out/r06k; mkdir -p $OUT
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "chip_order or soft_live or dibr_rasterization" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python scripts/dev/param_ab.py 16 0 1 0 1 0 1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
grep params $OUT/ab.txt
timeout -k 10 100 python scripts/dev/vox_trace.py > $OUT/vox.txt 2>&1; cat $OUT/vox.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/voxtr -o run -- python3 $R/scripts/dev/vox_trace.py 2 > $R/$OUT/voxtr.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06k/voxtr/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-60:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
