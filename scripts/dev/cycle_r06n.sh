#!/bin/bash
# r06n: voxelgrid -- later levels in one persistent launch, in-kernel normalisation, library zero fill
set -e
R=$(pwd); OUT=gpurun_out/r06n; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q -x -k "voxel" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "voxel" --timeout 200 --timeout-method thread > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
for i in 1 2; do timeout -k 10 100 python scripts/dev/vox_trace.py >> $OUT/vox.txt 2>&1; done; grep voxelgrid $OUT/vox.txt
timeout -k 10 200 python scripts/dev/vox_ab.py 21=0 21=1 21=3 21=4 > $OUT/vox_ab.txt 2>&1 || { tail $OUT/vox_ab.txt; exit 1; }; grep params $OUT/vox_ab.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/voxtr -o run -- python3 $R/scripts/dev/vox_trace.py 2 > $R/$OUT/voxtr.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06n/voxtr/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-24:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
