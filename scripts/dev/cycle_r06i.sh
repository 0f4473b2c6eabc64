#!/bin/bash
# r06i: p2m with the tiles' records precomputed (11=0) vs computed per workgroup (11=6); the _C soft mask
# with the first rows padded during the binning chain (16=0 default, 16=1 none, 16=7 / 9 more); tests
set -e
R=$(pwd); OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q -x -k "p2m or point_to_mesh or soft_mask or cfg2 or voxel" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python scripts/dev/p2m_ab.py 11=0 11=6 11=0 11=6 > $OUT/p2m_ab.txt 2>&1 || { tail $OUT/p2m_ab.txt; exit 1; }
grep params $OUT/p2m_ab.txt
timeout -k 10 200 python scripts/dev/csm_ab.py 16=0 16=1 16=7 16=9 > $OUT/csm_ab.txt 2>&1 || { tail $OUT/csm_ab.txt; exit 1; }
grep params $OUT/csm_ab.txt
timeout -k 10 100 python scripts/dev/vox_trace.py > $OUT/vox.txt 2>&1; cat $OUT/vox.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/voxtr -o run -- python3 $R/scripts/dev/vox_trace.py 2 > $R/$OUT/voxtr.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06i/voxtr/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-40:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
