#!/bin/bash
# r06t: raytrace kernel trace (where a call's time goes)
set -e
R=$(pwd); OUT=gpurun_out/r06t; mkdir -p $OUT
timeout -k 10 100 python scripts/dev/rt_trace.py > $OUT/rt.txt 2>&1; cat $OUT/rt.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/rttr -o run -- python3 $R/scripts/dev/rt_trace.py 2 > $R/$OUT/rttr.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06t/rttr/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-30:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
