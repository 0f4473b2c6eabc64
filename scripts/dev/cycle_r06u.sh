#!/bin/bash
# r06u: raytrace with its two outputs from one allocation and the pyramid checks on one list; tests + trace
set -e
R=$(pwd); OUT=gpurun_out/r06u; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q -x -k "raytrace or mesh_to_spc" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do timeout -k 10 100 python scripts/dev/rt_trace.py >> $OUT/rt.txt 2>&1; done
grep raytrace $OUT/rt.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/rttr -o run -- python3 $R/scripts/dev/rt_trace.py 2 > $R/$OUT/rttr.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06u/rttr/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-30:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
