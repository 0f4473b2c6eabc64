#!/bin/bash
# r06q: mesh_to_spc -- node kernel keeps (node, face) of its first chunks for the append pass, the three
# outputs from one allocation; tests (product + dev), timing and kernel trace; the _C soft-mask tests
set -e
R=$(pwd); OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q -x -k "mesh_to_spc or spc or raytrace or soft_mask_C" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "mesh_to_spc or soft_mask_C" --timeout 200 --timeout-method thread > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
for i in 1 2 3; do timeout -k 10 100 python scripts/dev/m2s_trace.py >> $OUT/m2s.txt 2>&1; done; grep mesh_to_spc $OUT/m2s.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/m2str -o run -- python3 $R/scripts/dev/m2s_trace.py 2 > $R/$OUT/m2str.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06q/m2str/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
rows=rows[-22:]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    print(r['Kernel_Name'][:60], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
