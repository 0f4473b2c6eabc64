#!/bin/bash
# r06al: the voxelgrid subdivide async / tail kernels at 5 waves per SIMD (-DVOX_MIN_WAVES=5: 96 VGPRs, no spills; the
# default build has 98 / 97 and 4 waves): scripts/dev/vox_trace.py alternating the product library and the A/B build
# (scripts/dev/_bin/vx5), kernel stats of both, then the GPU voxelgrid tests on the A/B build
set -e
R=$(pwd); OUT=gpurun_out/r06al; mkdir -p $OUT
B=$R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so; A=$R/scripts/dev/_bin/vx5/libkaolin_hip.so
for i in 1 2 3; do
  echo -n "base$i "; KAOLIN_HIP_LIB=$B timeout -k 10 120 python scripts/dev/vox_trace.py 2>/dev/null
  echo -n "vx5_$i "; KAOLIN_HIP_LIB=$A timeout -k 10 120 python scripts/dev/vox_trace.py 2>/dev/null
done
cd /tmp; export TMPDIR=/tmp
for t in base vx5; do
  L=$B; [ $t = vx5 ] && L=$A
  KAOLIN_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$t -o run -- python3 $R/scripts/dev/vox_trace.py > $R/$OUT/prof_$t.txt 2>&1
done
cd $R
python - <<'PY'
import csv
for t in ('base', 'vx5'):
    for r in csv.DictReader(open(f'gpurun_out/r06al/prof_{t}/run_kernel_stats.csv')):
        if 'subdivide_' in r['Name']:
            print(t, r['Name'][:40], r['Calls'], r['AverageNs'])
PY
KAOLIN_HIP_LIB=$A timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "voxel" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
