#!/bin/bash
# r06ai: the raytrace's rth_count_kernel at 8 waves per SIMD (-DRTH_MIN_WAVES=8: 63 VGPRs, no spills; the
# default build has 66 and 7 waves): scripts/dev/rt_trace.py alternating the product library and the A/B build
# (scripts/dev/_bin/rt8), kernel stats of both, then the GPU SPC / raytrace tests on the A/B build
set -e
R=$(pwd); OUT=gpurun_out/r06ai; mkdir -p $OUT
B=$R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so; A=$R/scripts/dev/_bin/rt8/libkaolin_hip.so
for i in 1 2 3; do
  echo -n "base$i "; KAOLIN_HIP_LIB=$B timeout -k 10 120 python scripts/dev/rt_trace.py 2>/dev/null
  echo -n "rt8_$i "; KAOLIN_HIP_LIB=$A timeout -k 10 120 python scripts/dev/rt_trace.py 2>/dev/null
done
cd /tmp; export TMPDIR=/tmp
for t in base rt8; do
  L=$B; [ $t = rt8 ] && L=$A
  KAOLIN_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$t -o run -- python3 $R/scripts/dev/rt_trace.py > $R/$OUT/prof_$t.txt 2>&1
done
cd $R
python - <<'PY'
import csv
for t in ('base', 'rt8'):
    for r in csv.DictReader(open(f'gpurun_out/r06ai/prof_{t}/run_kernel_stats.csv')):
        if 'rth_' in r['Name']:
            print(t, r['Name'][:40], r['Calls'], r['AverageNs'])
PY
KAOLIN_HIP_LIB=$A timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "raytrace or spc" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
