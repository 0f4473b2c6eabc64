#!/bin/bash
# r06b: 16-bit soft slot lists (LDS 40.6 -> 32 KB per item, 5 workgroups per CU): parity tests, then
# same-box A/B of dibr_forward against the r05 build and a 6-wave variant, bench line, kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "soft or dibr or fused or rasterize" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -x -q --timeout 200 --timeout-method thread -k "cfg3" > $OUT/tests_full.log 2>&1 || { tail -40 $OUT/tests_full.log; exit 1; }
tail -2 $OUT/tests_full.log
for i in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 29 0 1 0 1 >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/r05lib/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 0 | sed 's/^/r05 /' >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/mw6/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 0 | sed 's/^/mw6 /' >> $OUT/ab.txt 2>&1
done
cat $OUT/ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['mode'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06b/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('soft_tile','raster_tile','gather2','bin_word','countorder','dot2')):
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
