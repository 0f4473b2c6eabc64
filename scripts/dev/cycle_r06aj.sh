#!/bin/bash
# r06aj: the raster tile kernel at 8 waves per SIMD (-DRT_MIN_WAVES=8: 64 VGPRs, 6 spilled; the default build
# has 68 and 7 waves, 3 workgroups of 8 waves per CU): cfg3 bench lines alternating the product library and the A/B build
# (scripts/dev/_bin/rs8, make OUT=... EXTRA=-DRT_MIN_WAVES=8), kernel stats of both, then the GPU raster
# tests on the A/B build
set -e
R=$(pwd); OUT=gpurun_out/r06aj; mkdir -p $OUT
run() {  # tag, library
  KAOLIN_HIP_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 60 --warmup 5 > $OUT/b_$1.json 2> $OUT/b_$1.err
  python -c "import json;d=json.load(open('$OUT/b_$1.json'));o=d['ops'];print('$1',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in o.items()})"
}
for i in 1 2 3; do
  run base$i $R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so
  run rs8_$i $R/scripts/dev/_bin/rs8/libkaolin_hip.so
done
cd /tmp; export TMPDIR=/tmp
for t in base rs8; do
  L=$R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so; [ $t = rs8 ] && L=$R/scripts/dev/_bin/rs8/libkaolin_hip.so
  KAOLIN_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$t -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/prof_$t.json 2> $R/$OUT/prof_$t.err
done
cd $R
python - <<'PY'
import csv
for t in ('base', 'rs8'):
    for r in csv.DictReader(open(f'gpurun_out/r06aj/prof_{t}/run_kernel_stats.csv')):
        if r['Name'].startswith('void kl::raster_tile_kernel<float'):
            print(t, 'raster_tile', r['Calls'], r['AverageNs'])
PY
KAOLIN_HIP_LIB=$R/scripts/dev/_bin/rs8/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "raster or rasterize or dibr" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
