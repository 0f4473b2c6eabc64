#!/bin/bash
# r06ah: the soft forward at 5 waves per SIMD (-DST_FWD_MIN_WAVES=5: 95 VGPRs, no spills; the default build
# has 97 and 4 waves): cfg3 bench lines alternating the product library and the A/B build
# (scripts/dev/_bin/sf5, make OUT=... EXTRA=-DST_FWD_MIN_WAVES=5), kernel stats of both, then the GPU soft
# tests on the A/B build
set -e
R=$(pwd); OUT=gpurun_out/r06ah; mkdir -p $OUT
run() {  # tag, library
  KAOLIN_HIP_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 60 --warmup 5 > $OUT/b_$1.json 2> $OUT/b_$1.err
  python -c "import json;d=json.load(open('$OUT/b_$1.json'));o=d['ops'];print('$1',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in o.items()})"
}
for i in 1 2 3; do
  run base$i $R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so
  run sf5_$i $R/scripts/dev/_bin/sf5/libkaolin_hip.so
done
cd /tmp; export TMPDIR=/tmp
for t in base sf5; do
  L=$R/kaolin-windows_amd/kaolin/_lib/libkaolin_hip.so; [ $t = sf5 ] && L=$R/scripts/dev/_bin/sf5/libkaolin_hip.so
  KAOLIN_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$t -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/prof_$t.json 2> $R/$OUT/prof_$t.err
done
cd $R
python - <<'PY'
import csv
for t in ('base', 'sf5'):
    for r in csv.DictReader(open(f'gpurun_out/r06ah/prof_{t}/run_kernel_stats.csv')):
        if r['Name'].startswith('void kl::soft_tile_fwd_kernel<float, kl::SoftSrc'):
            print(t, 'soft_tile_fwd', r['Calls'], r['AverageNs'])
PY
KAOLIN_HIP_LIB=$R/scripts/dev/_bin/sf5/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
