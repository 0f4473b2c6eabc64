#!/bin/bash
# r06h: the loss kernel's strips in flight together (dot2 U=4): its test, the bench line, kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r06h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "loss_dot2 or dibr_rasterization" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['mode'],d['roofline']['frac'],d['p2m']['ms'],d['soft_mask_C']['ms'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06h/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
