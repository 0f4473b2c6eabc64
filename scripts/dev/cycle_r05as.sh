#!/bin/bash
# r05as: gather partials' row stride 65 (devlib/g2pad) against 64 (the in-tree build);
# short cfg3 lines alternated, then cfg5; the bench's parity block checks the gradients each line
set -e
R=$(pwd); OUT=gpurun_out/r05as; mkdir -p $OUT
for k in 1 2 3; do
  KAOLIN_HIP_LIB=$R/devlib/g2pad/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_pad_$k.json 2> $OUT/cfg3_pad_$k.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_nopad_$k.json 2> $OUT/cfg3_nopad_$k.err
done
KAOLIN_HIP_LIB=$R/devlib/g2pad/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_pad.json 2> $OUT/cfg5_pad.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_nopad.json 2> $OUT/cfg5_nopad.err
cd /tmp; export TMPDIR=/tmp
KAOLIN_HIP_LIB=$R/devlib/g2pad/libkaolin_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_pad -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/prof_pad.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_nopad -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/prof_nopad.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/g2pad/libkaolin_hip.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS --kernel-include-regex "gather2" --output-format csv \
    -d $R/$OUT/pmc_pad -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/pmc_pad.log 2>&1
cd $R
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$(basename $f)',d['value'],'eager',d['eager']['ms_per_step'],'bwd',d['ops']['dibr_backward']['ms'],d['parity']['grad_fvi_equal'],d['parity']['grad_feat_equal'])"; done
for v in pad nopad; do python -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$v/run_kernel_stats.csv')):
    if 'gather2' in r['Name'] or 'soft_tile_bwd' in r['Name']: print('$v', r['Name'][:40], round(float(r['AverageNs'])/1000,2))"; done
