#!/bin/bash
# r06r: validation of the r06 session-2 changes: the whole GPU suite (devlib + RCCL children included),
# smoke, the default bench line, kernel stats of the step
set -e
R=$(pwd); OUT=gpurun_out/r06r; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['mode'],d['roofline']['frac'],'p2m',d['p2m']['ms'],'csm',d['soft_mask_C']['ms'],d['soft_mask_C']['roofline']['frac'],'vox',d['cfg4']['voxelgrid']['ms'],'m2s',d['cfg4']['mesh_to_spc']['ms'],'rt',d['raytrace']['ms'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06r/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
for i in 1 2 3; do
  timeout -k 10 120 python scripts/dev/param_ab.py 0 0 >> $OUT/ab.txt 2>&1
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/sbvs7/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 | sed 's/^/sbvs7 /' >> $OUT/ab.txt 2>&1
done
grep params $OUT/ab.txt
