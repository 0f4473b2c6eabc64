#!/bin/bash
# r06am: final validation of round 6's last tree (voxelgrid subdivision at 5 waves per SIMD): the whole GPU
# suite (devlib + RCCL children), smoke, the default bench line, kernel stats of the step and of the legs
set -e
R=$(pwd); OUT=gpurun_out/r06am; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));t=d['deftet'];print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],'p2m',d['p2m']['ms'],'csm',d['soft_mask_C']['ms'],'vox',d['cfg4']['voxelgrid']['ms'],'m2s',d['cfg4']['mesh_to_spc']['ms'],'rt',d['raytrace']['ms'],d['raytrace']['fixed_capacity']['ms'],'deftet',t['ms'],t['fwd_ms'],'cs',d['check_sign']['ms'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sub -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 > $R/$OUT/bench_prof_sub.json 2> $R/$OUT/bench_prof_sub.err
echo done
