#!/bin/bash
# r05w: hit-list raytrace with the list offsets scanned by each pass's last workgroup (two launches
# per level): raytrace GPU tests, raytrace A/B + kernel trace
set -e
R=$(pwd); OUT=gpurun_out/r05w; mkdir -p $OUT
rc=0; timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "raytrace or spc" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
grep -v amdgpu.ids $OUT/rt_ab.log
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
