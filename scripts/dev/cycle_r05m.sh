#!/bin/bash
# r05m: DFS raytrace with slot pass + carried first child + overflow walk, compact cap-walk loop in
# the chip order kernel: GPU suite (stop on any failure), raytrace A/B, order stamps, soft stamps
# (banded / unbanded), p2m probe + counter passes, bench kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05m; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/order_stamps.log 2>&1
STAMPS_FLAGS=0 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_band.log 2>&1
STAMPS_FLAGS=0 STAMPS_PARAMS=0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_flat.log 2>&1
bash scripts/dev/p2m_pmc.sh
mkdir -p $OUT/p2m && cp -r gpurun_out/p2m_probe.log gpurun_out/p2mpmc1 gpurun_out/p2mpmc2 $OUT/p2m/
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
