#!/bin/bash
# rocprofv3 kernel stats of the soft-mask forward probe variants (development aid).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp; export TMPDIR=/tmp
for v in "bench K=30" "bench K=1" "none"; do
  d=$(echo $v | tr ' =' '__')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/probe_$d -o run -- python3 $R/scripts/dev/softfwd_probe.py "$v" > $R/gpurun_out/probe_$d.log 2>&1
done
