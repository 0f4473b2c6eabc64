# Full GPU cycle (development aid): all GPU tests, the default bench line, a kernel-trace
# profile of a short bench, and the check_sign probe under the profiler.
# usage (on the GPU box): bash scripts/dev/cycle_full.sh <tag>
set -e
T=${1:-cycle}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cs -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/cs_probe.py 5 > $O/cs_probe.txt 2>&1
