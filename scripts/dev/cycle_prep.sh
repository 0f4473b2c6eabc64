mkdir -p gpurun_out/prep
timeout -k 10 200 python -u -m pytest tests/test_prepare.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/prep/tests.log 2>&1
timeout -k 10 150 python scripts/dev/host_profile.py 300 > gpurun_out/prep/host_profile.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prep/c4 -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/cfg4_probe.py 5 > $GRAFT_REPO_ROOT/gpurun_out/prep/cfg4.txt 2>&1
