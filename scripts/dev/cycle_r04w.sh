set -e
OUT=gpurun_out/r04w; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --no-p2m --steps 10 > "$ROOT/$OUT/prof_bench.log" 2>&1
