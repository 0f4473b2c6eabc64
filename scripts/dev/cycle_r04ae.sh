set -e
OUT=gpurun_out/r04ae; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m > $OUT/cfg5.json 2> $OUT/cfg5.err
