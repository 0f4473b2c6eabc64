set -e
OUT=gpurun_out/r04ad; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "p2m or cfg2 or triangle" > $OUT/tests.log 2>&1
timeout -k 10 120 scripts/dev/_bin/p2m_probe > $OUT/probe.log 2>&1
timeout -k 10 200 python scripts/dev/p2m_ab.py 11=0 11=0 11=0 > $OUT/p2m_ab.log 2>&1
