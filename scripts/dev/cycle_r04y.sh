set -e
OUT=gpurun_out/r04y; mkdir -p $OUT
timeout -k 10 200 python scripts/dev/tutorial_host.py > $OUT/host.log 2>&1
