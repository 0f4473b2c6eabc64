set -e
OUT=gpurun_out/r04af; mkdir -p $OUT
timeout -k 10 300 python scripts/dev/param_ab.py combo 0=0 0=1,2=4096 1=1,3=4096 0=2,2=4096 1=2,3=4096 1=3,3=2048 0=0 > $OUT/ab.log 2>&1
