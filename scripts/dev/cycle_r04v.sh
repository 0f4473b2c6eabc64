set -e
OUT=gpurun_out/r04v; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python scripts/dev/param_ab.py combo 0=0 0=4 0=4,2=512 0=4,1=5 0=4,1=5,2=512,3=256 0=3,1=5,2=768,3=256 1=5,3=256 0=0 > $OUT/ab.log 2>&1
