set -e
OUT=gpurun_out/r04ac; mkdir -p $OUT
timeout -k 10 200 python scripts/dev/p2m_ab.py 11=0 11=4 11=5 11=0 11=4 11=5 > $OUT/p2m_ab.log 2>&1
