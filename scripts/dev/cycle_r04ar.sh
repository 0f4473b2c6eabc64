#!/bin/bash
# tutorial-shape host cost, piece by piece + cProfile
set -e
OUT=gpurun_out/r04ar; mkdir -p $OUT
timeout -k 10 200 python scripts/dev/tutorial_host.py > $OUT/host.txt 2>&1
