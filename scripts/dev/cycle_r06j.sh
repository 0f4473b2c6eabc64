#!/bin/bash
# r06j: r06h (loss kernel) + r06i (p2m precomputed tiles, _C soft-mask padding beside the binning chain,
# voxelgrid kernel trace) in one call
set -e
bash scripts/dev/cycle_r06i.sh
bash scripts/dev/cycle_r06h.sh
