"""prepare_vertices fwd + bwd on the bench leg's workload a few times (bench.prepare_leg), for a
rocprofv3 --kernel-trace --stats run (development aid).  usage: python scripts/dev/prep_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == '__main__':
    print(json.dumps(bench.prepare_leg(torch.device('cuda:0'), 20)))
