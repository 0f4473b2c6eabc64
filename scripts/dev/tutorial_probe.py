"""The bench's tutorial loop alone, for rocprofv3 --kernel-trace --stats (development aid).
usage: python scripts/dev/tutorial_probe.py [steps]   (SHAPE=1: the call-shape step only)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    st = bench.tutorial_setup('cuda')
    step = bench.tutorial_shape_step if os.environ.get('SHAPE') else bench.tutorial_step
    for _ in range(3):
        step(st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step(st)
    torch.cuda.synchronize()
    print(f'tutorial step: {(time.perf_counter() - t0) / n * 1e3:.3f} ms')


if __name__ == '__main__':
    main()
