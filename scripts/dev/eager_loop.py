"""The eager cfg3 step in a loop, for a rocprofv3 --hip-trace run (development aid).
usage: python scripts/dev/eager_loop.py [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    for _ in range(5):
        bench.dibr_step(inp, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        bench.dibr_step(inp, 1)
    torch.cuda.synchronize()
    print(f'eager: {(time.perf_counter() - t0) / n * 1e6:.1f} us/step')


if __name__ == '__main__':
    main()
