"""One cfg4 voxelgrid call after warm-up, for a rocprofv3 --kernel-trace of its kernels in order
(development aid): python scripts/dev/vox_trace.py [calls]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import kaolin as kal
    verts, faces = bench.cfg4_inputs('cuda')
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for _ in range(n):
        g = kal.ops.conversions.trianglemeshes_to_voxelgrids(verts[None], faces, 512)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        g = kal.ops.conversions.trianglemeshes_to_voxelgrids(verts[None], faces, 512)
    e.record()
    torch.cuda.synchronize()
    print(f'voxelgrid {s.elapsed_time(e) / 10:.4f} ms, occupied {int(g.sum())}', flush=True)


if __name__ == '__main__':
    main()
