"""check_sign on the bench workload (1M points vs the 50k-face sphere) a few times, for a
rocprofv3 --kernel-trace --stats run (development aid).
usage: python scripts/dev/cs_probe.py [n] [dev_flags ...]   (each flag set timed in turn)"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import kaolin as kal
    verts, faces = bench.uv_sphere(126, 200, 'cuda')
    g = torch.Generator().manual_seed(3)
    pts = (torch.rand((1, 1000000, 3), generator=g) * 2 - 1).to('cuda')
    v = verts.unsqueeze(0).contiguous()
    lib = kal._native.lib()
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    ref = kal.ops.mesh.check_sign(v, faces, pts)
    torch.cuda.synchronize()
    for flags in [int(x, 0) for x in sys.argv[2:]] or [0]:
        lib.kl_dev_set_flags(flags)
        assert torch.equal(kal.ops.mesh.check_sign(v, faces, pts), ref)
        for _ in range(n):
            t0 = time.perf_counter()
            kal.ops.mesh.check_sign(v, faces, pts)
            torch.cuda.synchronize()
            print(f'flags {flags:#x} check_sign {(time.perf_counter() - t0) * 1e3:.3f} ms', flush=True)
    lib.kl_dev_set_flags(0)


if __name__ == '__main__':
    main()
