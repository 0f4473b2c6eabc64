"""A/B of the raytrace marches on the bench's cfg4 SPC (development aid): the hit-list march
(default, 0), the per-level march (dev param 15 = 2), the fused level march (3) and the depth-first
march (4, host-sized entry only), host-sized and fixed-capacity, wall clock per call, and equality
of the answers; then the hit-list march with dev param 25 = 1 (the fixed entry fills all rows first
instead of the rows past its count afterwards) against the default."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kaolin as kal  # noqa: E402
from kaolin import _native as N  # noqa: E402


def wall(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    verts, faces = bench.cfg4_inputs('cuda')
    fv = kal.ops.mesh.index_vertices_by_faces(verts.unsqueeze(0), faces)[0].contiguous()
    octree = kal.ops.conversions.unbatched_mesh_to_spc(fv, 9)[0]
    L, pyr, exsum = kal.ops.spc.scan_octrees(octree, torch.tensor([octree.shape[0]], dtype=torch.int32))
    pts = kal.ops.spc.generate_points(octree, pyr, exsum)
    n = 512
    xs = (torch.arange(n, device='cuda', dtype=torch.float32) + 0.5) / n * 2 - 1
    tgt = torch.stack([xs.view(1, -1).expand(n, n), xs.view(-1, 1).expand(n, n), torch.zeros(n, n, device='cuda')], -1)
    o = torch.tensor([0., 0., 3.], device='cuda').expand(n * n, 3).contiguous()
    d = tgt.reshape(-1, 3) - o
    d = (d / d.norm(dim=-1, keepdim=True)).contiguous()
    res = {}
    for mode in (0, 2, 3, 4, 25):
        lib.kl_dev_set_param(15, 0 if mode == 25 else mode)
        lib.kl_dev_set_param(25, 1 if mode == 25 else 0)
        rt = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L)  # noqa: E731
        out = rt()
        ms = wall(rt)
        cap = 8 * 2000000
        rtf = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L, capacity=cap)  # noqa
        fo = rtf()
        msf = wall(rtf)
        res[mode] = (out, fo)
        print(f'mode {mode}: host-sized {ms:.3f} ms, fixed {msf:.3f} ms, hits {out[0].shape[0]}', flush=True)
    lib.kl_dev_set_param(15, 0)
    lib.kl_dev_set_param(25, 0)
    for m in (0, 3, 4, 25):
        (a, fa), (b, fb) = res[m], res[2]
        print(f'mode {m} vs 2 equal host-sized:', all(torch.equal(x, y) for x, y in zip(a, b)))
        print(f'mode {m} vs 2 equal fixed:', all(torch.equal(x, y) for x, y in zip(fa, fb)))


if __name__ == '__main__':
    main()
