"""cfg4 legs (voxelgrid R=512, mesh_to_spc L=9, raytrace 512^2) run a few times each with wall
timing, for a rocprofv3 --kernel-trace --stats run (development aid).
usage: python scripts/dev/cfg4_probe.py [reps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    if len(sys.argv) > 2:  # dev parameter overrides "IDX=V,IDX=V"
        import ctypes
        from kaolin import _native
        lib = _native.lib()
        lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
        for kv in sys.argv[2].split(','):
            i, v = (int(x) for x in kv.split('='))
            lib.kl_dev_set_param(i, v)
        print('params', sys.argv[2], flush=True)
    import kaolin as kal
    verts, faces = bench.cfg4_inputs('cuda')
    vb = verts.unsqueeze(0).contiguous()
    fv = kal.ops.mesh.index_vertices_by_faces(vb, faces)[0].contiguous()
    for name, fn in (('voxelgrid', lambda: kal.ops.conversions.trianglemeshes_to_voxelgrids(vb, faces, 512)),
                     ('mesh_to_spc', lambda: kal.ops.conversions.unbatched_mesh_to_spc(fv, 9))):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f'{name}: ' + ' '.join(f'{t:.3f}' for t in ts) + ' ms', flush=True)
    octree = kal.ops.conversions.unbatched_mesh_to_spc(fv, 9)[0]
    import ctypes
    from kaolin import _native
    cnt = (ctypes.c_int64 * 16)()
    nl = _native.lib().kl_mesh_to_spc_level_counts(cnt, 16)
    print('mesh_to_spc proposals per level:', list(cnt)[:nl], 'nodes', octree.shape[0], flush=True)
    L, pyr, exsum = kal.ops.spc.scan_octrees(octree, torch.tensor([octree.shape[0]], dtype=torch.int32))
    pts = kal.ops.spc.generate_points(octree, pyr, exsum)
    n = 512
    xs = (torch.arange(n, device='cuda', dtype=torch.float32) + 0.5) / n * 2 - 1
    tgt = torch.stack([xs.view(1, -1).expand(n, n), xs.view(-1, 1).expand(n, n), torch.zeros(n, n, device='cuda')], -1)
    o = torch.tensor([0., 0., 3.], device='cuda').expand(n * n, 3).contiguous()
    d = tgt.reshape(-1, 3) - o
    d = (d / d.norm(dim=-1, keepdim=True)).contiguous()
    rt = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L)  # noqa: E731
    rt()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rt()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print('raytrace: ' + ' '.join(f'{t:.3f}' for t in ts) + ' ms', flush=True)


if __name__ == '__main__':
    main()
