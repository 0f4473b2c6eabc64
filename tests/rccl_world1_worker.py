"""Child process of tests/test_gpu_rccl.py: kaolin.distributed over a one-rank RCCL ('nccl') process
group on cuda:0.  With a process group initialised the sharded helpers run their collective path
at world size 1 too, so every device-tensor collective they use (all_gather, all_reduce,
all_to_all_single, all_gather_into_tensor) executes through RCCL here; each sharded result is
compared with the unsharded op.  Prints one JSON line: {check: true | "error text"} plus the
number of calls of each collective and whether every one of them was given CUDA tensors.
"""
import json
import math
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'kaolin-windows_amd'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CALLS = {}
ON_DEVICE = {'all': True}


def _count(name, fn):
    def wrapped(*args, **kw):
        CALLS[name] = CALLS.get(name, 0) + 1
        ts = [a for a in args if isinstance(a, torch.Tensor)]
        ts += [t for a in args if isinstance(a, (list, tuple)) for t in a if isinstance(t, torch.Tensor)]
        ON_DEVICE['all'] = ON_DEVICE['all'] and all(t.is_cuda for t in ts)
        return fn(*args, **kw)
    return wrapped


for _n in ('all_gather', 'all_reduce', 'all_to_all_single', 'all_gather_into_tensor'):
    setattr(dist, _n, _count(_n, getattr(dist, _n)))


def uv_sphere(n_lat, n_lon, r):
    lat = np.linspace(0, math.pi, n_lat + 1)[1:-1]
    lon = np.arange(n_lon) * (2 * math.pi / n_lon)
    ring = np.stack([np.sin(lat)[:, None] * np.cos(lon)[None], np.repeat(np.cos(lat)[:, None], n_lon, 1),
                     np.sin(lat)[:, None] * np.sin(lon)[None]], -1).reshape(-1, 3)
    v = np.concatenate([[[0., 1., 0.]], ring, [[0., -1., 0.]]]) * r
    f = [[0, 1 + (j + 1) % n_lon, 1 + j] for j in range(n_lon)]
    for i in range(n_lat - 2):
        for j in range(n_lon):
            a, b = 1 + i * n_lon + j, 1 + i * n_lon + (j + 1) % n_lon
            f += [[a, b, b + n_lon], [a, b + n_lon, a + n_lon]]
    last = len(v) - 1
    f += [[1 + (n_lat - 2) * n_lon + j, 1 + (n_lat - 2) * n_lon + (j + 1) % n_lon, last] for j in range(n_lon)]
    return v.astype(np.float32), np.array(f, dtype=np.int64)


def main():
    from dibr_util import assert_grads_equal
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev, rank=0, world_size=1)
    import kaolin as kal
    from kaolin import distributed as kd
    res = {'backend': str(dist.get_backend()), 'world_size': dist.get_world_size()}

    def check(name, fn):
        try:
            fn()
            res[name] = True
        except Exception:  # noqa: BLE001 -- reported per check
            res[name] = traceback.format_exc()[-1500:]

    g = torch.Generator().manual_seed(0)

    def losses():
        loss = torch.tensor(3.25, device=dev)
        out = kd.gather_losses(loss)
        assert out.is_cuda and out.shape == (1,) and float(out[0]) == 3.25
        out, work = kd.gather_losses(loss * 2, async_op=True)  # the bench's overlapped form
        assert work is not None
        work.wait()
        assert float(out[0]) == 6.5

    def grads():
        p = torch.randn(1000, generator=g).to(dev).requires_grad_(True)
        q = torch.randn(10, generator=g, dtype=torch.float64).to(dev).requires_grad_(True)
        p.grad = torch.randn(1000, generator=g).to(dev)
        want = p.grad.clone()
        kd.allreduce_grads([p, q])
        assert torch.equal(p.grad, want) and torch.equal(q.grad, torch.zeros_like(q))
        kd.allreduce_grads([p], average=True)
        assert torch.equal(p.grad, want)

    def p2m():
        pts = torch.randn((20000, 3), generator=g).to(dev)
        fv = torch.randn((2000, 3, 3), generator=g).to(dev)
        gd = torch.rand((20000,), generator=g).to(dev)
        a, b = pts.clone().requires_grad_(True), fv.clone().requires_grad_(True)
        d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(a.unsqueeze(0), b.unsqueeze(0))
        d.backward(gd.unsqueeze(0))
        a2, b2 = pts.clone().requires_grad_(True), fv.clone().requires_grad_(True)
        n0 = CALLS.get('all_reduce', 0)
        d2, i2, t2 = kd.sharded_point_to_mesh_distance(a2, b2)
        d2.backward(gd)
        assert CALLS.get('all_reduce', 0) == n0 + 1  # the face sums went through RCCL
        assert torch.equal(d2, d[0]) and torch.equal(i2, i[0]) and torch.equal(t2, t[0])
        assert torch.equal(a2.grad, a.grad)
        assert_grads_equal(b2.grad.cpu().numpy(), b.grad.cpu().numpy())

    def p2m_batched():
        pc = torch.randn((2, 5000, 3), generator=g).to(dev)
        fv = torch.randn((2, 600, 3, 3), generator=g).to(dev)
        gd = torch.rand((2, 5000), generator=g).to(dev)
        a, b = pc.clone().requires_grad_(True), fv.clone().requires_grad_(True)
        d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(a, b)
        d.backward(gd)
        a2, b2 = pc.clone().requires_grad_(True), fv.clone().requires_grad_(True)
        d2, i2, t2 = kd.sharded_batched_point_to_mesh_distance(a2, b2)
        d2.backward(gd)
        assert torch.equal(d2, d) and torch.equal(i2, i) and torch.equal(t2, t)
        assert torch.equal(a2.grad, a.grad) and torch.equal(b2.grad, b.grad)

    def sided():
        p1 = torch.rand((2, 5000, 3), generator=g).to(dev)
        p2 = torch.rand((2, 700, 3), generator=g).to(dev)
        gd = torch.rand((2, 5000), generator=g).to(dev)
        a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        d, i = kal.metrics.pointcloud.sided_distance(a, b)
        d.backward(gd)
        a2, b2 = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        d2, i2 = kd.sharded_sided_distance(a2, b2)
        d2.backward(gd)
        assert torch.equal(d2, d) and torch.equal(i2, i) and torch.equal(a2.grad, a.grad)
        assert_grads_equal(b2.grad.cpu().numpy(), b.grad.cpu().numpy())

    def sided_half():
        # dtypes without the double-sum backward replay the shard's graph
        p1 = torch.rand((1, 3000, 3), generator=g).to(dev).half()
        p2 = torch.rand((1, 500, 3), generator=g).to(dev).half()
        gd = torch.rand((1, 3000), generator=g).to(dev).half()
        a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        d, i = kal.metrics.pointcloud.sided_distance(a, b)
        d.backward(gd)
        a2, b2 = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        d2, i2 = kd.sharded_sided_distance(a2, b2)
        d2.backward(gd)
        assert torch.equal(d2, d) and torch.equal(i2, i) and torch.equal(a2.grad, a.grad)
        torch.testing.assert_close(b2.grad.float(), b.grad.float(), rtol=2e-2, atol=2e-2)

    def chamfer():
        p1 = torch.rand((2, 3000, 3), generator=g).to(dev)
        p2 = torch.rand((2, 2000, 3), generator=g).to(dev)
        a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        c = kal.metrics.pointcloud.chamfer_distance(a, b, 0.7, 1.3)
        c.sum().backward()
        a2, b2 = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        c2 = kd.sharded_chamfer_distance(a2, b2, 0.7, 1.3)
        c2.sum().backward()
        assert torch.equal(c2, c)
        assert_grads_equal(a2.grad.cpu().numpy(), a.grad.cpu().numpy())
        assert_grads_equal(b2.grad.cpu().numpy(), b.grad.cpu().numpy())

    def raytrace():
        v, f = uv_sphere(24, 36, 0.8)
        fv = torch.from_numpy(v[f]).to(dev)
        L = 6
        octree, _, _ = kal.ops.conversions.unbatched_mesh_to_spc(fv, L)
        _, pyr, ex = kal.ops.spc.scan_octrees(octree, torch.tensor([octree.numel()], dtype=torch.int32))
        pts = kal.ops.spc.generate_points(octree, pyr, ex)
        n = 40
        ii, jj = np.meshgrid(np.linspace(-0.9, 0.9, n), np.linspace(-0.9, 0.9, n), indexing='ij')
        origin = np.stack([ii, jj, np.full_like(ii, 3.)], -1).reshape(-1, 3).astype(np.float32)
        d = np.stack([0.05 * ii, 0.03 * jj, -np.ones_like(ii)], -1).reshape(-1, 3)
        d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)
        o, dd = torch.from_numpy(origin).to(dev), torch.from_numpy(d).to(dev)
        for with_exit in (False, True):
            want = kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], ex, o, dd, L, return_depth=True,
                                                     with_exit=with_exit)
            got = kd.sharded_unbatched_raytrace(octree, pts, pyr[0], ex, o, dd, L, return_depth=True,
                                                with_exit=with_exit)
            assert len(got) == len(want) and want[0].numel() > 1000
            for x, y in zip(got, want):
                assert x.dtype == y.dtype and torch.equal(x, y)

    def voxelgrid():
        verts = torch.rand((2, 300, 3), generator=g).to(dev)
        faces = torch.randint(0, 300, (500, 3), generator=g).to(dev)
        n0 = CALLS.get('all_to_all_single', 0)
        for split in ('faces', 'batch'):
            for R in (64, 37):
                want = kal.ops.conversions.trianglemeshes_to_voxelgrids(verts, faces, R)
                got = kd.sharded_trianglemeshes_to_voxelgrids(verts, faces, R, split=split)
                assert got.dtype == want.dtype and torch.equal(got, want), (split, R)
        assert CALLS.get('all_to_all_single', 0) == n0 + 2  # the bit-grid OR (face split) ran through RCCL

    for name, fn in (('gather_losses', losses), ('allreduce_grads', grads), ('p2m', p2m),
                     ('p2m_batched', p2m_batched), ('sided', sided), ('sided_half', sided_half),
                     ('chamfer', chamfer), ('raytrace', raytrace), ('voxelgrid', voxelgrid)):
        check(name, fn)
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()
    res['calls'] = CALLS
    res['collective_tensors_on_device'] = ON_DEVICE['all']
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
