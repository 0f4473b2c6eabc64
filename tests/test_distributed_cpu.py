"""The bench's multi-GPU logic on CPU: world_size-2 gloo processes.

bench.py shards DIB-R views contiguously across ranks (weak scaling), all-gathers the
per-shard losses (its only collective) and reports whole-job throughput from the max
over ranks of the timed region.  The HIP step itself needs a GPU; everything around it
is exercised here with the same helper functions, over gloo on 127.0.0.1.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import bench
        per_rank = 4
        views = bench.views_for_rank(rank, world, per_rank)
        all_views = [None] * world
        dist.all_gather_object(all_views, views)
        # a per-shard "loss" that depends on the shard's views
        loss = torch.tensor(sum(math.cos(v) * (k + 1) for k, v in enumerate(views)), dtype=torch.float32)
        gathered = bench.gather_losses(loss, world)
        # ranks report different elapsed times; the job time is the max
        elapsed = bench.max_over_ranks(1.0 + 0.25 * rank, torch.device('cpu'), world)
        q.put((rank, all_views, gathered.tolist(), elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_bench_sharding_gather_and_timing(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    per_rank = 4
    views0 = res[0][1]
    flat = [v for vs in views0 for v in vs]
    # shards are disjoint, contiguous, and cover the job's views exactly once
    expect = [2 * math.pi * i / (per_rank * world) for i in range(per_rank * world)]
    assert flat == pytest.approx(expect)
    for rank, views, gathered, elapsed in res:
        assert views == views0
        # every rank sees every shard's loss, in rank order
        want = [sum(math.cos(v) * (k + 1) for k, v in enumerate(views0[r])) for r in range(world)]
        assert gathered == pytest.approx(want, rel=1e-6)
        assert elapsed == pytest.approx(1.0 + 0.25 * (world - 1))


def test_single_rank_is_identity():
    import bench
    assert bench.views_for_rank(0, 1, 4) == pytest.approx([0, math.pi / 2, math.pi, 3 * math.pi / 2])
    assert bench.max_over_ranks(2.5, torch.device('cpu'), 1) == 2.5


# ------------------------------------------------------------------ launcher + point sharding
import json  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize('world', [2, 3])
def test_bench_launcher_spawns_ranks_and_shards_p2m(world):
    """bench.py --gpus N (no torchrun) starts N rank processes itself; over gloo the sharded
    point_to_mesh_distance (points split, faces replicated, outputs all-gathered, face gradient
    all-reduced) equals the unsharded op on every rank."""
    r = _run_bench(['--device', 'cpu', '--gpus', str(world), '--steps', '1'])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line['n_ranks'] == world
    assert line['p2m']['parity_all_ranks'] is True
    assert line['p2m']['points_per_rank'] == -(-203 // world)


def test_bench_refuses_world_size_mismatch():
    r = _run_bench(['--gpus', '2'], env_extra={'WORLD_SIZE': '3', 'RANK': '0'})
    assert r.returncode == 2
    assert 'refusing' in r.stderr


def test_shard_bounds_cover_in_order():
    from kaolin.distributed import shard_bounds
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


# ------------------------------------------------------------------ raytrace / voxelgrid / grads sharding
def _spc_fixture(level=4, npts=300, nrays=97, seed=3):
    """A small SPC (oracle-built octree, pyramid, exsum, point hierarchy) and rays at it."""
    import numpy as np
    from oracle import oracle as orc
    rs = np.random.RandomState(seed)
    pts = np.unique(rs.randint(0, 2 ** level, size=(npts, 3)), axis=0)
    mort = np.unique(orc.to_morton(pts))
    octree = orc.morton_to_octree(mort, level)
    _, pyramid, exsum = orc.scan_octrees(octree, np.array([octree.shape[0]], np.int32))
    ph = orc.generate_points(octree, pyramid, exsum)
    o = rs.normal(size=(nrays, 3))
    o = 3.0 * o / np.linalg.norm(o, axis=1, keepdims=True)
    d = -o + 0.6 * rs.normal(size=(nrays, 3))
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    t = torch.from_numpy
    return (t(octree), t(ph), t(np.ascontiguousarray(pyramid[0])), t(exsum), t(o.astype(np.float32)),
            t(d.astype(np.float32)), level)


def _oracle_raytrace(octree, ph, pyramid, exsum, origin, direction, level, return_depth=True, with_exit=False):
    """unbatched_raytrace's contract on CPU tensors, computed by the oracle (test stand-in for the
    GPU op: the reference's raytrace is CUDA-only)."""
    from oracle import oracle as orc
    r = orc.raytrace(octree.numpy(), ph.numpy(), pyramid.numpy(), exsum.numpy(), origin.numpy(),
                     direction.numpy(), level, return_depth, with_exit)
    nug = torch.from_numpy(r[0])
    out = (nug[:, 0].contiguous(), nug[:, 1].contiguous())
    return out + (torch.from_numpy(r[1]),) if return_depth else out


def _shard_ops_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import kaolin
        import kaolin.render.spc.raytrace as rt
        from kaolin import distributed as kd
        rt.unbatched_raytrace = _oracle_raytrace
        fx = _spc_fixture()
        res = {}
        for with_exit in (False, True):
            res[f'ray{int(with_exit)}'] = [x.clone() for x in kd.sharded_unbatched_raytrace(*fx, with_exit=with_exit)]
        res['ray_nodepth'] = [x.clone() for x in kd.sharded_unbatched_raytrace(*fx, return_depth=False)]
        # voxelgrids: 3 meshes split by mesh ('auto' at world 2/3), one mesh split by face
        g = torch.Generator().manual_seed(7)
        verts = torch.rand((3, 40, 3), generator=g)
        faces = torch.randint(0, 40, (37, 3), generator=g)
        res['vox_batch'] = kd.sharded_trianglemeshes_to_voxelgrids(verts, faces, 16)
        res['vox_faces'] = kd.sharded_trianglemeshes_to_voxelgrids(verts[:1], faces, 16)
        res['vox_faces3'] = kd.sharded_trianglemeshes_to_voxelgrids(verts, faces, 16, split='faces')
        # data-parallel gradients of a shared mesh
        a = torch.zeros(5, requires_grad=True)
        b = torch.zeros((2, 3), requires_grad=True)
        a.grad = torch.arange(5.) * (rank + 1)
        b.grad = torch.full((2, 3), float(rank))
        c = torch.zeros(3, requires_grad=True)  # no gradient on rank 0
        if rank:
            c.grad = torch.ones(3)
        kd.allreduce_grads([a, b, c])
        res['grads_sum'] = (a.grad.clone(), b.grad.clone(), c.grad.clone())
        kd.allreduce_grads([a], average=True)
        res['grads_avg'] = a.grad.clone()
        # by value: a tensor sent through the queue is shared memory the exiting worker may release
        import numpy as np
        conv = lambda x: [np.array(t) for t in x] if isinstance(x, (list, tuple)) else np.array(x)  # noqa
        q.put((rank, {k: conv(v) for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_raytrace_voxelgrid_grads(world):
    """sharded_unbatched_raytrace (rays split, nuggets all-gathered with ray offsets),
    sharded_trianglemeshes_to_voxelgrids (mesh split; face split + max-reduce) and allreduce_grads
    over gloo world 2 / 3: every rank holds the unsharded result, bit for bit."""
    import kaolin
    from kaolin.ops.conversions import trianglemeshes_to_voxelgrids
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_ops_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fx = _spc_fixture()
    want = {f'ray{int(e)}': _oracle_raytrace(*fx, with_exit=e) for e in (False, True)}
    want['ray_nodepth'] = _oracle_raytrace(*fx, return_depth=False)
    assert want['ray0'][0].numel() > 50  # the rays hit the octree
    g = torch.Generator().manual_seed(7)
    verts = torch.rand((3, 40, 3), generator=g)
    faces = torch.randint(0, 40, (37, 3), generator=g)
    full = trianglemeshes_to_voxelgrids(verts, faces, 16)
    for rank in range(world):
        r = {k: [torch.from_numpy(t) for t in v] if isinstance(v, list) else torch.from_numpy(v)
             for k, v in res[rank].items()}
        for k in ('ray0', 'ray1', 'ray_nodepth'):
            assert len(r[k]) == len(want[k])
            for x, y in zip(r[k], want[k]):
                assert x.dtype == y.dtype and torch.equal(x, y), (rank, k)
        assert torch.equal(r['vox_batch'], full)
        assert torch.equal(r['vox_faces'], full[:1])
        assert torch.equal(r['vox_faces3'], full)
        a, b, c = r['grads_sum']
        tot = sum(range(1, world + 1))
        assert torch.equal(a, torch.arange(5.) * tot)
        assert torch.equal(b, torch.full((2, 3), float(sum(range(world)))))
        assert torch.equal(c, torch.full((3,), float(world - 1)))
        assert torch.allclose(r['grads_avg'], torch.arange(5.) * tot, rtol=0, atol=1e-6)  # average of equal sums


# ------------------------------------------------------------------ §8e: sided / chamfer / batched p2m
def _sided_fwd_standin(p1, p2):
    """sided_distance's forward on CPU tensors by the oracle (test stand-in: the reference op is
    CUDA-only)."""
    from oracle import oracle as orc
    d, i = orc.sided_distance_forward(p1.detach().numpy(), p2.detach().numpy())
    return torch.from_numpy(d), torch.from_numpy(i)


def _sided_sums_standin(g, p1, p2, idx):
    """(grad_p1, grad_p2's float64 double sums): the kernel's float terms, summed in double."""
    B, M = p2.shape[0], p2.shape[1]
    q = torch.gather(p2, 1, idx.unsqueeze(-1).expand(-1, -1, 3))
    g1 = 2 * (p1 - q) * g.unsqueeze(-1)
    t = (2 * (q - p1) * g.unsqueeze(-1)).double()
    sums = torch.zeros((B, M, 3), dtype=torch.float64)
    for b in range(B):
        sums[b].index_add_(0, idx[b], t[b])
    return g1, sums


class _SidedOneRank(torch.autograd.Function):
    """The unsharded sided_distance with the same stand-ins (grad_p2 rounded once)."""

    @staticmethod
    def forward(ctx, p1, p2):
        d, i = _sided_fwd_standin(p1, p2)
        ctx.save_for_backward(p1, p2, i)
        return d

    @staticmethod
    def backward(ctx, g):
        p1, p2, i = ctx.saved_tensors
        g1, sums = _sided_sums_standin(g, p1, p2, i)
        return g1, sums.to(p2.dtype)


def _metric_inputs():
    g = torch.Generator().manual_seed(11)
    p1 = torch.rand((2, 37, 3), generator=g)
    p2 = torch.rand((2, 23, 3), generator=g)
    pc = torch.randn((5, 19, 3), generator=g)
    fv = torch.randn((5, 13, 3, 3), generator=g)
    gp = torch.rand((5, 19), generator=g)
    return p1, p2, pc, fv, gp


def _shard_metrics_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import numpy as np
        import kaolin  # noqa: F401
        from kaolin import distributed as kd
        kd._sided_forward = _sided_fwd_standin
        kd._sided_backward_sums = _sided_sums_standin
        p1, p2, pc, fv, gp = _metric_inputs()
        res = {}
        # sided: p1 split, p2 replicated
        lo, hi = kd.shard_bounds(p1.shape[1], rank, world)
        a = p1[:, lo:hi].clone().requires_grad_(True)
        b = p2.clone().requires_grad_(True)
        d, i = kd.sharded_sided_distance(a, b)
        (d * torch.arange(1., d.shape[1] + 1)).sum().backward()
        res['sided'] = [d.detach(), i, a.grad, b.grad]
        # chamfer (squared and not, weights)
        for sq in (True, False):
            a = p1.clone().requires_grad_(True)
            b = p2.clone().requires_grad_(True)
            c = kd.sharded_chamfer_distance(a, b, w1=0.7, w2=1.3, squared=sq)
            c.sum().backward()
            res[f'chamfer{int(sq)}'] = [c.detach(), a.grad, b.grad]
        # batched point_to_mesh (CPU path), 5 elements; and 2 elements (world 3: one rank has none)
        for nb in (5, 2):
            x = pc[:nb].clone().requires_grad_(True)
            y = fv[:nb].clone().requires_grad_(True)
            dd, ii, tt = kd.sharded_batched_point_to_mesh_distance(x, y)
            (dd * gp[:nb]).sum().backward()
            res[f'p2m{nb}'] = [dd.detach(), ii, tt, x.grad, y.grad]
        q.put((rank, {k: [np.array(t) for t in v] for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_sided_chamfer_batched_p2m(world):
    """§8e row 2 over gloo world 2 / 3: sharded_sided_distance (p1 split, grad_p2 all-reduced as
    double sums, rounded once), sharded_chamfer_distance (both directions split) and
    sharded_batched_point_to_mesh_distance (batch elements split, gradients all-gathered) equal the
    one-rank results on every rank, bit for bit."""
    from kaolin.metrics.pointcloud import _chamfer_from_sided
    from kaolin.metrics.trianglemesh import point_to_mesh_distance
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_metrics_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    p1, p2, pc, fv, gp = _metric_inputs()
    want = {}
    a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
    d = _SidedOneRank.apply(a, b)
    (d * torch.arange(1., d.shape[1] + 1)).sum().backward()
    want['sided'] = [d.detach(), _sided_fwd_standin(p1, p2)[1], a.grad, b.grad]
    for sq in (True, False):
        a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        c = _chamfer_from_sided(_SidedOneRank.apply(a, b), _SidedOneRank.apply(b, a), 0.7, 1.3, sq)
        c.sum().backward()
        want[f'chamfer{int(sq)}'] = [c.detach(), a.grad, b.grad]
    for nb in (5, 2):
        x, y = pc[:nb].clone().requires_grad_(True), fv[:nb].clone().requires_grad_(True)
        dd, ii, tt = point_to_mesh_distance(x, y)
        (dd * gp[:nb]).sum().backward()
        want[f'p2m{nb}'] = [dd.detach(), ii, tt, x.grad, y.grad]
    from kaolin.distributed import shard_bounds
    for rank in range(world):
        for k, ws in want.items():
            got = res[rank][k]
            assert len(got) == len(ws)
            for n, (x, y) in enumerate(zip(got, ws)):
                if k == 'sided' and n == 2:  # local_p1's gradient: the rank's own rows
                    lo, hi = shard_bounds(p1.shape[1], rank, world)
                    y = y[:, lo:hi]
                y = y.numpy()
                assert x.dtype == y.dtype and x.shape == y.shape and (x == y).all(), (rank, k, n)


def test_bit_grid_pack_unpack_roundtrip():
    """The face split's bit grid (R^3 / 8 bytes) restores the dense grid exactly, also when R^3 is
    not a multiple of 8, and OR of packed grids is the packed union."""
    from kaolin.distributed import _pack_bits, _unpack_bits
    g = torch.Generator().manual_seed(5)
    for R in (5, 8, 13):
        a = (torch.rand((1, R, R, R), generator=g) < 0.3).float()
        b = (torch.rand((1, R, R, R), generator=g) < 0.3).float()
        pa, pb = _pack_bits(a), _pack_bits(b)
        assert pa.dtype == torch.uint8 and pa.numel() == -(-R ** 3 // 8)
        assert torch.equal(_unpack_bits(pa, a), a)
        assert torch.equal(_unpack_bits(pa | pb, a), torch.maximum(a, b))
        assert torch.equal(_unpack_bits(_pack_bits(a.bool()), a.bool()), a.bool())
