"""Multi-GPU sharding of the hot path: one process per GPU, RCCL over xGMI.

Kaolin itself is single-device; these helpers are what a data-parallel caller of its ops
runs on every rank.  Nothing here changes an op's arithmetic: a shard's outputs are the
unsharded op's outputs for those rows, bit for bit, and every gathered result equals the
unsharded op's result bit for bit.

* DIB-R: views are independent, so a rank renders a contiguous slice of them
  (``shard_bounds`` over the view count) with the mesh replicated; the caller gathers
  per-shard losses (``gather_losses``).  In a training loop over a shared mesh (the reference's
  dibr_tutorial.ipynb cell 14: one ``vertices`` / ``shift`` / texture, Adam) each rank's backward
  gives the gradient of its views; ``allreduce_grads`` sums (or averages) the parameters'
  gradients over the ranks in one flat bucket before the optimiser step.
* point_to_mesh_distance on one large cloud: the points are split contiguously over the
  ranks, the faces replicated.  ``sharded_point_to_mesh_distance`` evaluates the rank's points
  and all-gathers (dist, face_idx, dist_type).  In the backward each rank's points get their
  gradient locally; the face gradient, a sum over all points, is all-reduced as the per-rank
  DOUBLE sums of the per-point float terms and rounded once (GPU, float32 inputs), which is the
  unsharded backward's gradient (itself such a double sum rounded once) up to the one-ulp
  allowance of the summation order that bench.py and tests/dibr_util.py document: float32 terms
  add exactly in double unless their magnitudes span more than ~2^29.
* point_to_mesh_distance on a batch (reference metrics/trianglemesh.py:79-91 loops over the
  batch): ``sharded_batched_point_to_mesh_distance`` splits the batch elements over the ranks;
  each element is independent, so the all-gathered outputs and gradients are the unsharded
  ones bit for bit.
* sided_distance / chamfer_distance (reference metrics/pointcloud.py:20-136):
  ``sharded_sided_distance`` splits p1's points, p2 replicated; (dist, idx) are all-gathered and
  grad_p2 is all-reduced as double sums and rounded once, as for point_to_mesh.
  ``sharded_chamfer_distance`` runs both directions that way (p1 split for p1 -> p2, p2 split for
  p2 -> p1) and applies the reference's means to the gathered distances.
* unbatched_raytrace (reference render/spc/raytrace.py:31-84): the rays are split contiguously,
  the octree replicated; each rank marches its rays, offsets its ray indices by its first ray
  and the nuggets are all-gathered with their per-rank counts (all-gather-v).  The reference's
  output is ray-major, so the rank-order concatenation is the unsharded output.
* trianglemeshes_to_voxelgrids (reference ops/conversions/trianglemesh.py:29-110): a batch is
  split by mesh (grids all-gathered); one mesh (or fewer meshes than ranks) is split by face
  and the per-rank grids are OR-reduced as bit grids (R^3 / 8 bytes: 16 MB at R = 512, against
  537 MB for the dense float grid) -- the voxel set is a union over faces (every rank also marks
  the vertices), so the OR of the shards is the unsharded grid.  RCCL has no bitwise reduction:
  the OR is a reduce-scatter done by hand (all_to_all of the packed bytes, an OR of the world's
  copies of the rank's slice, all_gather of the slices), the same bytes on the links as a ring
  all-reduce.
"""
import torch
import torch.distributed as dist

__all__ = ['shard_bounds', 'gather_losses', 'allreduce_grads', 'sharded_point_to_mesh_distance',
           'sharded_batched_point_to_mesh_distance', 'sharded_sided_distance', 'sharded_chamfer_distance',
           'sharded_unbatched_raytrace', 'sharded_trianglemeshes_to_voxelgrids']


def shard_bounds(n, rank, world):
    """[lo, hi) of rank's contiguous share of n items; shares differ by at most one and
    are in rank order, so concatenating them in rank order restores the original order."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _active():
    """An initialised process group: the sharded paths then run their collectives, at world size 1
    too (an RCCL group of one rank runs every all_gather / all_reduce / all_to_all on the device, so
    the collective path is exercised on a one-GPU box, tests/test_gpu_rccl.py).  Without one, the
    helpers call the unsharded op."""
    return dist.is_available() and dist.is_initialized()


def _world(group):
    return dist.get_world_size(group) if _active() else 1


def _rank(group):
    return dist.get_rank(group) if _active() else 0


def _staged(t, group):
    """gloo has no all_gather for device tensors: such collectives go through host copies."""
    return t.is_cuda and dist.get_backend(group) == 'gloo'


def _all_gather(outs, t, group):
    if _staged(t, group):
        host = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
        dist.all_gather(host, t.cpu(), group=group)
        for o, h in zip(outs, host):
            o.copy_(h)
    else:
        dist.all_gather(outs, t, group=group)


def _all_reduce(t, op, group):
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def _all_to_all(out, t, group):
    if _staged(t, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, t.cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_to_all_single(out, t, group=group)


def _all_gather_flat(out, t, group):
    if _staged(t, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, t.cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, t, group=group)


def gather_losses(loss, group=None, async_op=False):
    """All-gather one scalar loss per rank -> (world,) in rank order.

    ``async_op=True`` returns ``(out, work)``: ``out`` holds the losses once ``work.wait()`` has
    returned (RCCL: the caller's current stream then waits for the gather; ``work`` is None when
    the gather already completed, as with no process group or gloo's host-staged path).  A training
    loop waits for step k's gather after queueing step k + 1, so the gather's latency over xGMI
    overlaps the next step's kernels instead of sitting between the steps."""
    world = _world(group)
    flat = loss.detach().reshape(1)
    if not _active():
        return (flat, None) if async_op else flat
    out = flat.new_empty(world)
    work = None
    if _staged(flat, group):
        _all_gather_flat(out, flat, group)
    else:
        work = dist.all_gather_into_tensor(out, flat, group=group, async_op=async_op)
    return (out, work) if async_op else out


def allreduce_grads(params, group=None, average=False):
    """Sum (``average``: mean) the ``.grad`` of ``params`` over the ranks, in place: the shared
    mesh's data-parallel step (each rank rendered its views; the unsharded gradient is the sum
    over all views).  One flat bucket, one all_reduce per dtype/device (the tutorial's vertices,
    shift and texture: ~0.3 MB + 3 MB at cfg3).  Parameters without a gradient on this rank
    contribute zeros.  The per-rank gradients are rounded before the sum, so the result equals
    the unsharded gradient up to float summation order (the exact variant needs the ops' double
    sums, as sharded_point_to_mesh_distance does)."""
    world = _world(group)
    params = [p for p in params if p.requires_grad]
    if not _active() or not params:
        return
    buckets = {}
    for p in params:
        buckets.setdefault((p.dtype, p.device), []).append(p)
    for ps in buckets.values():
        flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in ps])
        _all_reduce(flat, dist.ReduceOp.SUM, group)
        if average:
            flat /= world
        off = 0
        for p in ps:
            n = p.numel()
            g = flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += n


def _sizes(n, device, group):
    """every rank's row count, in rank order"""
    world = _world(group)
    t = torch.tensor([n], dtype=torch.int64, device=device)
    ns = [torch.empty_like(t) for _ in range(world)]
    _all_gather(ns, t, group)
    return [int(x) for x in ns]


def _all_gather_rows(t, sizes, group):
    """Concatenate every rank's (n_r, ...) tensor in rank order (rows padded to the
    largest share for the collective, then trimmed): all-gather-v."""
    world = len(sizes)
    m = max(sizes)
    if m == 0:
        return t[:0]
    if t.shape[0] < m:
        t = torch.cat([t, t.new_zeros((m - t.shape[0],) + tuple(t.shape[1:]))])
    bufs = [torch.empty_like(t) for _ in range(world)]
    _all_gather(bufs, t.contiguous(), group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


def _p2m_face_sums(g_local, lp, fv, i, t):
    """(grad_points, the face gradient's double sums) of the rank's points (GPU, distance.hip)."""
    from . import _native as N
    P, F = lp.shape[0], fv.shape[0]
    gp = torch.empty_like(lp)
    sums = torch.empty((F, 3, 3), dtype=torch.float64, device=lp.device)
    with N.on_device(lp.device):
        N.check(N.lib().kl_unbatched_triangle_distance_backward_sums(
            N.dtype_code(lp.dtype), P, F, N.ptr(g_local.contiguous()), N.ptr(lp.contiguous()),
            N.ptr(fv.contiguous()), N.ptr(i.contiguous()), N.ptr(t.contiguous()), N.ptr(gp), N.ptr(sums),
            N.stream_of(lp.device)), 'sharded_point_to_mesh_distance backward')
    return gp, sums


class _ShardedP2M(torch.autograd.Function):

    @staticmethod
    def forward(ctx, local_points, face_vertices, sizes, group):
        from .metrics.trianglemesh import point_to_mesh_distance
        ctx.sizes, ctx.group = sizes, group
        ctx.exact = local_points.is_cuda and local_points.dtype in (torch.float32, torch.float64)
        if ctx.exact:
            # forward outputs only; the backward's face sums come from the double-sum entry point
            with torch.no_grad():
                d, i, t = point_to_mesh_distance(local_points.unsqueeze(0), face_vertices.unsqueeze(0))
            ctx.save_for_backward(local_points, face_vertices, i[0], t[0])
        else:
            with torch.enable_grad():
                lp = local_points.detach().requires_grad_(local_points.requires_grad)
                fv = face_vertices.detach().requires_grad_(face_vertices.requires_grad)
                d, i, t = point_to_mesh_distance(lp.unsqueeze(0), fv.unsqueeze(0))
            ctx.local = (lp, fv, d)  # the shard's own graph, replayed by backward
        out_i, out_t = _all_gather_rows(i[0], sizes, group), _all_gather_rows(t[0], sizes, group)
        ctx.mark_non_differentiable(out_i, out_t)
        return _all_gather_rows(d[0].detach(), sizes, group), out_i, out_t

    @staticmethod
    def backward(ctx, g_dist, g_idx, g_type):
        rank = dist.get_rank(ctx.group)
        lo = sum(ctx.sizes[:rank])
        g_local = g_dist[lo:lo + ctx.sizes[rank]]
        if ctx.exact:
            lp, fv, i, t = ctx.saved_tensors
            gp, sums = _p2m_face_sums(g_local, lp, fv, i, t)
            g_fv = None
            if ctx.needs_input_grad[1]:
                # the ranks' double sums added (exact for float32 terms within ~2^29 of each other)
                # and rounded once, as the unsharded backward rounds its own double sum
                _all_reduce(sums, dist.ReduceOp.SUM, ctx.group)
                g_fv = sums.to(fv.dtype)
            return (gp if ctx.needs_input_grad[0] else None), g_fv, None, None
        lp, fv, d = ctx.local
        inputs = [x for x in (lp, fv) if x.requires_grad]
        grads = torch.autograd.grad(d, inputs, g_local.reshape(1, -1).contiguous(), allow_unused=True) \
            if inputs else []
        it = iter(grads)
        g_lp = next(it) if lp.requires_grad else None
        g_fv = next(it) if fv.requires_grad else None
        if g_fv is not None:
            g_fv = g_fv.contiguous()
            _all_reduce(g_fv, dist.ReduceOp.SUM, ctx.group)
        return g_lp, g_fv, None, None


def _split_sizes(n, world):
    return [hi - lo for lo, hi in (shard_bounds(n, r, world) for r in range(world))]


class _ShardedBatchedP2M(torch.autograd.Function):

    @staticmethod
    def forward(ctx, pointclouds, face_vertices, lo, hi, sizes, group):
        from .metrics.trianglemesh import point_to_mesh_distance
        ctx.lo, ctx.hi, ctx.sizes, ctx.group = lo, hi, sizes, group
        with torch.enable_grad():
            lp = pointclouds[lo:hi].detach().requires_grad_(pointclouds.requires_grad)
            fv = face_vertices[lo:hi].detach().requires_grad_(face_vertices.requires_grad)
            if hi > lo:
                d, i, t = point_to_mesh_distance(lp, fv)
            else:  # more ranks than batch elements: this rank has none
                P = pointclouds.shape[1]
                d = pointclouds.new_empty((0, P))
                i = torch.empty((0, P), dtype=torch.long, device=pointclouds.device)
                t = torch.empty((0, P), dtype=torch.int32, device=pointclouds.device)
        ctx.local = (lp, fv, d)
        out_i, out_t = _all_gather_rows(i, sizes, group), _all_gather_rows(t, sizes, group)
        ctx.mark_non_differentiable(out_i, out_t)
        return _all_gather_rows(d.detach(), sizes, group), out_i, out_t

    @staticmethod
    def backward(ctx, g_dist, g_idx, g_type):
        lp, fv, d = ctx.local
        inputs = [x for x in (lp, fv) if x.requires_grad]
        grads = []
        if inputs and ctx.hi > ctx.lo:
            grads = torch.autograd.grad(d, inputs, g_dist[ctx.lo:ctx.hi].contiguous(), allow_unused=True)
        it = iter(grads)
        out = []
        for x, need in ((lp, ctx.needs_input_grad[0]), (fv, ctx.needs_input_grad[1])):
            g = next(it, None) if x.requires_grad else None
            if not need:
                out.append(None)
                continue
            g = torch.zeros_like(x) if g is None else g.contiguous()
            out.append(_all_gather_rows(g, ctx.sizes, ctx.group))  # every element's own gradient
        return out[0], out[1], None, None, None, None


def sharded_batched_point_to_mesh_distance(pointclouds, face_vertices, group=None):
    r"""point_to_mesh_distance of a batch, (B,P,3) points against (B,F,3,3) triangles, with the
    batch elements split contiguously over the ranks of ``group`` (the reference loops over them,
    metrics/trianglemesh.py:79-91).  Both inputs are the whole batch on every rank.  Returns the
    unsharded (dist (B,P), face_idx (B,P) int64, dist_type (B,P) int32) on every rank; gradients
    reach both inputs for every element (each rank's elements' gradients are all-gathered), so
    every rank holds the unsharded gradients, bit for bit."""
    world, rank = _world(group), _rank(group)
    if not _active():
        from .metrics.trianglemesh import point_to_mesh_distance
        return point_to_mesh_distance(pointclouds, face_vertices)
    B = pointclouds.shape[0]
    lo, hi = shard_bounds(B, rank, world)
    return _ShardedBatchedP2M.apply(pointclouds, face_vertices, lo, hi, _split_sizes(B, world), group)


def _all_gather_points(t, sizes, group):
    """all-gather-v along dim 1 (points) of (B, n_r, ...) tensors, in rank order."""
    return _all_gather_rows(t.transpose(0, 1).contiguous(), sizes, group).transpose(0, 1).contiguous()


def _sided_forward(p1, p2):
    from .metrics.pointcloud import sided_distance
    with torch.no_grad():
        return sided_distance(p1, p2)


def _sided_backward_sums(grad, p1, p2, idx):
    """(grad_p1, grad_p2's (B,M,3) float64 double sums) of the rank's p1 points (GPU, distance.hip)."""
    from . import _C
    return _C.sided_distance_backward_sums(grad, p1, p2, idx)


class _ShardedSided(torch.autograd.Function):

    @staticmethod
    def forward(ctx, p1, p2, lo, hi, sizes, group, full):
        # full: p1 is the whole cloud (replicated) and the rank evaluates points [lo, hi); its
        # gradient is then all-gathered so that every rank holds all of it.  Else p1 is the
        # rank's share and its gradient stays local.
        lp = (p1[:, lo:hi] if full else p1).contiguous()
        p2c = p2.contiguous()
        ctx.lo, ctx.sizes, ctx.group, ctx.full = lo, sizes, group, full
        # the double-sum backward takes float32 / float64 GPU inputs; any other dtype (float16: the
        # unsharded op's half atomics) replays the shard's own graph and all-reduces its float grad_p2
        ctx.exact = not p1.is_cuda or p1.dtype in (torch.float32, torch.float64)
        if ctx.exact:
            d, i = _sided_forward(lp, p2c)
            ctx.save_for_backward(lp, p2c, i)
        else:
            from .metrics.pointcloud import sided_distance
            with torch.enable_grad():
                lpg = lp.detach().requires_grad_(p1.requires_grad)
                p2g = p2c.detach().requires_grad_(p2.requires_grad)
                d, i = sided_distance(lpg, p2g)
            ctx.local = (lpg, p2g, d)
            d = d.detach()
        out_i = _all_gather_points(i, sizes, group)
        ctx.mark_non_differentiable(out_i)
        return _all_gather_points(d, sizes, group), out_i

    @staticmethod
    def backward(ctx, g_dist, g_idx):
        if not ctx.exact:
            return _ShardedSided._replayed_backward(ctx, g_dist)
        lp, p2, i = ctx.saved_tensors
        n = lp.shape[1]
        g1, sums = _sided_backward_sums(g_dist[:, ctx.lo:ctx.lo + n].contiguous(), lp, p2, i)
        g2 = None
        if ctx.needs_input_grad[1]:
            _all_reduce(sums, dist.ReduceOp.SUM, ctx.group)  # exact double sums (float32 terms)
            g2 = sums.to(p2.dtype)                           # rounded once, as the unsharded backward
        if not ctx.needs_input_grad[0]:
            g1 = None
        elif ctx.full:
            g1 = _all_gather_points(g1, ctx.sizes, ctx.group)
        return g1, g2, None, None, None, None, None

    @staticmethod
    def _replayed_backward(ctx, g_dist):
        """The shard's sided_distance graph replayed (its own dtype's backward); grad_p2 all-reduced
        in the input dtype: the unsharded gradient up to the summation order of its atomics."""
        lp, p2, d = ctx.local
        n = lp.shape[1]
        inputs = [x for x in (lp, p2) if x.requires_grad]
        grads = torch.autograd.grad(d, inputs, g_dist[:, ctx.lo:ctx.lo + n].contiguous(), allow_unused=True) \
            if inputs else []
        it = iter(grads)
        g1 = next(it) if lp.requires_grad else None
        g2 = next(it) if p2.requires_grad else None
        if ctx.needs_input_grad[1]:
            g2 = torch.zeros_like(p2) if g2 is None else g2.contiguous()
            _all_reduce(g2, dist.ReduceOp.SUM, ctx.group)
        else:
            g2 = None
        if not ctx.needs_input_grad[0]:
            g1 = None
        elif g1 is not None and ctx.full:
            g1 = _all_gather_points(g1.contiguous(), ctx.sizes, ctx.group)
        return g1, g2, None, None, None, None, None


def sharded_sided_distance(local_p1, p2, group=None):
    r"""sided_distance(p1, p2) with p1's points split over the ranks of ``group``.

    ``local_p1`` (B, n_r, 3) is this rank's contiguous share of p1's points
    (``shard_bounds(N, rank, world)``), ``p2`` (B,M,3) is the same on every rank.  Returns the
    whole (dist (B,N), idx (B,N) int64) on every rank.  Gradients: ``local_p1`` gets its rows;
    ``p2`` gets the sum over every rank's points, formed from the ranks' double sums of the
    per-point float terms and rounded once (GPU, float32 / float64), which is the unsharded
    backward's (itself a double sum rounded once, _C.sided_distance_backward_cuda) up to the
    documented one-ulp allowance."""
    if not _active():
        from .metrics.pointcloud import sided_distance
        return sided_distance(local_p1, p2)
    sizes = _sizes(local_p1.shape[1], local_p1.device, group)
    lo = sum(sizes[:_rank(group)])
    return _ShardedSided.apply(local_p1, p2, lo, lo + local_p1.shape[1], sizes, group, False)


def sharded_chamfer_distance(p1, p2, w1=1., w2=1., squared=True, group=None):
    r"""chamfer_distance (reference metrics/pointcloud.py:89-136) over the ranks of ``group``; both
    clouds are the whole (B,N,3) / (B,M,3) on every rank.  The p1 -> p2 direction splits p1's
    points, the p2 -> p1 direction splits p2's (``sharded_sided_distance``'s scheme); the gathered
    distances go through the reference's means, so every rank holds the unsharded distance, and
    both clouds' whole gradients (split rows all-gathered, replicated terms all-reduced as double
    sums)."""
    from .metrics.pointcloud import chamfer_distance, _chamfer_from_sided
    world, rank = _world(group), _rank(group)
    if not _active():
        return chamfer_distance(p1, p2, w1, w2, squared)
    n, m = p1.shape[1], p2.shape[1]
    lo1, hi1 = shard_bounds(n, rank, world)
    lo2, hi2 = shard_bounds(m, rank, world)
    sdist1 = _ShardedSided.apply(p1, p2, lo1, hi1, _split_sizes(n, world), group, True)[0]
    sdist2 = _ShardedSided.apply(p2, p1, lo2, hi2, _split_sizes(m, world), group, True)[0]
    return _chamfer_from_sided(sdist1, sdist2, w1, w2, squared)


def sharded_point_to_mesh_distance(local_points, face_vertices, group=None):
    r"""point_to_mesh_distance of one (P,3) cloud against (F,3,3) triangles with the
    points split over the ranks of ``group``.

    ``local_points`` is this rank's contiguous share (``shard_bounds(P, rank, world)``
    rows of the cloud); ``face_vertices`` is the same on every rank.  Returns the whole
    cloud's (dist (P), face_idx (P) int64, dist_type (P) int32) on every rank.  Gradients:
    ``local_points`` gets the rows of its share; ``face_vertices`` gets the sum over every
    rank's points.  On the GPU that sum is formed from the ranks' double sums of the per-point
    float terms and rounded once: the unsharded gradient, for float32 inputs bit for bit up to the
    documented one-ulp allowance of summation order (float64 terms do not add exactly in double,
    so there the two agree to the last bits only).  On the CPU (the
    reference's torch path, whose autograd sums in float) the ranks' float gradients are added:
    equal to the unsharded gradient up to float summation order.
    """
    if not _active():
        from .metrics.trianglemesh import point_to_mesh_distance
        d, i, t = point_to_mesh_distance(local_points.unsqueeze(0), face_vertices.unsqueeze(0))
        return d[0], i[0], t[0]
    sizes = _sizes(local_points.shape[0], local_points.device, group)
    return _ShardedP2M.apply(local_points, face_vertices, sizes, group)


def sharded_unbatched_raytrace(octree, point_hierarchy, pyramid, exsum, origin, direction, level,
                               return_depth=True, with_exit=False, group=None):
    r"""unbatched_raytrace with the rays split contiguously over the ranks of ``group``.

    Every argument is the unsharded call's (the rays replicated on every rank; the rank marches
    rows ``shard_bounds(N, rank, world)`` of them).  Returns the unsharded call's outputs on every
    rank: ray_index (offset by each shard's first ray), point_index and the depths, all-gathered
    with the per-rank nugget counts -- the reference's ray-major order is the rank order."""
    from .render.spc.raytrace import unbatched_raytrace
    world, rank = _world(group), _rank(group)
    lo, hi = shard_bounds(origin.shape[0], rank, world)
    out = unbatched_raytrace(octree, point_hierarchy, pyramid, exsum, origin[lo:hi], direction[lo:hi], level,
                             return_depth=return_depth, with_exit=with_exit)
    if not _active():
        return out
    ridx = out[0] + lo
    sizes = _sizes(ridx.shape[0], ridx.device, group)
    nug = _all_gather_rows(torch.stack([ridx, out[1].to(ridx.dtype)], -1), sizes, group)
    res = (nug[:, 0].contiguous(), nug[:, 1].contiguous().to(out[1].dtype))
    if return_depth:
        res = res + (_all_gather_rows(out[2].contiguous(), sizes, group),)
    return res


def sharded_trianglemeshes_to_voxelgrids(vertices, faces, resolution, origin=None, scale=None, split='auto',
                                         group=None):
    r"""trianglemeshes_to_voxelgrids (dense grids) over the ranks of ``group``; every argument is
    the unsharded call's, replicated.  ``split``: 'batch' (each rank converts a contiguous share of
    the meshes; the grids are all-gathered), 'faces' (each rank converts every mesh with a
    contiguous share of the faces; the grids are OR-reduced as bit grids), or 'auto' ('batch' when there are
    at least as many meshes as ranks).  The default origin / scale are the whole mesh's (computed
    before splitting, so every shard normalises the same way).  Returns the unsharded (B,R,R,R)
    grid on every rank."""
    from .ops.conversions.trianglemesh import trianglemeshes_to_voxelgrids
    world, rank = _world(group), _rank(group)
    if not _active():
        return trianglemeshes_to_voxelgrids(vertices, faces, resolution, origin, scale)
    if origin is None:
        origin = torch.min(vertices, dim=1)[0]
    if scale is None:
        scale = torch.max(torch.max(vertices, dim=1)[0] - origin, dim=1)[0]
    B = vertices.shape[0]
    if split == 'auto':
        split = 'batch' if B >= world else 'faces'
    if split == 'batch':
        lo, hi = shard_bounds(B, rank, world)
        grid = trianglemeshes_to_voxelgrids(vertices[lo:hi], faces, resolution, origin[lo:hi], scale[lo:hi])
        return _all_gather_rows(grid, [b - a for a, b in (shard_bounds(B, r, world) for r in range(world))], group)
    if split != 'faces':
        raise ValueError(f"split must be 'auto', 'batch' or 'faces', got {split!r}")
    lo, hi = shard_bounds(faces.shape[0], rank, world)
    grid = trianglemeshes_to_voxelgrids(vertices, faces[lo:hi], resolution, origin, scale)
    bits = _or_all_reduce(_pack_bits(grid), group)
    return _unpack_bits(bits, grid)


_BIT_WEIGHTS = {}


def _bit_weights(device):
    w = _BIT_WEIGHTS.get(device)
    if w is None:
        w = _BIT_WEIGHTS[device] = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=device)
    return w


def _pack_bits(grid):
    """Occupancy (non-zero) of a dense grid as bits, 8 cells per byte in memory order."""
    flat = grid.reshape(-1) != 0
    pad = (-flat.numel()) % 8
    if pad:
        flat = torch.cat([flat, flat.new_zeros(pad)])
    return (flat.view(-1, 8).to(torch.uint8) * _bit_weights(grid.device)).sum(-1, dtype=torch.uint8)


def _unpack_bits(bits, like):
    """The grid of `like`'s shape and dtype holding 1 where `bits` is set, else 0."""
    cells = (bits.unsqueeze(-1) & _bit_weights(bits.device)) != 0
    return cells.reshape(-1)[:like.numel()].reshape(like.shape).to(like.dtype)


def _or_all_reduce(bits, group):
    """Bitwise OR of a uint8 vector over the ranks: a reduce-scatter by hand (all_to_all of the
    world's slices, OR of the copies of this rank's slice) and an all_gather of the slices."""
    world = _world(group)
    n = bits.numel()
    chunk = -(-n // world)
    buf = bits.new_zeros(world * chunk)
    buf[:n] = bits
    recv = torch.empty_like(buf)
    _all_to_all(recv, buf, group)
    part = recv.view(world, chunk)
    mine = part[0].clone()
    for r in range(1, world):
        mine |= part[r]
    out = torch.empty_like(buf)
    _all_gather_flat(out, mine, group)
    return out[:n]
