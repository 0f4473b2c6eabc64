"""Multi-GPU sharding of the hot path: one process per GPU, RCCL over xGMI.

Kaolin itself is single-device; these helpers are what a data-parallel caller of its ops
runs on every rank.  Nothing here changes an op's arithmetic: a shard's outputs are the
unsharded op's outputs for those rows, bit for bit.

* DIB-R: views are independent, so a rank renders a contiguous slice of them
  (``shard_bounds`` over the view count) with the mesh replicated; the caller gathers
  per-shard losses (``gather_losses``).
* point_to_mesh_distance on one large cloud: the points are split contiguously over the
  ranks (``shard_bounds``), the faces are replicated.  ``sharded_point_to_mesh_distance``
  evaluates the rank's points and all-gathers (dist, face_idx, dist_type) so every rank
  holds the whole result.  In the backward the rank's points get their gradient locally
  and the face gradient, a sum over all points, is all-reduced.
"""
import torch
import torch.distributed as dist

__all__ = ['shard_bounds', 'gather_losses', 'sharded_point_to_mesh_distance']


def shard_bounds(n, rank, world):
    """[lo, hi) of rank's contiguous share of n items; shares differ by at most one and
    are in rank order, so concatenating them in rank order restores the original order."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def gather_losses(loss, group=None):
    """All-gather one scalar loss per rank -> (world,) in rank order."""
    world = _world(group)
    if world == 1:
        return loss.detach().reshape(1)
    out = [torch.empty_like(loss) for _ in range(world)]
    dist.all_gather(out, loss.detach(), group=group)
    return torch.stack(out)


def _all_gather_rows(t, sizes, group):
    """Concatenate every rank's (n_r, ...) tensor in rank order (rows padded to the
    largest share for the collective, then trimmed)."""
    world = len(sizes)
    m = max(sizes)
    if t.shape[0] < m:
        t = torch.cat([t, t.new_zeros((m - t.shape[0],) + tuple(t.shape[1:]))])
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t.contiguous(), group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


class _ShardedP2M(torch.autograd.Function):

    @staticmethod
    def forward(ctx, local_points, face_vertices, sizes, group):
        from .metrics.trianglemesh import point_to_mesh_distance
        with torch.enable_grad():
            lp = local_points.detach().requires_grad_(local_points.requires_grad)
            fv = face_vertices.detach().requires_grad_(face_vertices.requires_grad)
            d, i, t = point_to_mesh_distance(lp.unsqueeze(0), fv.unsqueeze(0))
        ctx.local = (lp, fv, d)  # the shard's own graph, replayed by backward
        ctx.sizes, ctx.group = sizes, group
        out_i, out_t = _all_gather_rows(i[0], sizes, group), _all_gather_rows(t[0], sizes, group)
        ctx.mark_non_differentiable(out_i, out_t)
        return _all_gather_rows(d[0].detach(), sizes, group), out_i, out_t

    @staticmethod
    def backward(ctx, g_dist, g_idx, g_type):
        lp, fv, d = ctx.local
        rank = dist.get_rank(ctx.group)
        lo = sum(ctx.sizes[:rank])
        g_local = g_dist[lo:lo + ctx.sizes[rank]].reshape(1, -1).contiguous()
        inputs = [x for x in (lp, fv) if x.requires_grad]
        grads = torch.autograd.grad(d, inputs, g_local, allow_unused=True) if inputs else []
        it = iter(grads)
        g_lp = next(it) if lp.requires_grad else None
        g_fv = next(it) if fv.requires_grad else None
        if g_fv is not None:
            g_fv = g_fv.contiguous()
            dist.all_reduce(g_fv, op=dist.ReduceOp.SUM, group=ctx.group)
        return g_lp, g_fv, None, None


def sharded_point_to_mesh_distance(local_points, face_vertices, group=None):
    r"""point_to_mesh_distance of one (P,3) cloud against (F,3,3) triangles with the
    points split over the ranks of ``group``.

    ``local_points`` is this rank's contiguous share (``shard_bounds(P, rank, world)``
    rows of the cloud); ``face_vertices`` is the same on every rank.  Returns the whole
    cloud's (dist (P), face_idx (P) int64, dist_type (P) int32) on every rank.  Gradients:
    ``local_points`` gets the rows of its share; ``face_vertices`` gets the sum over every
    rank's points (an all_reduce), i.e. the unsharded gradient.
    """
    world = _world(group)
    if world == 1:
        from .metrics.trianglemesh import point_to_mesh_distance
        d, i, t = point_to_mesh_distance(local_points.unsqueeze(0), face_vertices.unsqueeze(0))
        return d[0], i[0], t[0]
    n = torch.tensor([local_points.shape[0]], dtype=torch.int64, device=local_points.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    sizes = [int(x) for x in ns]
    return _ShardedP2M.apply(local_points, face_vertices, sizes, group)
