"""unbatched_raytrace and the packed ray ops (kaolin/render/spc/raytrace.py:31-296) over the HIP path.

The autograd rules are the reference's: sum_reduce's backward gathers the pack gradient
back onto its rows, cumsum's is the reverse-direction cumsum, cumprod's is the
reverse cumsum of prod * grad divided by feats with NaNs zeroed (the TensorFlow rule,
raytrace.py:169-185); exponential_integration is the reference's cumsum reformulation.
"""
import torch

from ... import _C

__all__ = ['unbatched_raytrace', 'mark_pack_boundaries', 'mark_first_hit', 'diff', 'sum_reduce', 'cumsum',
           'cumprod', 'exponential_integration']


def unbatched_raytrace(octree, point_hierarchy, pyramid, exsum, origin, direction, level,
                       return_depth=True, with_exit=False, capacity=None):
    r"""Ray march an unbatched SPC ([-1, 1]^3) at ``level``.  Returns ray_index,
    point_index (int32, ray-major, front-to-back) and optionally the entry (and exit)
    depth (N,1) / (N,2).

    ``capacity`` (an extension; the reference sizes the output on the host, one count read per
    level, raytrace_cuda.cu:557-560): fixed-size outputs of ``capacity`` rows and nothing read
    back, so the call can be captured into a CUDA/HIP graph.  Then a fourth (third without depth)
    value is returned, ``result`` (2,) int64 on the device = (rows written, 1 if the march held
    more than ``capacity`` nuggets at some level).  The rows written are always the first
    result[0] rows of the full answer; after a truncation (result[1] == 1) result[0] <= capacity --
    a level truncated early can lose descendants that later levels would have culled anyway, so
    fewer than ``capacity`` rows may come back.  Rows past result[0] hold index -1 and depth 0."""
    if capacity is not None:
        out = _C.render.spc.raytrace_fixed_cuda(octree.contiguous(), point_hierarchy.contiguous(),
                                                 pyramid.contiguous(), exsum.contiguous(), origin.contiguous(),
                                                 direction.contiguous(), level, return_depth, with_exit, capacity)
        ridx, pidx = out[0][..., 0], out[0][..., 1]
        return (ridx, pidx, out[1], out[2]) if return_depth else (ridx, pidx, out[1])
    output = _C.render.spc.raytrace_cuda(octree.contiguous(), point_hierarchy.contiguous(), pyramid.contiguous(),
                                         exsum.contiguous(), origin.contiguous(), direction.contiguous(), level,
                                         return_depth, with_exit)
    nuggets = output[0]
    ray_index = nuggets[..., 0]
    point_index = nuggets[..., 1]
    if return_depth:
        return ray_index, point_index, output[1]
    return ray_index, point_index


def mark_pack_boundaries(pack_ids):
    r"""Boolean mask, True at the first element of every run of equal (sorted) ids."""
    return _C.render.spc.mark_pack_boundaries_cuda(pack_ids.contiguous()).bool()


def mark_first_hit(ridx):
    r"""Deprecated alias of mark_pack_boundaries (raytrace.py:130-143)."""
    return mark_pack_boundaries(ridx)


def _pack_starts(boundaries):
    """Row indices of the True entries (the pack starts), int32 as the scans take them."""
    return torch.nonzero(boundaries).int().contiguous()[..., 0]


def diff(feats, boundaries):
    r"""Per-pack forward difference ``out[i] = feats[i+1] - feats[i]``, 0 on each pack's last
    row (raytrace.py:146-171).  feats (num_rays, num_feats) or any (..., num_feats)."""
    shape = feats.shape
    dim = shape[-1]
    starts = torch.nonzero(boundaries).contiguous()[..., 0]
    return _C.render.spc.diff_cuda(feats.reshape(-1, dim).contiguous(), starts.contiguous()).reshape(*shape)


class SumReduce(torch.autograd.Function):
    """raytrace.py:173-188."""

    @staticmethod
    def forward(ctx, feats, info):
        inclusive_sum = _C.render.spc.inclusive_sum_cuda(info.int().contiguous())
        ctx.save_for_backward(inclusive_sum)
        return _C.render.spc.sum_reduce_cuda(feats, inclusive_sum)

    @staticmethod
    def backward(ctx, grad_output):
        inclusive_sum, = ctx.saved_tensors
        grad_feats = grad_output[(inclusive_sum - 1).long()] if ctx.needs_input_grad[0] else None
        return grad_feats, None


class Cumsum(torch.autograd.Function):
    """raytrace.py:212-228."""

    @staticmethod
    def forward(ctx, feats, info, exclusive, reverse):
        starts = _pack_starts(info)
        ctx.save_for_backward(starts)
        ctx.flags = (exclusive, reverse)
        return _C.render.spc.cumsum_cuda(feats, starts, exclusive, reverse)

    @staticmethod
    def backward(ctx, grad_output):
        starts, = ctx.saved_tensors
        exclusive, reverse = ctx.flags
        return _C.render.spc.cumsum_cuda(grad_output.contiguous(), starts, exclusive, not reverse), None, None, None


class Cumprod(torch.autograd.Function):
    """raytrace.py:190-210."""

    @staticmethod
    def forward(ctx, feats, info, exclusive, reverse):
        starts = _pack_starts(info)
        prod = _C.render.spc.cumprod_cuda(feats, starts, exclusive, reverse)
        ctx.save_for_backward(feats, starts, prod)
        ctx.flags = (exclusive, reverse)
        return prod

    @staticmethod
    def backward(ctx, grad_output):
        feats, starts, prod = ctx.saved_tensors
        exclusive, reverse = ctx.flags
        out = _C.render.spc.cumsum_cuda((prod * grad_output).contiguous(), starts, exclusive, not reverse)
        grad_feats = None
        if ctx.needs_input_grad[0]:
            grad_feats = out / feats  # approximate gradient, as TensorFlow's
            grad_feats[grad_feats.isnan()] = 0
        return grad_feats, None, None, None


def sum_reduce(feats, boundaries):
    r"""Sum of each pack's rows: (num_packs, num_feats) (raytrace.py:230-243)."""
    return SumReduce.apply(feats.contiguous(), boundaries.contiguous())


def cumsum(feats, boundaries, exclusive=False, reverse=False):
    r"""Per-pack cumulative sum, tf.math.cumsum's exclusive / reverse options (raytrace.py:245-264)."""
    return Cumsum.apply(feats.contiguous(), boundaries.contiguous(), exclusive, reverse)


def cumprod(feats, boundaries, exclusive=False, reverse=False):
    r"""Per-pack cumulative product, tf.math.cumprod's options; the backward zeroes NaNs
    (raytrace.py:266-290)."""
    return Cumprod.apply(feats.contiguous(), boundaries.contiguous(), exclusive, reverse)


def exponential_integration(feats, tau, boundaries, exclusive=True):
    r"""Beer-Lambert integration along packs (raytrace.py:292-330): transmittance
    ``exp(-cumsum(tau)) * (1 - exp(-tau))`` and the per-pack sum of ``transmittance * feats``.
    Returns (integrated feats (num_packs, num_feats), transmittance (num_rays, 1))."""
    tau = tau.contiguous()
    alpha = 1.0 - torch.exp(-tau)
    transmittance = torch.exp(-1.0 * cumsum(tau, boundaries.contiguous(), exclusive=exclusive)) * alpha
    feats_out = sum_reduce(transmittance * feats.contiguous(), boundaries.contiguous())
    return feats_out, transmittance
