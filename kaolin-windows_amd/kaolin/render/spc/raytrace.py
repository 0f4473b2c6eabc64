"""unbatched_raytrace / mark_pack_boundaries (kaolin/render/spc/raytrace.py:31-130) over the HIP path."""
from ... import _C

__all__ = ['unbatched_raytrace', 'mark_pack_boundaries', 'mark_first_hit']


def unbatched_raytrace(octree, point_hierarchy, pyramid, exsum, origin, direction, level,
                       return_depth=True, with_exit=False):
    r"""Ray march an unbatched SPC ([-1, 1]^3) at ``level``.  Returns ray_index,
    point_index (int32, ray-major, front-to-back) and optionally the entry (and exit)
    depth (N,1) / (N,2)."""
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
