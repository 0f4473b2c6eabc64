"""check_sign (reference kaolin/ops/mesh/check_sign.py:25-154).

Same API and argument errors as the reference.  The GPU path is one HIP launch for the whole
batch (csrc/checksign.hip): the kernel gathers each face's corners from (verts, faces) and
applies the reference's ``/ maxlen`` normalisation on load, instead of the reference's
per-mesh Python loop of ``index_select`` gathers and ``unbatched_mesh_intersection_cuda``
calls.  The reference's CPU path (a Cython triangle hash) is not provided: CPU tensors raise.
"""
import torch

from ... import _C
from ... import _native as N

__all__ = ['check_sign', '_unbatched_check_sign_cuda']


def _unbatched_check_sign_cuda(verts, faces, points):
    """check_sign.py:25-35 (one mesh, already normalised)."""
    points = points.contiguous()
    v1 = torch.index_select(verts, 0, faces[:, 0]).view(-1, 3).contiguous()
    v2 = torch.index_select(verts, 0, faces[:, 1]).view(-1, 3).contiguous()
    v3 = torch.index_select(verts, 0, faces[:, 2]).view(-1, 3).contiguous()
    ints = _C.ops.mesh.unbatched_mesh_intersection_cuda(points, v1, v2, v3)
    return ints % 2 == 1.


def check_sign(verts, faces, points, hash_resolution=512):
    r"""Checks if a set of points is contained inside a watertight triangle mesh, by the parity
    of the number of mesh faces a ray from each point toward +x crosses.

    Args:
        verts (torch.Tensor): (B, V, 3) vertices.
        faces (torch.LongTensor): (F, 3) faces.
        points (torch.Tensor): (B, P, 3) points to check.
        hash_resolution (int): used only by the reference's CPU path (not provided here).

    Returns:
        (torch.BoolTensor): (B, P), True where the point is inside the mesh.
    """
    assert verts.device == points.device
    assert faces.device == points.device
    if not faces.dtype == torch.int64:
        raise TypeError(f"Expected faces entries to be torch.int64 but got {faces.dtype}.")
    if not isinstance(hash_resolution, int):
        raise TypeError(f"Expected hash_resolution to be int but got {type(hash_resolution)}.")
    if verts.ndim != 3:
        raise ValueError(f"Expected verts to have 3 dimensions but got {verts.ndim} dimensions.")
    if faces.ndim != 2:
        raise ValueError(f"Expected faces to have 2 dimensions but got {faces.ndim} dimensions.")
    if points.ndim != 3:
        raise ValueError(f"Expected points to have 3 dimensions but got {points.ndim} dimensions.")
    if verts.shape[2] != 3:
        raise ValueError(f"Expected verts to have 3 coordinates but got {verts.shape[2]} coordinates.")
    if faces.shape[1] != 3:
        raise ValueError(f"Expected faces to have 3 vertices but got {faces.shape[1]} vertices.")
    if points.shape[2] != 3:
        raise ValueError(f"Expected points to have 3 coordinates but got {points.shape[2]} coordinates.")
    N.require_gpu('check_sign', verts, faces, points)
    if verts.dtype not in (torch.float32, torch.float64) or points.dtype != verts.dtype:
        raise RuntimeError(f'check_sign: expected float or double verts and points of the same dtype, '
                           f'got {verts.dtype} and {points.dtype}')
    # check_sign.py:140-146: the largest bbox extent of each mesh, taken by the library on the
    # device (kl_voxelgrid_bounds: exact min / max, NaN propagated as torch's reductions do);
    # torch's reductions only for a mesh without vertices, where they raise as the reference's
    maxlen = None
    if verts.shape[1] == 0:
        vmax = verts.max(dim=1)[0]
        vmin = verts.min(dim=1)[0]
        maxlen = (vmax - vmin).max(dim=1)[0].contiguous()
    return _C.check_sign_batched(verts.contiguous(), faces.contiguous(), points.contiguous(), maxlen)
