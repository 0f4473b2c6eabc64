"""Morton code helpers (kaolin/ops/spc/points.py:31-131) over the HIP path.

points_to_morton / morton_to_points call the reference's _C names
(``_C.ops.spc.points_to_morton_cuda`` / ``morton_to_points_cuda``, point_utils.cpp:36-64),
which are HIP kernels here (spc.hip).  Like the reference they need GPU tensors.
"""
import torch

from ... import _C


def quantize_points(x, level):
    r"""Float coordinates in [-1, 1] -> int16 grid points of ``level`` (points.py:31-48)."""
    res = 2 ** level
    return torch.floor(torch.clamp(res * (x + 1.0) / 2.0, 0, res - 1.)).short()


def points_to_morton(points):
    r"""int16 (..., 3) -> int64 (...) morton codes (bit 3i+2 = x_i, 3i+1 = y_i, 3i = z_i)."""
    shape = list(points.shape)[:-1]
    return _C.ops.spc.points_to_morton_cuda(points.reshape(-1, 3).contiguous()).reshape(*shape)


def morton_to_points(morton):
    r"""int64 (...) morton codes -> int16 (..., 3) points."""
    shape = list(morton.shape) + [3]
    return _C.ops.spc.morton_to_points_cuda(morton.reshape(-1).contiguous()).reshape(*shape)


def unbatched_points_to_octree(points, level, sorted=False):
    r"""Octree of the quantized points (N,3) int16 at ``level`` (points.py:50-77).  With
    ``sorted=False`` the points are deduplicated and put in morton order first."""
    if not sorted:
        unique = torch.unique(points.contiguous(), dim=0).contiguous()
        morton = torch.sort(points_to_morton(unique).contiguous())[0]
        points = morton_to_points(morton.contiguous())
    return _C.ops.spc.points_to_octree(points.contiguous(), level)
