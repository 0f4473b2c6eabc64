"""Morton code helpers (kaolin/ops/spc/points.py, spc_math.h:93-121) in vectorised torch integer ops."""
import torch

from ... import _C


def points_to_morton(points):
    r"""int16 (N,3) -> int64 morton codes (bit 3i+2 = x_i, 3i+1 = y_i, 3i = z_i)."""
    p = points.to(torch.int64) & 0xFFFF
    m = torch.zeros(points.shape[:-1], dtype=torch.int64, device=points.device)
    for i in range(15):
        m |= ((p[..., 2] >> i) & 1) << (3 * i)
        m |= ((p[..., 1] >> i) & 1) << (3 * i + 1)
        m |= ((p[..., 0] >> i) & 1) << (3 * i + 2)
    return m


def morton_to_points(morton):
    r"""int64 morton codes -> int16 (N,3) points."""
    out = torch.zeros(morton.shape + (3,), dtype=torch.int64, device=morton.device)
    for i in range(15):
        out[..., 0] |= ((morton >> (3 * i + 2)) & 1) << i
        out[..., 1] |= ((morton >> (3 * i + 1)) & 1) << i
        out[..., 2] |= ((morton >> (3 * i)) & 1) << i
    return out.to(torch.int16)


def unbatched_points_to_octree(points, level, sorted=False):
    r"""Octree of the unique quantized points (N,3) int16 at ``level``."""
    morton = points_to_morton(points.contiguous())
    if not sorted:
        morton = torch.sort(morton)[0]
    morton = torch.unique_consecutive(morton)
    return _C.ops.spc.morton_to_octree(morton, level)
