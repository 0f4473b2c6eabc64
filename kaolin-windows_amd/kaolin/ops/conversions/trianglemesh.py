"""trianglemeshes_to_voxelgrids / unbatched_mesh_to_spc (kaolin/ops/conversions/trianglemesh.py:29-140)
over the HIP path."""
import ctypes

import torch

from ... import _C
from ... import _native as N

__all__ = ['trianglemeshes_to_voxelgrids', 'unbatched_mesh_to_spc']


def trianglemeshes_to_voxelgrids(vertices, faces, resolution, origin=None, scale=None, return_sparse=False):
    r"""Surface voxelgrids (B,R,R,R) of meshes: vertices are normalised by
    ``(v - origin) / scale`` (defaults: per-mesh min and max extent), triangles are
    recursively split until every edge is <= (R-1)/R^2, and every generated vertex is
    rounded to the grid (trianglemesh.py:29-110).  GPU tensors only."""
    if not isinstance(resolution, int):
        raise TypeError(f"Expected resolution to be int but got {type(resolution)}.")
    N.require_gpu('trianglemeshes_to_voxelgrids', vertices, faces)
    if origin is None:
        origin = torch.min(vertices, dim=1)[0]
    if scale is None:
        scale = torch.max(torch.max(vertices, dim=1)[0] - origin, dim=1)[0]
    batch_size = vertices.shape[0]
    out_dtype = vertices.dtype
    work = vertices if vertices.dtype in (torch.float32, torch.float64) else vertices.float()
    points = ((work - origin.to(work.dtype).unsqueeze(1)) / scale.to(work.dtype).view(-1, 1, 1)).contiguous()
    faces = faces.to(torch.int64).contiguous()
    R = resolution
    grid_dtype = out_dtype if not return_sparse else torch.float32
    grid = torch.zeros((batch_size, R, R, R), dtype=grid_dtype, device=vertices.device)
    lib = N.lib()
    fn = lib.kl_voxelgrid_mark if work.dtype == torch.float32 else lib.kl_voxelgrid_mark_f64
    dev = vertices.device
    with torch.cuda.device(dev):
        for i in range(batch_size):
            arena = N.Arena(dev)
            N.check(fn(points.shape[1], N.ptr(points[i]), faces.shape[0], N.ptr(faces), R,
                       N.dtype_code(grid_dtype), N.ptr(grid[i]), arena.fn, None, N.stream_of(dev)),
                    'trianglemeshes_to_voxelgrids')
    if return_sparse:
        return grid.to_sparse()
    return grid


def unbatched_mesh_to_spc(face_vertices, level):
    r"""Conservative voxelisation of a mesh in [-1, 1]^3 to an SPC of ``level`` levels.
    Returns (octree u8, face_idx int64 per leaf, barycentric (num_leaves, 2) f32)."""
    if face_vertices.shape[-1] != 3:
        raise NotImplementedError("unbatched_mesh_to_spc is only implemented for triangle meshes")
    return _C.ops.conversions.mesh_to_spc_cuda(face_vertices.contiguous(), level)
