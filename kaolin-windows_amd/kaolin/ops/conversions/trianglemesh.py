"""trianglemeshes_to_voxelgrids / unbatched_mesh_to_spc (kaolin/ops/conversions/trianglemesh.py:29-140)
over the HIP path."""
import ctypes

import torch

from ... import _C
from ... import _native as N

__all__ = ['trianglemeshes_to_voxelgrids', 'unbatched_mesh_to_spc']

# True: the subdivision sized on the host (kl_voxelgrid_mark, one count read per round) instead of
# the device-counted kl_voxelgrid_mark_async; the two grids are equal (tests / bench compare them)
HOST_SIZED = False


def trianglemeshes_to_voxelgrids(vertices, faces, resolution, origin=None, scale=None, return_sparse=False):
    r"""Surface voxelgrids (B,R,R,R) of meshes: vertices are normalised by
    ``(v - origin) / scale`` (defaults: per-mesh min and max extent), triangles are
    recursively split until every edge is <= (R-1)/R^2, and every generated vertex is
    rounded to the grid (trianglemesh.py:29-110).  GPU tensors run the HIP subdivision
    (voxel.hip); CPU tensors the torch path below, as the reference is device-agnostic."""
    if not isinstance(resolution, int):
        raise TypeError(f"Expected resolution to be int but got {type(resolution)}.")
    if not vertices.is_cuda:
        return _voxelgrids_cpu(vertices, faces, resolution, origin, scale, return_sparse)
    N.require_gpu('trianglemeshes_to_voxelgrids', vertices, faces)
    if (origin is None or scale is None) and vertices.dtype in (torch.float32, torch.float64) \
            and vertices.shape[1] > 0:
        # the reference's torch.min / torch.max defaults (trianglemesh.py:74-77) in one reduction
        vc = vertices.contiguous()
        B = vc.shape[0]
        o = torch.empty((B, 3), dtype=vc.dtype, device=vc.device)
        sc = torch.empty((B,), dtype=vc.dtype, device=vc.device)
        nb = N.lib().kl_voxelgrid_bounds_workspace_bytes(B)
        ws = torch.empty(nb, dtype=torch.uint8, device=vc.device)
        with N.on_device(vc.device):
            N.check(N.lib().kl_voxelgrid_bounds(N.dtype_code(vc.dtype), B, vc.shape[1], N.ptr(vc), N.ptr(o), N.ptr(sc),
                                                N.ptr(ws), nb, N.stream_of(vc.device)), 'trianglemeshes_to_voxelgrids')
        if origin is None:
            origin = o
        if scale is None:
            scale = torch.max(torch.max(vertices, dim=1)[0] - origin, dim=1)[0] if origin is not o else sc
    if origin is None:
        origin = torch.min(vertices, dim=1)[0]
    if scale is None:
        scale = torch.max(torch.max(vertices, dim=1)[0] - origin, dim=1)[0]
    batch_size = vertices.shape[0]
    out_dtype = vertices.dtype
    work = vertices if vertices.dtype in (torch.float32, torch.float64) else vertices.float()
    faces = faces.to(torch.int64).contiguous()
    R = resolution
    grid_dtype = out_dtype if not return_sparse else torch.float32
    lib = N.lib()
    dev = vertices.device
    if HOST_SIZED and not N.capturing(dev):
        points = ((work - origin.to(work.dtype).unsqueeze(1)) / scale.to(work.dtype).view(-1, 1, 1)).contiguous()
        grid = torch.zeros((batch_size, R, R, R), dtype=grid_dtype, device=dev)
        fn = lib.kl_voxelgrid_mark if work.dtype == torch.float32 else lib.kl_voxelgrid_mark_f64
        with N.on_device(dev):
            for i in range(batch_size):
                arena = N.Arena(dev)
                N.check(fn(points.shape[1], N.ptr(points[i]), faces.shape[0], N.ptr(faces), R,
                           N.dtype_code(grid_dtype), N.ptr(grid[i]), arena.fn, None, N.stream_of(dev)),
                        'trianglemeshes_to_voxelgrids')
    else:
        # nothing read back per round (graph-capturable); one status read per call in eager mode.
        # (r06) kl_voxelgrid_async zero-fills each grid and normalises the vertices in its kernels
        # ((v - origin) / scale, rounded as the tensor expression above): no normalised copy, no zeros
        F = faces.shape[0]
        # ping-pong triangle buffers (2 x cap x 9 coordinates): capped at 2^23 triangles (0.6 GB in
        # f32) -- work past the cap is finished depth-first by the thread holding it, same grid
        cap = min(max(16 * F, 1 << 20), 1 << 23)
        code = N.dtype_code(work.dtype)
        verts = work.contiguous()
        org = origin.to(device=dev, dtype=work.dtype).reshape(-1, 3).expand(batch_size, 3).contiguous()
        scl = scale.to(device=dev, dtype=work.dtype).reshape(-1).expand(batch_size).contiguous()
        grid = torch.empty((batch_size, R, R, R), dtype=grid_dtype, device=dev)
        nb = lib.kl_voxelgrid_mark_async_workspace_bytes(code, cap)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        status = torch.empty(max(batch_size, 1), dtype=torch.int32, device=dev)
        with N.on_device(dev):
            for i in range(batch_size):
                N.check(lib.kl_voxelgrid_async(code, verts.shape[1], N.ptr(verts[i]), N.ptr(org[i]), N.ptr(scl[i:]),
                                               F, N.ptr(faces), R, N.dtype_code(grid_dtype), N.ptr(grid[i]), cap,
                                               N.ptr(status[i:]), N.ptr(ws), nb, N.stream_of(dev)),
                        'trianglemeshes_to_voxelgrids')
        if not N.capturing(dev) and batch_size > 0:
            st = 0
            for v in status.cpu().tolist():  # one device-to-host read
                st |= v
            if st & 1:
                raise RuntimeError('trianglemeshes_to_voxelgrids: a triangle needs more than 2^20 subdivisions '
                                   '(vertices far outside the unit cube after origin / scale?)')
            if st & 4:
                raise RuntimeError('trianglemeshes_to_voxelgrids: the subdivision kernel\'s workgroups could not '
                                   'all be resident (GPU shared with other work?); grid incomplete')
    if return_sparse:
        return grid.to_sparse()
    return grid


def _mark_grid(grid, pts, R):
    """Set the voxels of the grid points nearest to pts (round half to even), dropping
    those outside [0, R-1] (pointcloud.py:22-75)."""
    q = torch.round(pts * (R - 1)).long()
    inside = ((q >= 0) & (q <= R - 1)).all(1)
    q = q[inside]
    grid[q[:, 0], q[:, 1], q[:, 2]] = 1


def _voxelgrids_cpu(vertices, faces, R, origin, scale, return_sparse):
    """CPU path.  Per mesh: every vertex and every edge midpoint generated by splitting
    triangles into 4 while their longest squared edge exceeds ((R-1)/R^2)^2 is rounded onto
    the grid (trianglemesh.py:339-457).  The midpoints are marked as they are made, so the
    reference's per-round torch.unique over the growing vertex set is not needed: the
    marked set is the same."""
    if origin is None:
        origin = torch.min(vertices, dim=1)[0]
    if scale is None:
        scale = torch.max(torch.max(vertices, dim=1)[0] - origin, dim=1)[0]
    assert R > 1
    thr = ((R - 1) / (R ** 2)) ** 2
    pts_all = (vertices - origin.unsqueeze(1)) / scale.view(-1, 1, 1)
    grid = torch.zeros((vertices.shape[0], R, R, R), dtype=vertices.dtype)
    faces = faces.long()
    for b in range(vertices.shape[0]):
        pts = pts_all[b]
        _mark_grid(grid[b], pts, R)
        a, c, e = pts[faces[:, 0]], pts[faces[:, 1]], pts[faces[:, 2]]
        while a.shape[0] > 0:
            lens = torch.stack([torch.sum((a - c) ** 2, dim=1), torch.sum((c - e) ** 2, dim=1),
                                torch.sum((e - a) ** 2, dim=1)], 1)
            split = torch.max(lens, dim=1)[0] > thr
            a, c, e = a[split], c[split], e[split]
            if a.shape[0] == 0:
                break
            m_ae, m_ac, m_ce = (a + e) / 2, (a + c) / 2, (c + e) / 2
            for m in (m_ae, m_ac, m_ce):
                _mark_grid(grid[b], m, R)
            a, c, e = (torch.cat((a, c, m_ae, e)), torch.cat((m_ae, m_ac, m_ac, m_ae)),
                       torch.cat((m_ac, m_ce, m_ce, m_ce)))
    if return_sparse:
        return grid.to_sparse()
    return grid


def unbatched_mesh_to_spc(face_vertices, level, capacity=None):
    r"""Conservative voxelisation of a mesh in [-1, 1]^3 to an SPC of ``level`` levels.
    Returns (octree u8, face_idx int64 per leaf, barycentric (num_leaves, 2) f32).

    ``capacity`` (an extension; the reference reads the counts back to size the outputs,
    mesh_to_spc_cuda.cu:351-352,438): N or (node_capacity, leaf_capacity) gives fixed-size outputs
    and nothing read back, so the call can be captured into a graph; it then returns (octree,
    face_idx, bary, result) with result = (num_nodes, num_leaves, status) on the device -- status 0:
    the first num_nodes / num_leaves rows are the eager call's; 1: a capacity too small (nothing
    written, the sizes needed in result); 2: the per-level pair buffers overflowed (nothing
    written: call without ``capacity``)."""
    if face_vertices.shape[-1] != 3:
        raise NotImplementedError("unbatched_mesh_to_spc is only implemented for triangle meshes")
    if capacity is not None:
        return _C.ops.conversions.mesh_to_spc_fixed_cuda(face_vertices.contiguous(), level, capacity)
    return _C.ops.conversions.mesh_to_spc_cuda(face_vertices.contiguous(), level)
