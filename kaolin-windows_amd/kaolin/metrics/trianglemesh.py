"""point_to_mesh_distance (kaolin/metrics/trianglemesh.py:20-268).

GPU tensors go through the HIP kernels behind ``_C.metrics.unbatched_triangle_distance_*``
(distance.hip).  CPU tensors take the reference's CPU path: the brute-force torch
evaluation of ``_unbatched_naive_point_to_mesh_distance`` (trianglemesh.py:143-268), same
per-(point, face) float operations and the same type bookkeeping, evaluated here in point
chunks so that memory stays bounded, with autograd through the recomputed closest points.
"""
import torch

from .. import _C

__all__ = ['point_to_mesh_distance']


class _UnbatchedTriangleDistanceCuda(torch.autograd.Function):
    """trianglemesh.py:117-141."""

    @staticmethod
    def forward(ctx, points, face_vertices):
        num_points = points.shape[0]
        min_dist = torch.empty((num_points,), device=points.device, dtype=points.dtype)
        min_dist_idx = torch.empty((num_points,), device=points.device, dtype=torch.long)
        dist_type = torch.empty((num_points,), device=points.device, dtype=torch.int32)
        points = points.contiguous()
        face_vertices = face_vertices.contiguous()
        _C.metrics.unbatched_triangle_distance_forward_cuda(points, face_vertices, min_dist, min_dist_idx,
                                                            dist_type)
        ctx.save_for_backward(points, face_vertices, min_dist_idx, dist_type)
        ctx.mark_non_differentiable(min_dist_idx, dist_type)
        return min_dist, min_dist_idx, dist_type

    @staticmethod
    def backward(ctx, grad_dist, grad_face_idx, grad_dist_type):
        points, face_vertices, face_idx, dist_type = ctx.saved_tensors
        grad_dist = grad_dist.contiguous()
        grad_points = torch.empty_like(points)
        grad_face_vertices = torch.empty_like(face_vertices)
        _C.metrics.unbatched_triangle_distance_backward_cuda(grad_dist, points, face_vertices, face_idx, dist_type,
                                                             grad_points, grad_face_vertices)
        return grad_points, grad_face_vertices


# ------------------------------------------------------------------------- CPU path
def _dot3(a, b):
    # x, y, z products summed left to right (trianglemesh.py:93-96)
    return a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1] + a[..., 2] * b[..., 2]


def _edge_param(origin, edge, p):
    """Position of p's projection along origin + t * edge."""
    return _dot3(p - origin, edge) / _dot3(edge, edge)


def _plane_foot(origin, unit_normal, p):
    return p - unit_normal * _dot3(p - origin, unit_normal).unsqueeze(-1)


def _unit(n):
    return n / torch.norm(n, dim=-1, keepdim=True)


class _Tri:
    """Corners, edges (v2-v1, v3-v2, v1-v3) and the normal of (F,3,3) triangles."""

    def __init__(self, fv):
        self.v = (fv[:, 0], fv[:, 1], fv[:, 2])
        v1, v2, v3 = self.v
        self.e = (v2 - v1, v3 - v2, v1 - v3)
        self.n = -torch.cross(self.e[0], self.e[2], dim=-1)


def _regions(tri, p):
    """Per (point, face): the three edge parameters and the six region flags of the
    reference's classification (trianglemesh.py:192-205)."""
    u = [_edge_param(tri.v[k].unsqueeze(0), tri.e[k].unsqueeze(0), p.unsqueeze(1)) for k in range(3)]
    flags = []
    for k in range(3):  # vertex regions 1..3: past the end of edge k-1, before the start of edge k
        flags.append((u[(k + 2) % 3] > 1.) & (u[k] < 0.))
    for k in range(3):  # edge regions 4..6: inside edge k's span and not above it
        side = torch.cross(tri.n, tri.e[k], dim=-1)
        below = _dot3(side.unsqueeze(0), p.unsqueeze(1) - tri.v[k].unsqueeze(0)) <= 0
        flags.append((u[k] >= 0.) & (u[k] <= 1.) & below)
    return u, flags


def _naive_select(points, face_vertices, chunk_elems=1 << 22):
    """Nearest face and its type for every point (no autograd), in chunks of points."""
    P, F = points.shape[0], face_vertices.shape[0]
    tri = _Tri(face_vertices)
    un = _unit(tri.n)
    step = max(1, chunk_elems // max(F, 1))
    idx_out = torch.empty((P,), dtype=torch.long)
    typ_out = torch.empty((P,), dtype=torch.int32)
    for s in range(0, P, step):
        p = points[s:s + step]
        u, fl = _regions(tri, p)
        # the reference fills the closest points type by type (0, then 1..6): a later
        # type overwrites an earlier one where several flags hold
        cp = _plane_foot(tri.v[0].unsqueeze(0), un.unsqueeze(0), p.unsqueeze(1))
        for k in range(3):
            cp = torch.where(fl[k].unsqueeze(-1), tri.v[k].unsqueeze(0), cp)
        for k in range(3):
            on_edge = tri.v[k].unsqueeze(0) + tri.e[k].unsqueeze(0) * u[k].unsqueeze(-1)
            cp = torch.where(fl[3 + k].unsqueeze(-1), on_edge, cp)
        diff = cp - p.unsqueeze(1)
        d = _dot3(diff, diff)
        _, best = torch.min(d, dim=-1)
        types = sum(f.int() * (k + 1) for k, f in enumerate(fl))  # flags are summed, as the reference does
        idx_out[s:s + step] = best
        typ_out[s:s + step] = types.gather(1, best.unsqueeze(1)).squeeze(1)
    return idx_out, typ_out


def _unbatched_naive_point_to_mesh_distance(points, face_vertices):
    r"""CPU point-to-mesh distance of (P,3) points and (F,3,3) triangles
    (trianglemesh.py:143-268): returns (squared distance (P), face index (P) int64,
    distance type (P) int32).  The distance is recomputed on the selected faces with
    autograd, so gradients reach only the nearest triangles."""
    with torch.no_grad():
        face_idx, dist_type = _naive_select(points.detach(), face_vertices.detach())
    tri = _Tri(face_vertices[face_idx])
    u = [_edge_param(tri.v[k], tri.e[k], points) for k in range(3)]
    closest = torch.zeros_like(points)
    for k in range(3):
        closest = torch.where((dist_type == k + 1).unsqueeze(-1), tri.v[k], closest)
    for k in range(3):
        on_edge = tri.v[k] + tri.e[k] * u[k].unsqueeze(-1)
        closest = torch.where((dist_type == k + 4).unsqueeze(-1), on_edge, closest)
    foot = _plane_foot(tri.v[0], _unit(tri.n), points)
    closest = torch.where((dist_type == 0).unsqueeze(-1), foot, closest)
    min_dist = torch.sum((closest - points) ** 2, dim=-1)
    return min_dist, face_idx, dist_type


def point_to_mesh_distance(pointclouds, face_vertices):
    r"""Squared distance from each point of (B,P,3) to the closest triangle of
    face_vertices (B,F,3,3), with that face's index and the distance type
    (0 face, 1-3 vertex, 4-6 edge)."""
    distance, face_idx, dist_type = [], [], []
    for i in range(pointclouds.shape[0]):
        if pointclouds.is_cuda:
            d, f, t = _UnbatchedTriangleDistanceCuda.apply(pointclouds[i], face_vertices[i])
        else:
            d, f, t = _unbatched_naive_point_to_mesh_distance(pointclouds[i], face_vertices[i])
        distance.append(d)
        face_idx.append(f)
        dist_type.append(t)
    return torch.stack(distance, dim=0), torch.stack(face_idx, dim=0), torch.stack(dist_type, dim=0)
