"""point_to_mesh_distance (kaolin/metrics/trianglemesh.py:20-141) over the HIP path."""
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


def point_to_mesh_distance(pointclouds, face_vertices):
    r"""Squared distance from each point of (B,P,3) to the closest triangle of
    face_vertices (B,F,3,3), with that face's index and the distance type
    (0 face, 1-3 vertex, 4-6 edge).  GPU tensors only."""
    if not pointclouds.is_cuda:
        raise RuntimeError('point_to_mesh_distance: kaolin-mi355x runs only on GPU tensors; there is no CPU path')
    distance, face_idx, dist_type = [], [], []
    for i in range(pointclouds.shape[0]):
        d, f, t = _UnbatchedTriangleDistanceCuda.apply(pointclouds[i], face_vertices[i])
        distance.append(d)
        face_idx.append(f)
        dist_type.append(t)
    return torch.stack(distance, dim=0), torch.stack(face_idx, dim=0), torch.stack(dist_type, dim=0)
