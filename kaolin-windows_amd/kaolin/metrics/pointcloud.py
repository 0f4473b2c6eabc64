"""sided_distance / chamfer_distance / f_score (kaolin/metrics/pointcloud.py:20-184) over the HIP path."""
import torch

from .. import _C

__all__ = ['sided_distance', 'chamfer_distance', 'f_score']


class _SidedDistanceFunction(torch.autograd.Function):
    """pointcloud.py:20-49."""

    @staticmethod
    def forward(ctx, p1, p2):
        p1 = p1.contiguous()
        p2 = p2.contiguous()
        dist, idx = _C.metrics.sided_distance_forward_cuda(p1, p2)
        ctx.save_for_backward(p1, p2, idx)
        ctx.mark_non_differentiable(idx)
        return dist, idx

    @staticmethod
    def backward(ctx, grad_output_dist, grad_output_idx):
        grad_output_dist = grad_output_dist.contiguous()
        p1, p2, idx = ctx.saved_tensors
        grad_p1, grad_p2 = _C.metrics.sided_distance_backward_cuda(grad_output_dist, p1, p2, idx)
        return grad_p1, grad_p2


def sided_distance(p1, p2):
    r"""For each point of p1 (B,N,3), the squared distance to and index of the nearest
    point of p2 (B,M,3) (lowest index on ties)."""
    return _SidedDistanceFunction.apply(p1, p2)


def chamfer_distance(p1, p2, w1=1., w2=1., squared=True):
    r"""w1 * mean_i min_j |p1_i - p2_j|^2 + w2 * mean_j min_i |p2_j - p1_i|^2 (pointcloud.py:89-135)."""
    return _chamfer_from_sided(sided_distance(p1, p2)[0], sided_distance(p2, p1)[0], w1, w2, squared)


def _chamfer_from_sided(sdist1, sdist2, w1, w2, squared):
    """chamfer_distance's reduction of the two sided distances (pointcloud.py:124-135); shared with
    kaolin.distributed.sharded_chamfer_distance, which gathers the distances first."""
    if not squared:
        sdist1 = torch.sqrt(sdist1)
        sdist2 = torch.sqrt(sdist2)
    dist_to_p2 = sdist1.mean(dim=-1)
    dist_to_p1 = sdist2.mean(dim=-1)
    if w1 == 1 and w2 == 1:
        return dist_to_p2 + dist_to_p1
    return w1 * dist_to_p2 + w2 * dist_to_p1


def f_score(gt_points, pred_points, radius=0.01, eps=1e-8):
    r"""F-score of two point sets with hits within ``radius`` (pointcloud.py:137-184)."""
    pred_distances = torch.sqrt(sided_distance(gt_points, pred_points)[0])
    gt_distances = torch.sqrt(sided_distance(pred_points, gt_points)[0])
    data_type = gt_points.dtype
    fn = torch.sum(pred_distances > radius, dim=1).type(data_type)
    fp = torch.sum(gt_distances > radius, dim=1).type(data_type)
    tp = (gt_distances.shape[1] - fp).type(data_type)
    precision = tp / (tp + fp)
    recall = tp / (tp + fn)
    return 2 * (precision * recall) / (precision + recall + eps)


def _sided_distance(p1, p2):
    """The reference's pure-torch sided distance (pointcloud.py:186-197; used by its tests and as
    the CPU path timed beside the HIP kernel): min_j |p1_i - p2_j|^2 over a (B,N,M) difference."""
    b = p1.shape[0]
    diff = (p1.reshape(b, -1, 1, 3) - p2.reshape(b, 1, -1, 3)) ** 2
    return torch.min(torch.sum(diff, dim=-1), dim=-1).values
