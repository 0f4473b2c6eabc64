"""center_points (kaolin/ops/pointcloud.py:20-43): the tutorial's mesh centring (torch)."""
import torch

__all__ = ['center_points']


def center_points(points: torch.Tensor, normalize: bool = False, eps=1e-6):
    """Each point cloud (B, N, C) moved so its bbox centre is the origin; with ``normalize``
    also scaled by its largest bbox extent (clipped at ``eps``) into [-0.5, 0.5]."""
    assert len(points.shape) == 3, f'Points have unexpected shape {points.shape}'
    vmin = points.min(dim=1, keepdim=True)[0]
    vmax = points.max(dim=1, keepdim=True)[0]
    res = points - (vmin + vmax) / 2
    if normalize:
        res = res / (vmax - vmin).max(dim=-1, keepdim=True)[0].clip(min=eps)
    return res
