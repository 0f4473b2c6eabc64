"""mask_iou (kaolin/metrics/render.py:18-40): the silhouette loss used with dibr_soft_mask."""
import torch


def mask_iou(lhs_mask, rhs_mask):
    batch_size, height, width = lhs_mask.shape
    assert rhs_mask.shape == lhs_mask.shape
    sil_mul = lhs_mask * rhs_mask
    sil_add = lhs_mask + rhs_mask
    iou_up = torch.sum(sil_mul.reshape(batch_size, -1), dim=1)
    iou_down = torch.sum((sil_add - sil_mul).reshape(batch_size, -1), dim=1)
    iou_neg = iou_up / (iou_down + 1e-10)
    return 1.0 - torch.mean(iou_neg)
