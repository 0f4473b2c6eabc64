"""DIB-R soft mask and dibr_rasterization (kaolin/render/mesh/dibr.py:27-209) over the HIP path."""
import torch
from torch.autograd import Function

from ... import _fused
from .rasterization import rasterize

__all__ = ['dibr_soft_mask', 'dibr_rasterization']


class DibrSoftMaskCuda(Function):
    """dibr.py:27-73 on the fused HIP path: ``* multiplier`` and the enlarged bboxes are
    evaluated in-kernel; the UNSCALED face_vertices_image is saved for backward."""

    @staticmethod
    def forward(ctx, face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier):
        face_vertices_image = face_vertices_image.contiguous()
        selected_face_idx = selected_face_idx.contiguous()
        soft_mask, close_face_prob, close_face_idx, close_face_dist_type, hits = _fused.soft_mask_forward(
            face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier, with_hits=True)
        ctx.multiplier = multiplier
        ctx.sigmainv = sigmainv
        ctx.save_for_backward(soft_mask, face_vertices_image, selected_face_idx, close_face_prob, close_face_idx,
                              close_face_dist_type, hits)
        return soft_mask

    @staticmethod
    def backward(ctx, grad_soft_mask):
        soft_mask, face_vertices_image, selected_face_idx, close_face_prob, close_face_idx, close_face_dist_type, \
            hits = ctx.saved_tensors
        grad_face_vertices_image = _fused.soft_mask_backward(
            grad_soft_mask, soft_mask, selected_face_idx, close_face_prob, close_face_idx, close_face_dist_type,
            face_vertices_image, ctx.sigmainv, ctx.multiplier, hits)
        return grad_face_vertices_image, None, None, None, None, None


def dibr_soft_mask(face_vertices_image, selected_face_idx, sigmainv=7000, boxlen=0.02, knum=30, multiplier=1000.):
    r"""Soft silhouette of DIB-R (Chen et al., NeurIPS 2019): for every pixel not covered
    by a rasterized face, 1 - prod(1 - exp(-sigmainv * d^2)) over the first ``knum``
    faces (index order) whose bbox enlarged by ``boxlen`` contains it; 1 where covered."""
    return DibrSoftMaskCuda.apply(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier)


def dibr_rasterization(height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z,
                       sigmainv=7000, boxlen=0.02, knum=30, multiplier=None, eps=None, rast_backend='cuda'):
    r"""DIB-R renderer: rasterize(valid = face_normals_z >= 0) + dibr_soft_mask.
    Returns (features, soft_mask, face_idx) as dibr.py:119-209."""
    interpolated_features, face_idx = rasterize(height, width, face_vertices_z, face_vertices_image, face_features,
                                                face_normals_z >= 0., multiplier, eps, rast_backend)
    _multiplier = 1000. if multiplier is None else multiplier
    soft_mask = dibr_soft_mask(face_vertices_image, face_idx, sigmainv, boxlen, knum, _multiplier)
    return interpolated_features, soft_mask, face_idx
