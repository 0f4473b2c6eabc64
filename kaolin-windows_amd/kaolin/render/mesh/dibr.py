"""DIB-R soft mask and dibr_rasterization (kaolin/render/mesh/dibr.py:27-209) over the HIP path."""
import torch
from torch.autograd import Function

from ... import _ext
from ... import _fused
from ... import _native as N
from .rasterization import rasterize

__all__ = ['dibr_soft_mask', 'dibr_rasterization']


class DibrSoftMaskCuda(Function):
    """dibr.py:27-73 on the fused HIP path: ``* multiplier`` and the enlarged bboxes are
    evaluated in-kernel; the UNSCALED face_vertices_image is saved for backward.

    For knum <= 255 the saved state is compact (softtile.hip): per-pixel filled-slot counts
    and one record per filled slot, instead of the reference's four (B,H,W,knum) slot
    tensors -- the returned soft mask and the gradient are the same."""

    @staticmethod
    def forward(ctx, face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier):
        face_vertices_image = face_vertices_image.contiguous()
        selected_face_idx = selected_face_idx.contiguous()
        ctx.multiplier = multiplier
        ctx.sigmainv = sigmainv
        ctx.compact = 0 <= int(knum) <= 255
        if ctx.compact:
            soft_mask, state = _fused.soft_mask_forward_compact(face_vertices_image, selected_face_idx, sigmainv,
                                                                boxlen, knum, multiplier)
            ctx.knum = state.knum
            ctx.save_for_backward(soft_mask, face_vertices_image, *state.tensors())
            return soft_mask
        soft_mask, close_face_prob, close_face_idx, close_face_dist_type, hits = _fused.soft_mask_forward(
            face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier, with_hits=True)
        ctx.save_for_backward(soft_mask, face_vertices_image, selected_face_idx, close_face_prob, close_face_idx,
                              close_face_dist_type, hits)
        return soft_mask

    @staticmethod
    def backward(ctx, grad_soft_mask):
        if ctx.compact:
            soft_mask, face_vertices_image, *st = ctx.saved_tensors
            state = _fused.SoftMaskState(*st, ctx.knum)
            grad_face_vertices_image = _fused.soft_mask_backward_compact(
                grad_soft_mask, soft_mask, state, face_vertices_image, ctx.sigmainv, ctx.multiplier)
            return grad_face_vertices_image, None, None, None, None, None
        soft_mask, face_vertices_image, selected_face_idx, close_face_prob, close_face_idx, close_face_dist_type, \
            hits = ctx.saved_tensors
        grad_face_vertices_image = _fused.soft_mask_backward(
            grad_soft_mask, soft_mask, selected_face_idx, close_face_prob, close_face_idx, close_face_dist_type,
            face_vertices_image, ctx.sigmainv, ctx.multiplier, hits)
        return grad_face_vertices_image, None, None, None, None, None


class DibrRasterizationCuda(Function):
    """dibr_rasterization (dibr.py:119-209) as one autograd node: rasterize with
    valid = face_normals_z >= 0 evaluated in-kernel, then the compact soft mask on its
    face index.  The backward is one call: the soft-mask terms summed in double, then the
    rasterizer's gather, which writes every face's gradient as its rounded sum plus the soft
    mask's -- no zero fill and no separate sum of the two gradients.  Outputs and gradients
    equal rasterize + dibr_soft_mask's."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z, sigmainv,
                boxlen, knum, multiplier, eps):
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        face_normals_z = face_normals_z.detach().contiguous()
        if face_normals_z.dtype == face_vertices_image.dtype:  # one call, one shared binning pass
            feats, face_idx, weights, soft_mask, state, ranges = _fused.dibr_forward(
                height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z, sigmainv, boxlen,
                knum, multiplier, eps)
        else:
            ranges = None
            feats, face_idx, weights = _fused.rasterize_forward(height, width, face_vertices_z, face_vertices_image,
                                                                face_features, None, multiplier, eps,
                                                                face_normals_z=face_normals_z)
            soft_mask, state = _fused.soft_mask_forward_compact(face_vertices_image, face_idx, sigmainv, boxlen, knum,
                                                                multiplier)
        ctx.mark_non_differentiable(face_idx)
        ctx.set_materialize_grads(False)  # no zero-filled grads for face_idx (or unused outputs)
        ctx.sigmainv, ctx.multiplier, ctx.eps, ctx.knum = sigmainv, multiplier, eps, state.knum
        ctx.has_ranges = ranges is not None and ranges.numel() > 0
        ctx.save_for_backward(face_idx, weights, face_vertices_image, face_features, face_normals_z, soft_mask,
                              ranges if ctx.has_ranges else None, *state.tensors())
        return feats, soft_mask, face_idx

    @staticmethod
    def backward(ctx, grad_feats, grad_soft_mask, grad_face_idx):
        face_idx, weights, fvi, feat, fnz, soft_mask, ranges, *st = ctx.saved_tensors
        state = _fused.SoftMaskState(*st, ctx.knum)
        if grad_feats is None and grad_soft_mask is None:
            return None, None, None, None, None, None, None, None, None, None, None
        if grad_feats is None:
            grad_feats = torch.zeros(face_idx.shape + (feat.shape[-1],), dtype=feat.dtype, device=feat.device)
        if fnz.dtype == fvi.dtype:
            g_img, g_feat = _fused.dibr_backward(grad_feats, grad_soft_mask, face_idx, weights, fvi, feat, fnz,
                                                 soft_mask, state, ctx.sigmainv, ctx.multiplier, ctx.eps, ranges)
        else:  # face_normals_z of another dtype: the two stages (the rasterizer's reads a valid mask)
            g_img, g_feat = _fused.rasterize_backward(grad_feats, face_idx, weights, fvi, feat, None, ctx.multiplier,
                                                      ctx.eps, face_normals_z=fnz, face_ranges=ranges)
            if grad_soft_mask is not None:
                _fused.soft_mask_backward_compact(grad_soft_mask, soft_mask, state, fvi, ctx.sigmainv,
                                                  ctx.multiplier, out=g_img)
        return None, None, None, g_img, g_feat, None, None, None, None, None, None


def dibr_soft_mask(face_vertices_image, selected_face_idx, sigmainv=7000, boxlen=0.02, knum=30, multiplier=1000.):
    r"""Soft silhouette of DIB-R (Chen et al., NeurIPS 2019): for every pixel not covered
    by a rasterized face, 1 - prod(1 - exp(-sigmainv * d^2)) over the first ``knum``
    faces (index order) whose bbox enlarged by ``boxlen`` contains it; 1 where covered."""
    return DibrSoftMaskCuda.apply(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier)


def dibr_rasterization(height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z,
                       sigmainv=7000, boxlen=0.02, knum=30, multiplier=None, eps=None, rast_backend='cuda'):
    r"""DIB-R renderer: rasterize(valid = face_normals_z >= 0) + dibr_soft_mask.
    Returns (features, soft_mask, face_idx) as dibr.py:119-209; ``face_features`` may be a
    list, then features is a tuple of per-element views."""
    _multiplier = 1000. if multiplier is None else multiplier
    _eps = 1e-8 if eps is None else eps
    is_list = isinstance(face_features, (list, tuple))
    # a feature list (the tutorial's [face_uvs, ones]) is concatenated and the outputs split as
    # rasterize does (rasterization.py:480-481,498-505); the single node serves both shapes
    _face_features = torch.cat(face_features, dim=-1) if is_list else face_features
    if (rast_backend in ('cuda', 'hip') and _face_features.shape[-1] <= 8 and 0 <= int(knum) <= 255
            and face_vertices_image.dtype in (torch.float32, torch.float64)):
        ext = _ext.get()
        dev = face_vertices_image.device
        if (ext is not None and N._TIMER is None and face_vertices_image.is_cuda
                and face_normals_z.dtype == face_vertices_image.dtype
                and face_vertices_z.dtype == face_vertices_image.dtype
                and _face_features.dtype == face_vertices_image.dtype
                and all(t.device == dev for t in (face_vertices_z, _face_features, face_normals_z))
                and dev.index == torch.cuda.current_device()):
            # the same node compiled (csrc/torch_ops.cpp): the eager host path without Python in
            # the autograd node (bench's per-op HIP-event pass keeps the Python node)
            feats, soft_mask, face_idx = ext.dibr_rasterization(
                int(height), int(width), face_vertices_z, face_vertices_image, _face_features, face_normals_z,
                float(sigmainv), float(boxlen), int(knum), float(_multiplier), float(_eps), N.stream_of(dev))
        else:
            N.require_gpu('dibr_rasterization', face_vertices_z, face_vertices_image, face_normals_z)
            feats, soft_mask, face_idx = DibrRasterizationCuda.apply(
                height, width, face_vertices_z, face_vertices_image, _face_features, face_normals_z, sigmainv, boxlen,
                knum, _multiplier, _eps)
        if is_list:
            out, cur = [], 0
            for ff in face_features:
                out.append(feats[..., cur:cur + ff.shape[-1]])
                cur += ff.shape[-1]
            feats = tuple(out)
        return feats, soft_mask, face_idx
    interpolated_features, face_idx = rasterize(height, width, face_vertices_z, face_vertices_image, face_features,
                                                face_normals_z >= 0., multiplier, eps, rast_backend)
    soft_mask = dibr_soft_mask(face_vertices_image, face_idx, sigmainv, boxlen, knum, _multiplier)
    return interpolated_features, soft_mask, face_idx
