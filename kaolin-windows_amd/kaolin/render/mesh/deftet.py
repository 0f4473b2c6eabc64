"""DefTet sparse volumetric rendering (reference kaolin/render/mesh/deftet.py:269-417).

Same API as the reference: ``deftet_sparse_render(pixel_coords, render_ranges,
face_vertices_z, face_vertices_image, face_features, knum=300, eps=1e-8)`` returns the
interpolated features (B, P, knum, D) (a tuple when ``face_features`` is a list) and the
face index (B, P, knum) int64, -1 for void, hits sorted by depth (closest first).

The forward is two HIP kernels (csrc/deftet.hip): the face walk (the reference's
``deftet_sparse_render_forward_cuda``, with the bboxes computed in-kernel instead of the
torch min / max / cat of deftet.py:290-292) and one resolve kernel for the torch glue of
deftet.py:294-306 (argsort by depth, gathers, weights, interpolation).  The backward is
``_C.render.mesh.deftet_sparse_render_backward_cuda``.  There is no CPU path.
"""
import torch
from torch.autograd import Function

from ... import _C
from ... import _native as N

__all__ = ['deftet_sparse_render']


class DeftetSparseRenderer(Function):
    """torch.autograd.Function for :func:`deftet_sparse_render` (deftet.py:269-326)."""

    @staticmethod
    def forward(ctx, pixel_coords, render_ranges, face_vertices_z, face_vertices_image, face_features, knum, eps):
        func = 'deftet_sparse_render_forward_cuda'
        N.require_gpu(func, face_vertices_z, face_vertices_image, pixel_coords, render_ranges, face_features)
        pixel_coords = pixel_coords.contiguous()
        render_ranges = render_ranges.contiguous()
        face_vertices_z = face_vertices_z.contiguous()
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        batch_size, num_faces = face_vertices_z.shape[:2]
        num_pixels = pixel_coords.shape[1]
        feat_dim = face_features.shape[-1]
        if face_vertices_z.dtype not in (torch.float32, torch.float64):
            raise RuntimeError(f'"{func}" not implemented for \'{face_vertices_z.dtype}\'')
        expect = {'face_vertices_image': (face_vertices_image, (batch_size, num_faces, 3, 2)),
                  'pixel_coords': (pixel_coords, (batch_size, num_pixels, 2)),
                  'render_ranges': (render_ranges, (batch_size, num_pixels, 2)),
                  'face_features': (face_features, (batch_size, num_faces, 3, feat_dim))}
        for name, (t, shape) in expect.items():
            if tuple(t.shape) != shape:
                raise RuntimeError(f'{func}: expected {name} of size {list(shape)}, got {list(t.shape)}')
            if t.dtype != face_vertices_z.dtype:
                raise RuntimeError(f'{func}: {name} has dtype {t.dtype}, expected {face_vertices_z.dtype}')
        face_idx, pixel_depth, w0, w1 = _C.deftet_forward(
            func, face_vertices_z, face_vertices_image, None, pixel_coords, render_ranges, knum, eps)
        sorted_face_idx, weights, interpolated_features = _C.deftet_resolve(
            face_idx, pixel_depth, w0, w1, face_features)
        ctx.save_for_backward(sorted_face_idx, weights, face_vertices_image, face_features)
        ctx.mark_non_differentiable(sorted_face_idx)
        ctx.eps = eps
        return interpolated_features, sorted_face_idx

    @staticmethod
    def backward(ctx, grad_interpolated_features, grad_face_idx):
        face_idx, weights, face_vertices_image, face_features = ctx.saved_tensors
        grad_face_vertices_image, grad_face_features = _C.render.mesh.deftet_sparse_render_backward_cuda(
            grad_interpolated_features.contiguous(), face_idx, weights, face_vertices_image, face_features, ctx.eps)
        return None, None, None, grad_face_vertices_image, grad_face_features, None, None


def deftet_sparse_render(pixel_coords, render_ranges, face_vertices_z, face_vertices_image, face_features,
                         knum=300, eps=1e-8):
    r"""Fully differentiable volumetric renderer of *Gao et al.*, "Learning Deformable
    Tetrahedral Meshes for 3D Reconstruction" (NeurIPS 2020) -- deftet.py:328-417.

    Renders every intersection of each pixel's ray with the mesh inside ``render_ranges``
    (``[min, max)`` along the camera z), up to ``knum`` of them (the first ``knum`` in mesh
    order, as the reference kernel), sorted by depth with the closest first.  Not
    differentiable w.r.t. ``pixel_coords``, ``render_ranges`` or ``face_vertices_z``.

    Args:
        pixel_coords (torch.Tensor): (B, P, 2) image coordinates.
        render_ranges (torch.Tensor): (B, P, 2) depth ranges.
        face_vertices_z (torch.Tensor): (B, F, 3) camera-space z of the face vertices.
        face_vertices_image (torch.Tensor): (B, F, 3, 2) image-plane face vertices.
        face_features (torch.Tensor or list of torch.Tensor): (B, F, 3, D) per-vertex per-face
            features, or a list of such tensors (concatenated, then split on output).
        knum (int): maximum number of faces per pixel.  Default: 300.
        eps (float): barycentric normalisation epsilon.  Default: 1e-8.

    Returns:
        (torch.Tensor or tuple of torch.Tensor, torch.LongTensor): features (B, P, knum, D)
        and face index (B, P, knum), -1 for void.
    """
    _face_features = torch.cat(face_features, dim=-1) if isinstance(face_features, (list, tuple)) \
        else face_features
    image_features, face_idx = DeftetSparseRenderer.apply(
        pixel_coords, render_ranges, face_vertices_z, face_vertices_image, _face_features, knum, eps)
    if isinstance(face_features, (list, tuple)):
        out, cur = [], 0
        for f in face_features:
            out.append(image_features[..., cur:cur + f.shape[-1]])
            cur += f.shape[-1]
        image_features = tuple(out)
    return image_features, face_idx
