"""rasterize() front-end (kaolin/render/mesh/rasterization.py:243-506) over the HIP path.

Same signature, defaults (multiplier=1000, eps=1e-8), feature list concat/split and
valid-face packing as the reference; backend 'cuda' (alias 'hip') runs
``_C.render.mesh.packed_rasterize_forward_cuda`` / ``rasterize_backward_cuda`` on
gfx950.  The nvdiffrast backends of the reference are out of scope.
"""
import torch
from torch.autograd import Function

from ... import _C
from ... import _fused

__all__ = ['rasterize']


def _pack_valid_faces(face_vertices_z, face_vertices_image, face_features, valid_faces):
    """rasterization.py:309-334: pack the valid faces of every mesh contiguously."""
    batch_size, num_faces = face_vertices_z.shape[:2]
    feat_dim = face_features.shape[-1]
    device = face_vertices_z.device
    if valid_faces is None:
        valid_faces_idx = (
            torch.arange(batch_size, dtype=torch.long, device=device).reshape(-1, 1).repeat(1, num_faces).reshape(-1),
            torch.arange(num_faces, dtype=torch.long, device=device).reshape(1, -1).repeat(batch_size, 1).reshape(-1))
        vfvi = face_vertices_image.reshape(batch_size * num_faces, 3, 2)
        vfvz = face_vertices_z.reshape(batch_size * num_faces, 3)
        vfeat = face_features.reshape(batch_size * num_faces, 3, feat_dim)
        num_faces_per_mesh = torch.full((batch_size,), num_faces, dtype=torch.long, device=device)
    else:
        valid_faces_idx = torch.where(valid_faces)
        vfvi = face_vertices_image[valid_faces_idx[0], valid_faces_idx[1]]
        vfvz = face_vertices_z[valid_faces_idx[0], valid_faces_idx[1]]
        vfeat = face_features[valid_faces_idx[0], valid_faces_idx[1]]
        num_faces_per_mesh = torch.sum(valid_faces.reshape(batch_size, -1), dim=1)
    first_idx = torch.zeros(batch_size + 1, dtype=torch.long, device=device)
    torch.cumsum(num_faces_per_mesh, dim=0, out=first_idx[1:])
    return valid_faces_idx, vfvi, vfvz, vfeat, first_idx


class RasterizeCuda(Function):
    """torch.autograd.Function for ``rasterize`` with backend 'cuda' (rasterization.py:243-388).

    Runs the fused HIP path: the valid-face packing, ``* multiplier``, bboxes and the
    packed->original index remap of the reference front-end happen inside the kernels
    (same float operations), and the backward is an atomic-free per-face gather.
    ``_C.render.mesh.packed_rasterize_forward_cuda`` / ``rasterize_backward_cuda`` keep
    the reference's packed contract for direct callers.
    """

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features, valid_faces, multiplier,
                eps):
        face_features = face_features.contiguous()
        face_vertices_image = face_vertices_image.contiguous()
        interpolated_features, face_idx, output_weights = _fused.rasterize_forward(
            height, width, face_vertices_z, face_vertices_image, face_features, valid_faces, multiplier, eps)
        ctx.save_for_backward(face_idx, output_weights, face_vertices_image, face_features, valid_faces)
        ctx.mark_non_differentiable(face_idx)
        ctx.eps = eps
        ctx.multiplier = multiplier
        return interpolated_features, face_idx

    @staticmethod
    def backward(ctx, grad_interpolated_features, grad_face_idx):
        face_idx, output_weights, face_vertices_image, face_features, valid_faces = ctx.saved_tensors
        grad_face_vertices_image, grad_face_features = _fused.rasterize_backward(
            grad_interpolated_features, face_idx, output_weights, face_vertices_image, face_features, valid_faces,
            ctx.multiplier, ctx.eps)
        return None, None, None, grad_face_vertices_image, grad_face_features, None, None, None


class RasterizeCudaPacked(Function):
    """The reference's exact chain (rasterization.py:290-388): torch packing + the
    packed ``_C`` entry points.  Kept for parity checks of the _C contract."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features, valid_faces, multiplier,
                eps):
        face_features = face_features.contiguous()
        face_vertices_image = face_vertices_image.contiguous()
        num_faces = face_vertices_z.shape[1]
        valid_faces_idx, vfvi, vfvz, vfeat, first_idx = _pack_valid_faces(
            face_vertices_z, face_vertices_image, face_features, valid_faces)
        vfvi = vfvi * multiplier
        points_min = torch.min(vfvi, dim=1)[0]
        points_max = torch.max(vfvi, dim=1)[0]
        vbboxes = torch.cat((points_min, points_max), dim=1)
        interpolated_features, selected_face_idx, output_weights = _C.render.mesh.packed_rasterize_forward_cuda(
            height, width, vfvz.contiguous(), vfvi.contiguous(), vbboxes.contiguous(), vfeat.contiguous(),
            first_idx.contiguous(), multiplier, eps, max_faces_per_mesh=num_faces)
        face_idx = valid_faces_idx[1][(selected_face_idx + first_idx[:-1].reshape(-1, 1, 1)).reshape(-1)]
        face_idx = face_idx.reshape(selected_face_idx.shape).contiguous()
        face_idx[selected_face_idx == -1] = -1
        ctx.save_for_backward(interpolated_features, face_idx, output_weights, face_vertices_image, face_features)
        ctx.mark_non_differentiable(face_idx)
        ctx.eps = eps
        return interpolated_features, face_idx

    @staticmethod
    def backward(ctx, grad_interpolated_features, grad_face_idx):
        interpolated_features, face_idx, output_weights, face_vertices_image, face_features = ctx.saved_tensors
        grad_face_vertices_image, grad_face_features = _C.render.mesh.rasterize_backward_cuda(
            grad_interpolated_features.contiguous(), interpolated_features, face_idx, output_weights,
            face_vertices_image, face_features, ctx.eps)
        return None, None, None, grad_face_vertices_image, grad_face_features, None, None, None


def rasterize(height, width, face_vertices_z, face_vertices_image, face_features, valid_faces=None, multiplier=None,
              eps=None, backend='cuda'):
    r"""Fully differentiable rasterization of triangle meshes with per-vertex per-face
    features into feature images (DIB-R interpolation rasterizer).

    Args and returns as the reference (rasterization.py:390-470): ``face_vertices_z``
    (B,F,3), ``face_vertices_image`` (B,F,3,2), ``face_features`` (B,F,3,D) or a list,
    ``valid_faces`` (B,F) bool; returns the (B,H,W,D) features (or a tuple when
    ``face_features`` is a list) and the (B,H,W) int64 face index (-1 = none).
    """
    if multiplier is None:
        multiplier = 1000
    if eps is None:
        eps = 1e-8
    if backend not in ('cuda', 'hip', 'cuda_packed'):
        raise ValueError(f'"{backend}" is not a valid backend for kaolin-mi355x, valid choices are ["cuda", "hip"] '
                         '(the nvdiffrast backends are not available on ROCm)')
    _face_features = torch.cat(face_features, dim=-1) if isinstance(face_features, (list, tuple)) else face_features
    fn = RasterizeCudaPacked if backend == 'cuda_packed' else RasterizeCuda
    image_features, face_idx = fn.apply(height, width, face_vertices_z, face_vertices_image, _face_features,
                                        valid_faces, multiplier, eps)
    if isinstance(face_features, (list, tuple)):
        out = []
        cur = 0
        for ff in face_features:
            out.append(image_features[..., cur:cur + ff.shape[-1]])
            cur += ff.shape[-1]
        image_features = tuple(out)
    return image_features, face_idx
