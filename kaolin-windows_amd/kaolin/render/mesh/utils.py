"""prepare_vertices (kaolin/render/mesh/utils.py:128-175): camera transform, perspective
projection, index_vertices_by_faces and unit face normals -- the inputs of every DIB-R call.

GPU f32 / f64 tensors run one HIP launch forward and one backward call (csrc/prepare.hip,
``kl_prepare_vertices_forward`` / ``_backward``), with gradients to the vertices and to every
camera tensor that requires one.  Other devices and dtypes run the reference's torch chain, as
the reference does on every device.
"""
import weakref

import torch
from torch.autograd import Function

from ... import _ext, _native as N
from ...ops.mesh import face_normals as _face_normals
from ...ops.mesh import index_vertices_by_faces
from ..camera import perspective_camera, rotate_translate_points

__all__ = ['prepare_vertices', 'texture_mapping']


def _prepare_vertices_torch(vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform):
    """The reference's chain (utils.py:160-175), for devices / dtypes the HIP path does not take."""
    if camera_transform is None:
        vertices_camera = rotate_translate_points(vertices, camera_rot, camera_trans)
    else:
        padded_vertices = torch.nn.functional.pad(vertices, (0, 1), mode='constant', value=1.)
        vertices_camera = padded_vertices @ camera_transform
    vertices_image = perspective_camera(vertices_camera, camera_proj)
    face_vertices_camera = index_vertices_by_faces(vertices_camera, faces)
    face_vertices_image = index_vertices_by_faces(vertices_image, faces)
    face_normals = _face_normals(face_vertices_camera, unit=True)
    return face_vertices_camera, face_vertices_image, face_normals


def _batches(vertices, camera_proj, camera_rot, camera_trans, camera_transform):
    """(B, Bv, Bc, Bp) as torch's broadcasting forms them, or None when the shapes fall outside
    what the kernel takes (the torch chain then runs and raises / broadcasts as the reference)."""
    if vertices.ndim != 3 or vertices.shape[-1] != 3:
        return None
    Bv = vertices.shape[0]
    if camera_transform is None:
        if camera_rot.ndim != 3 or camera_rot.shape[1:] != (3, 3) or camera_trans.numel() % 3:
            return None
        Bc = camera_rot.shape[0]
        if camera_trans.numel() // 3 != Bc:
            return None
    else:
        if camera_transform.ndim != 3 or camera_transform.shape[1:] != (4, 3):
            return None
        Bc = camera_transform.shape[0]
    if camera_proj.numel() % 3:
        return None
    Bp = camera_proj.numel() // 3
    B = max(Bv, Bc, Bp)
    if any(x not in (1, B) for x in (Bv, Bc, Bp)):
        return None
    if max(Bv, Bc) == 1 < Bp:  # torch gives face_vertices_camera / face_normals a batch of 1 here
        return None
    return B, Bv, Bc, Bp


_CHECKED_FACES = {}  # id(faces) -> (weakref to faces, (version, shape, V) checked)


def _check_faces(faces, num_vertices):
    """index_vertices_by_faces' gather raises on an index outside [0, V); the kernel
    would give NaN outputs instead.  A faces tensor is checked once (one host read) and
    remembered (weakly) with its version, shape and V: the meshes of a training loop are fixed, so the
    steady state reads nothing back.  Skipped under graph capture (no host reads there)."""
    key = (faces._version, tuple(faces.shape), int(num_vertices))
    hit = _CHECKED_FACES.get(id(faces))
    if (hit is not None and hit[0]() is faces and hit[1] == key) or (faces.is_cuda and torch.cuda.is_current_stream_capturing()):
        return
    if faces.numel() > 0:
        lo, hi = torch.aminmax(faces)
        lo, hi = int(lo), int(hi)
        if lo < 0 or hi >= num_vertices:  # torch.gather's check (index_vertices_by_faces)
            bad = lo if lo < 0 else hi
            raise RuntimeError(f'index {bad} is out of bounds for dimension 1 with size {num_vertices}')
    for k in [k for k, (r, _) in _CHECKED_FACES.items() if r() is None]:
        del _CHECKED_FACES[k]
    _CHECKED_FACES[id(faces)] = (weakref.ref(faces), key)


class PrepareVerticesHip(Function):
    """One autograd node for prepare_vertices on the HIP path (csrc/prepare.hip)."""

    @staticmethod
    def forward(ctx, vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform, batches):
        B, Bv, Bc, Bp = batches
        dtype, dev = vertices.dtype, vertices.device
        V, F = vertices.shape[1], faces.shape[0]
        verts = vertices.contiguous()
        fc = faces.contiguous()
        proj = camera_proj.contiguous()
        rot = camera_rot.contiguous() if camera_transform is None else None
        trans = camera_trans.contiguous() if camera_transform is None else None
        xf = camera_transform.contiguous() if camera_transform is not None else None
        fvc = torch.empty((B, F, 3, 3), dtype=dtype, device=dev)
        fvi = torch.empty((B, F, 3, 2), dtype=dtype, device=dev)
        fn = torch.empty((B, F, 3), dtype=dtype, device=dev)
        with N.on_device(dev), N.timed('prepare_vertices_forward', dev):
            N.check(N.lib().kl_prepare_vertices_forward(
                N.dtype_code(dtype), B, Bv, Bc, Bp, V, F, N.ptr(verts), N.ptr(fc), N.ptr(rot), N.ptr(trans), N.ptr(xf),
                N.ptr(proj), N.ptr(fvc), N.ptr(fvi), N.ptr(fn), N.stream_of(dev)), 'prepare_vertices')
        ctx.batches = batches
        ctx.shapes = (camera_proj.shape, None if camera_trans is None else camera_trans.shape)
        # the inputs themselves (a double backward differentiates the reference's chain of them)
        ctx.save_for_backward(vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform)
        ctx.set_materialize_grads(False)
        return fvc, fvi, fn

    @staticmethod
    def backward(ctx, g_fvc, g_fvi, g_fn):
        verts, fc, proj, rot, trans, xf = ctx.saved_tensors
        if torch.is_grad_enabled():  # create_graph: the reference's torch gradient, differentiable
            from ..._double_backward import prepare_vertices as dd
            g = dd(verts, fc, proj, rot, trans, xf, g_fvc, g_fvi, g_fn)
            return g[0], None, g[2], g[3], g[4], g[5], None
        verts, fc, proj = verts.contiguous(), fc.contiguous(), proj.contiguous()
        rot, trans, xf = (None if x is None else x.contiguous() for x in (rot, trans, xf))
        B, Bv, Bc, Bp = ctx.batches
        need_v, _, need_p, need_r, need_t, need_x, _ = ctx.needs_input_grad
        if g_fvc is None and g_fvi is None and g_fn is None:
            return None, None, None, None, None, None, None
        dtype, dev = verts.dtype, verts.device
        V, F = verts.shape[1], fc.shape[0]
        g_v = torch.empty_like(verts) if need_v else None
        g_cam = torch.empty((Bc, 12), dtype=dtype, device=dev) if (need_r or need_t or need_x) else None
        g_proj = torch.empty((Bp, 3), dtype=dtype, device=dev) if need_p else None
        lib = N.lib()
        nbytes = lib.kl_prepare_vertices_bwd_workspace_bytes(B, V)
        ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
        with N.on_device(dev), N.timed('prepare_vertices_backward', dev):
            N.check(lib.kl_prepare_vertices_backward(
                N.dtype_code(dtype), B, Bv, Bc, Bp, V, F, N.ptr(verts), N.ptr(fc), N.ptr(rot), N.ptr(trans), N.ptr(xf),
                N.ptr(proj), N.ptr(None if g_fvc is None else g_fvc.contiguous()),
                N.ptr(None if g_fvi is None else g_fvi.contiguous()), N.ptr(None if g_fn is None else g_fn.contiguous()),
                N.ptr(g_v), N.ptr(g_cam), N.ptr(g_proj), N.ptr(ws), nbytes, N.stream_of(dev)),
                'prepare_vertices backward')
        proj_shape, trans_shape = ctx.shapes
        g_r = g_cam[:, :9].reshape(Bc, 3, 3) if need_r else None
        g_t = g_cam[:, 9:].reshape(trans_shape) if need_t else None
        g_x = g_cam.reshape(Bc, 4, 3) if need_x else None
        g_p = g_proj.reshape(proj_shape) if need_p else None
        return g_v, None, g_p, g_r, g_t, g_x, None


def prepare_vertices(vertices, faces, camera_proj, camera_rot=None, camera_trans=None, camera_transform=None):
    r"""Move and project vertices to the cameras, then index them by faces (utils.py:128-175).

    Args:
        vertices (torch.Tensor): (batch_size, num_vertices, 3).
        faces (torch.LongTensor): (num_faces, 3).
        camera_proj (torch.Tensor): (3, 1).
        camera_rot (torch.Tensor, optional): (batch_size, 3, 3).
        camera_trans (torch.Tensor, optional): (batch_size, 3).
        camera_transform (torch.Tensor, optional): (batch_size, 4, 3); replaces rot and trans.
    Returns:
        face_vertices_camera (B, F, 3, 3), face_vertices_image (B, F, 3, 2),
        face_normals (B, F, 3) (unit).
    """
    if camera_transform is None:
        assert camera_trans is not None and camera_rot is not None, \
            "camera_transform or camera_trans and camera_rot must be defined"
        cams = (camera_rot, camera_trans)
    else:
        assert camera_trans is None and camera_rot is None, \
            "camera_trans and camera_rot must be None when camera_transform is defined"
        cams = (camera_transform,)
    tensors = (vertices, faces, camera_proj) + cams
    batches = None
    if (all(t.is_cuda for t in tensors) and len({t.device for t in tensors}) == 1
            and vertices.dtype in (torch.float32, torch.float64)
            and all(t.dtype == vertices.dtype for t in (camera_proj,) + cams)
            and faces.dtype == torch.long and faces.ndim == 2 and faces.shape[-1] == 3):
        batches = _batches(vertices, camera_proj, camera_rot, camera_trans, camera_transform)
    if batches is None:
        return _prepare_vertices_torch(vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform)
    _check_faces(faces, vertices.shape[1])
    ext = _ext.get()
    if ext is not None and N._TIMER is None and vertices.device.index == torch.cuda.current_device():
        # the same node compiled (csrc/torch_ops.cpp): no Python in the autograd node
        return ext.prepare_vertices(vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform,
                                    list(batches), N.stream_of(vertices.device))
    return PrepareVerticesHip.apply(vertices, faces, camera_proj, camera_rot, camera_trans, camera_transform, batches)


class TextureMappingHip(Function):
    """texture_mapping's clamp -> [-1, 1] (y reversed) -> grid_sample(border, align_corners=False)
    chain as one HIP launch each way (csrc/texture.hip): the forward and the coordinate gradient
    with grid_sample's own arithmetic; the texture gradient summed in double (deterministic), with
    the terms of zero incoming gradients skipped."""

    @staticmethod
    def forward(ctx, coords, texture_maps, mode):
        B, C, TH, TW = texture_maps.shape
        c = coords.contiguous()
        tex = texture_maps.contiguous()
        n = c.numel() // (2 * B) if B else 0
        out = torch.empty((B, n, C), dtype=tex.dtype, device=tex.device)
        with N.on_device(tex.device):
            N.check(N.lib().kl_texture_mapping_forward(N.dtype_code(tex.dtype), mode, B, n, C, TH, TW, N.ptr(c),
                                                       N.ptr(tex), N.ptr(out), N.stream_of(tex.device)),
                    'texture_mapping')
        ctx.mode, ctx.n = mode, n
        ctx.save_for_backward(coords, texture_maps)  # the inputs themselves (double backward)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        c, tex = ctx.saved_tensors
        if torch.is_grad_enabled():  # create_graph: the reference's torch gradient, differentiable
            from ..._double_backward import texture_mapping as dd
            g = dd(c, tex, ctx.mode, grad_out)
            return g[0], g[1], None
        c, tex = c.contiguous(), tex.contiguous()
        B, C, TH, TW = tex.shape
        need_c, need_t, _ = ctx.needs_input_grad
        gc = torch.empty_like(c) if need_c else None
        gt = torch.empty_like(tex) if need_t else None
        if gc is None and gt is None:
            return None, None, None
        nbytes = N.size('kl_texture_mapping_bwd_workspace_bytes', B, C, TH, TW) if need_t else 0
        ws = N.workspace(nbytes, tex.device) if need_t else None
        with N.on_device(tex.device):
            N.check(N.lib().kl_texture_mapping_backward(
                N.dtype_code(tex.dtype), ctx.mode, B, ctx.n, C, TH, TW, N.ptr(grad_out.contiguous()), N.ptr(c),
                N.ptr(tex), N.ptr(gc), N.ptr(gt), N.ptr(ws), nbytes, N.stream_of(tex.device)),
                'texture_mapping backward')
        return gc, gt, None


def texture_mapping(texture_coordinates, texture_maps, mode='nearest'):
    r"""Sample ``texture_maps`` (B, C, h', w') at ``texture_coordinates`` (B, h, w, 2) or (B, N, 2)
    in OpenGL convention ([0, 1], y up) -> (B, h, w, C) / (B, N, C) (render/mesh/utils.py:23-75).

    The caller-side step after dibr_rasterization in the reference's tutorial loop
    (dibr_tutorial.ipynb cell 12): coordinates clamped to [0, 1], mapped to grid_sample's
    [-1, 1] with y reversed, border padding, align_corners=False.  GPU f32 / f64 tensors with
    mode 'nearest' or 'bilinear' run one HIP launch each way (TextureMappingHip); anything else
    runs the reference's torch chain."""
    batch_size = texture_coordinates.shape[0]
    num_channels = texture_maps.shape[1]
    if (texture_coordinates.is_cuda and texture_maps.is_cuda and texture_coordinates.device == texture_maps.device
            and mode in ('nearest', 'bilinear') and texture_maps.dtype in (torch.float32, torch.float64)
            and texture_coordinates.dtype == texture_maps.dtype and texture_maps.dim() == 4
            and texture_coordinates.shape[-1] == 2 and texture_maps.shape[0] == batch_size):
        ext = _ext.get()
        if ext is not None and N._TIMER is None and texture_maps.device.index == torch.cuda.current_device():
            out = ext.texture_mapping(texture_coordinates, texture_maps, 1 if mode == 'bilinear' else 0,
                                      N.stream_of(texture_maps.device))
        else:
            out = TextureMappingHip.apply(texture_coordinates, texture_maps, 1 if mode == 'bilinear' else 0)
        return out.reshape(batch_size, *texture_coordinates.shape[1:-1], num_channels)
    return _texture_mapping_torch(texture_coordinates, texture_maps, mode)


def _texture_mapping_torch(texture_coordinates, texture_maps, mode):
    """The reference's torch chain (utils.py:64-75)."""
    batch_size = texture_coordinates.shape[0]
    num_channels = texture_maps.shape[1]
    coords = texture_coordinates.reshape(batch_size, -1, 1, 2)
    coords = torch.clamp(coords, 0., 1.) * 2 - 1
    coords[..., 1] = -coords[..., 1]
    out = torch.nn.functional.grid_sample(texture_maps, coords, mode=mode, align_corners=False,
                                          padding_mode='border')
    return out.permute(0, 2, 3, 1).reshape(batch_size, *texture_coordinates.shape[1:-1], num_channels)
