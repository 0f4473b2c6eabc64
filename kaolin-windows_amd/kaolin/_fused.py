"""Fused DIB-R entry points used by the front-ends (not part of the reference's _C registry).

The reference front-ends run ~10 PyTorch ops around each native call: valid-face
packing with ``torch.where`` (a host sync), gathers, ``* multiplier``, bbox min/max/cat,
a cumsum for ``first_idx`` and a packed->original index remap (rasterization.py:309-367,
dibr.py:31-39).  These entry points take the unpacked inputs and do all of it inside
the HIP kernels with the same float operations, so the results are identical to the
unfused chain (tests/test_gpu_parity.py checks both against the oracle).
"""
import torch

from . import _native as N


_ws = N.workspace


def _valid_u8(valid_faces):
    if valid_faces is None:
        return None
    valid = valid_faces.contiguous()
    return valid.view(torch.uint8) if valid.dtype == torch.bool else (valid != 0).view(torch.uint8)


def _validity(valid_faces, face_normals_z, dtype):
    """(uint8 valid mask, face_normals_z for the in-kernel `>= 0` test): exactly one is used."""
    if valid_faces is not None or face_normals_z is None:
        return _valid_u8(valid_faces), None
    if face_normals_z.dtype != dtype:  # the in-kernel test reads the tensor dtype
        return _valid_u8(face_normals_z >= 0), None
    return None, face_normals_z.contiguous()


def rasterize_forward(height, width, face_vertices_z, face_vertices_image, face_features, valid_faces, multiplier,
                      eps, face_normals_z=None):
    """-> interpolated_features (B,H,W,D), face_idx (B,H,W) original index, output_weights (B,H,W,3).
    With ``valid_faces`` None and ``face_normals_z`` given, valid = face_normals_z >= 0 in-kernel."""
    func = 'rasterize'
    N.require_gpu(func, face_vertices_z)
    B, F = face_vertices_z.shape[:2]
    D = face_features.shape[-1]
    dev = face_vertices_z.device
    dtype = face_vertices_z.dtype
    if dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f'"{func}" not implemented for {dtype}')
    for name, t in (('face_vertices_image', face_vertices_image), ('face_features', face_features)):
        if t.dtype != dtype:  # the reference's data_ptr<scalar_t>() check (rasterization_cuda.cu)
            raise RuntimeError(f'{func}: expected {name} of dtype {dtype} (face_vertices_z), found {t.dtype}')
    fvz = face_vertices_z.contiguous()
    fvi = face_vertices_image.contiguous()
    feat = face_features.contiguous()
    valid, fnz = _validity(valid_faces, face_normals_z, dtype)
    feats = torch.empty((B, height, width, D), dtype=dtype, device=dev)
    idx = torch.empty((B, height, width), dtype=torch.long, device=dev)
    w = torch.empty((B, height, width, 3), dtype=dtype, device=dev)
    lib = N.lib()
    nbytes = lib.kl_dibr_rasterize_workspace_bytes(B, height, width, F)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_rasterize_forward', dev):
        N.check(lib.kl_dibr_rasterize_forward(
            N.dtype_code(dtype), height, width, B, F, D, N.ptr(fvz), N.ptr(fvi), N.ptr(feat), N.ptr(valid),
            N.ptr(fnz), float(multiplier), float(eps), N.ptr(feats), N.ptr(idx), N.ptr(w), N.ptr(ws), nbytes, N.stream_of(dev)),
            func)
    return feats, idx, w


def rasterize_backward(grad, face_idx, weights, face_vertices_image, face_features, valid_faces, multiplier, eps,
                       face_normals_z=None, scratch=None, face_ranges=None):
    """Gather backward; valid_faces / face_normals_z / multiplier must be the forward's.
    ``scratch``: the zeroed int32 of a compact soft-mask state (see soft_mask_forward_compact).
    ``face_ranges``: the per-face pixel ranges dibr_forward returned (reused, not recomputed)."""
    func = 'rasterize backward'
    B, H, W, D = grad.shape
    F = face_vertices_image.shape[1]
    dev = face_vertices_image.device
    g_img = torch.empty_like(face_vertices_image)
    g_feat = torch.empty_like(face_features)
    valid, fnz = _validity(valid_faces, face_normals_z, face_vertices_image.dtype)
    lib = N.lib()
    nbytes = lib.kl_dibr_rasterize_bwd_workspace_bytes(B, H, W, F, D)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_rasterize_backward', dev):
        N.check(lib.kl_dibr_rasterize_backward(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, D, N.ptr(grad.contiguous()), N.ptr(face_idx),
            N.ptr(weights), N.ptr(face_vertices_image), N.ptr(face_features), N.ptr(valid), N.ptr(fnz),
            float(multiplier), float(eps), N.ptr(g_img), N.ptr(g_feat), N.ptr(scratch), N.ptr(face_ranges), N.ptr(ws),
            nbytes, N.stream_of(dev)), func)
    return g_img, g_feat


def soft_mask_forward(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier, with_hits=False):
    """face_vertices_image UNSCALED -> soft_mask, close_face_prob, close_face_idx, close_face_dist_type
    (+ the per-pixel filled-slot counts, uint8, when ``with_hits``; None if knum > 255)."""
    func = 'dibr_soft_mask'
    N.require_gpu(func, face_vertices_image)
    fvi = face_vertices_image.contiguous()
    sel = selected_face_idx.contiguous()
    B, F = fvi.shape[:2]
    H, W = sel.shape[1:]
    dev = fvi.device
    dtype = fvi.dtype
    if dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f'"{func}" not implemented for {dtype}')
    K = int(knum)
    mask = torch.empty((B, H, W), dtype=dtype, device=dev)
    prob = torch.empty((B, H, W, K), dtype=dtype, device=dev)
    cidx = torch.empty((B, H, W, K), dtype=torch.long, device=dev)
    ctype = torch.empty((B, H, W, K), dtype=torch.uint8, device=dev)
    hits = torch.empty((B, H, W), dtype=torch.uint8, device=dev) if with_hits and K <= 255 else None
    lib = N.lib()
    nbytes = lib.kl_soft_mask_workspace_bytes(B, H, W, F)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_soft_mask_forward', dev):
        N.check(lib.kl_dibr_soft_mask_forward_fused(
            N.dtype_code(dtype), B, H, W, F, K, N.ptr(fvi), N.ptr(sel), float(sigmainv), float(boxlen * multiplier),
            float(multiplier), N.ptr(mask), N.ptr(prob), N.ptr(cidx), N.ptr(ctype), N.ptr(hits), N.ptr(ws), nbytes,
            N.stream_of(dev)), func)
    if with_hits:
        return mask, prob, cidx, ctype, hits
    return mask, prob, cidx, ctype


def soft_mask_backward(grad, mask, sel, prob, cidx, ctype, face_vertices_image, sigmainv, multiplier, hits=None):
    func = 'dibr_soft_mask backward'
    B, F = face_vertices_image.shape[:2]
    H, W = sel.shape[1:]
    K = cidx.shape[-1]
    dev = face_vertices_image.device
    g = torch.empty_like(face_vertices_image)
    nbytes = N.lib().kl_soft_mask_backward_workspace_bytes(B, F)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_soft_mask_backward', dev):
        N.check(N.lib().kl_dibr_soft_mask_backward_fused(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, K, N.ptr(grad.contiguous()), N.ptr(mask),
            N.ptr(sel), N.ptr(prob), N.ptr(cidx), N.ptr(ctype), N.ptr(hits), N.ptr(face_vertices_image), float(sigmainv),
            float(multiplier), N.ptr(g), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return g


class SoftMaskState:
    """The compact saved state of the soft mask (softtile.hip): per-pixel filled-slot
    counts, the per-hit records, the per-row-segment hit totals and ``scratch``: the zeroed
    int32 word of the standalone soft mask, or dibr_forward's state bytes (the backward's work
    items, kl_dibr_state_bytes)."""
    __slots__ = ('hits', 'rec_face', 'rec_prob', 'seg_tot', 'scratch', 'knum')

    def __init__(self, hits, rec_face, rec_prob, seg_tot, scratch, knum):
        self.hits, self.rec_face, self.rec_prob = hits, rec_face, rec_prob
        self.seg_tot, self.scratch, self.knum = seg_tot, scratch, knum

    def tensors(self):
        return self.hits, self.rec_face, self.rec_prob, self.seg_tot, self.scratch


def soft_mask_forward_compact(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier):
    """face_vertices_image UNSCALED -> soft_mask (B,H,W), SoftMaskState.  knum <= 255."""
    func = 'dibr_soft_mask'
    N.require_gpu(func, face_vertices_image, selected_face_idx)
    fvi = face_vertices_image.contiguous()
    sel = selected_face_idx.contiguous()
    B, F = fvi.shape[:2]
    H, W = sel.shape[1:]
    dev = fvi.device
    dtype = fvi.dtype
    if dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f'"{func}" not implemented for {dtype}')
    K = int(knum)
    lib = N.lib()
    mask = torch.empty((B, H, W), dtype=dtype, device=dev)
    hits = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    nrec = lib.kl_soft_mask_compact_records(B, H, W, K)
    rec_face = torch.empty(max(nrec, 1), dtype=torch.int32, device=dev)
    rec_prob = torch.empty(max(nrec, 1), dtype=dtype, device=dev)
    seg_tot = torch.empty(max(lib.kl_soft_mask_compact_segments(B, H, W), 1), dtype=torch.int32, device=dev)
    scratch = torch.empty(1, dtype=torch.int32, device=dev)
    nbytes = lib.kl_soft_mask_compact_workspace_bytes(B, H, W, F)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_soft_mask_forward', dev):
        N.check(lib.kl_dibr_soft_mask_forward_compact(
            N.dtype_code(dtype), B, H, W, F, K, N.ptr(fvi), N.ptr(sel), float(sigmainv), float(boxlen * multiplier),
            float(multiplier), N.ptr(mask), N.ptr(hits), N.ptr(rec_face), N.ptr(rec_prob), N.ptr(seg_tot),
            N.ptr(scratch), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return mask, SoftMaskState(hits, rec_face, rec_prob, seg_tot, scratch, K)


def soft_mask_backward_compact(grad, mask, state, face_vertices_image, sigmainv, multiplier, out=None):
    """-> grad_face_vertices_image (the terms summed in double, rounded once); with ``out`` that
    rounded sum is added onto it (returned), as autograd adds it to the rasterizer's gradient."""
    func = 'dibr_soft_mask backward'
    B, F = face_vertices_image.shape[:2]
    H, W = mask.shape[1:]
    dev = face_vertices_image.device
    g = out if out is not None else torch.empty_like(face_vertices_image)
    lib = N.lib()
    nbytes = lib.kl_soft_mask_compact_bwd_workspace_bytes(B, H, W, F, state.knum)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_soft_mask_backward', dev):
        N.check(lib.kl_dibr_soft_mask_backward_compact(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, state.knum, N.ptr(grad.contiguous()), N.ptr(mask),
            N.ptr(state.hits), N.ptr(state.rec_face), N.ptr(state.rec_prob), N.ptr(state.seg_tot),
            N.ptr(face_vertices_image), float(sigmainv), float(multiplier), N.ptr(g), 1 if out is not None else 0,
            N.ptr(state.scratch), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return g


def dibr_backward(grad_feats, grad_soft_mask, face_idx, weights, face_vertices_image, face_features, face_normals_z,
                  soft_mask, state, sigmainv, multiplier, eps, face_ranges=None):
    """dibr_rasterization's backward in one call (kl_dibr_backward): the soft-mask terms summed in
    double first, then the rasterizer's gather writes every face's gradient as its own rounded
    sum plus the soft mask's (as autograd adds the two).  grad_soft_mask may be None.
    -> grad_face_vertices_image, grad_face_features."""
    func = 'dibr_rasterization backward'
    B, H, W, D = grad_feats.shape
    F = face_vertices_image.shape[1]
    dev = face_vertices_image.device
    g_img = torch.empty_like(face_vertices_image)
    g_feat = torch.empty_like(face_features)
    lib = N.lib()
    nbytes = N.size('kl_dibr_bwd_workspace_bytes', B, H, W, F, state.knum)
    ws = _ws(nbytes, dev)
    gm = grad_soft_mask.contiguous() if grad_soft_mask is not None else None
    acc = N.zero_kept(N.size('kl_dibr_soft_acc_bytes', B, F), dev) if gm is not None else None
    with N.on_device(dev), N.timed('dibr_backward', dev):
        N.check(lib.kl_dibr_backward(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, D, state.knum, N.ptr(grad_feats.contiguous()),
            N.ptr(gm), N.ptr(face_idx), N.ptr(weights), N.ptr(face_vertices_image), N.ptr(face_features),
            N.ptr(face_normals_z), N.ptr(soft_mask), N.ptr(state.hits), N.ptr(state.rec_face), N.ptr(state.rec_prob),
            N.ptr(state.seg_tot), float(sigmainv), float(multiplier), float(eps), N.ptr(g_img), N.ptr(g_feat),
            N.ptr(state.scratch), N.ptr(face_ranges), N.ptr(acc), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return g_img, g_feat


def dibr_forward(height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z, sigmainv, boxlen,
                 knum, multiplier, eps):
    """dibr_rasterization's forward in one call (kl_dibr_forward): rasterize with valid =
    face_normals_z >= 0 and the compact soft mask, sharing one binning pass.
    -> features (B,H,W,D), face_idx (B,H,W), weights (B,H,W,3), soft_mask (B,H,W), SoftMaskState,
    face_ranges (B,F,2) int32 (each face's exact pixel ranges, for rasterize_backward).
    face_normals_z must have the dtype of face_vertices_image."""
    func = 'dibr_rasterization'
    N.require_gpu(func, face_vertices_z, face_vertices_image, face_normals_z)
    B, F = face_vertices_z.shape[:2]
    D = face_features.shape[-1]
    dev = face_vertices_z.device
    dtype = face_vertices_z.dtype
    if dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f'"{func}" not implemented for {dtype}')
    for name, t in (('face_vertices_image', face_vertices_image), ('face_features', face_features),
                    ('face_normals_z', face_normals_z)):
        if t.dtype != dtype:  # the reference's data_ptr<scalar_t>() check (rasterization_cuda.cu)
            raise RuntimeError(f'{func}: expected {name} of dtype {dtype} (face_vertices_z), found {t.dtype}')
    H, W, K = int(height), int(width), int(knum)
    fvz = face_vertices_z.contiguous()
    fvi = face_vertices_image.contiguous()
    feat = face_features.contiguous()
    fnz = face_normals_z.contiguous()
    lib = N.lib()
    feats = torch.empty((B, H, W, D), dtype=dtype, device=dev)
    idx = torch.empty((B, H, W), dtype=torch.long, device=dev)
    w = torch.empty((B, H, W, 3), dtype=dtype, device=dev)
    mask = torch.empty((B, H, W), dtype=dtype, device=dev)
    hits = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    nrec = N.size('kl_soft_mask_compact_records', B, H, W, K)
    rec_face = torch.empty(max(nrec, 1), dtype=torch.int32, device=dev)
    rec_prob = torch.empty(max(nrec, 1), dtype=dtype, device=dev)
    seg_tot = torch.empty(max(N.size('kl_soft_mask_compact_segments', B, H, W), 1), dtype=torch.int32, device=dev)
    # the fused path's state: the backward's soft-mask work items
    state = torch.empty(N.size('kl_dibr_state_bytes', B, H, W, F, K), dtype=torch.uint8, device=dev)
    ranges = torch.empty((B, F, 2), dtype=torch.int32, device=dev)
    nbytes = N.size('kl_dibr_workspace_bytes', B, H, W, F)
    ws = _ws(nbytes, dev)
    with N.on_device(dev), N.timed('dibr_forward', dev):
        N.check(lib.kl_dibr_forward(
            N.dtype_code(dtype), B, H, W, F, D, K, N.ptr(fvz), N.ptr(fvi), N.ptr(feat), N.ptr(fnz), float(sigmainv),
            float(boxlen * multiplier), float(multiplier), float(eps), N.ptr(feats), N.ptr(idx), N.ptr(w),
            N.ptr(mask), N.ptr(hits), N.ptr(rec_face), N.ptr(rec_prob), N.ptr(seg_tot), N.ptr(state),
            N.ptr(ranges if F > 0 else None), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return feats, idx, w, mask, SoftMaskState(hits, rec_face, rec_prob, seg_tot, state, K), ranges
