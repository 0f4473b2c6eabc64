"""ctypes front-end for the CPU oracle (oracle/kaolin_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package (kaolin-windows_amd/).
All functions take / return numpy arrays and mirror the argument meaning of the
reference's ``kaolin._C`` entry points, plus the thin PyTorch
glue of the reference front-ends where a test needs the whole chain.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, '_build', 'libkaolin_oracle.so')
_lib = None

_P = ctypes.c_void_p


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.or_mesh_to_spc_leaves.restype = ctypes.c_int64
        _lib.or_morton_to_octree.restype = ctypes.c_int64
        _lib.or_raytrace.restype = ctypes.c_int64
        _lib.or_scan_octrees.restype = ctypes.c_int
        _lib.or_to_morton.restype = ctypes.c_uint64
        _lib.or_mesh_to_spc_leaves.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint, ctypes.c_void_p,
                                               ctypes.c_void_p]
        _lib.or_bary_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_uint, ctypes.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(_P) if a is not None else None


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _suffix(dtype):
    if dtype == np.float32:
        return 'f32'
    if dtype == np.float64:
        return 'f64'
    raise TypeError(f'oracle supports float32/float64, got {dtype}')


# ----------------------------------------------------------------- rasterize
def packed_rasterize_forward(height, width, fvz, fvi, bboxes, feat, first_idx, multiplier, eps):
    """rasterization.cpp:49-104 (packed inputs, coordinates already x multiplier)."""
    dt = np.asarray(fvz).dtype
    sfx = _suffix(dt)
    fvz, fvi, bboxes, feat = (_c(a, dt) for a in (fvz, fvi, bboxes, feat))
    first_idx = _c(first_idx, np.int64)
    B = first_idx.shape[0] - 1
    D = feat.shape[-1]
    out_feat = np.zeros((B, height, width, D), dt)
    out_idx = np.full((B, height, width), -1, np.int64)
    out_w = np.zeros((B, height, width, 3), dt)
    getattr(lib(), f'or_rasterize_fwd_{sfx}')(
        height, width, B, D, _p(fvz), _p(fvi), _p(bboxes), _p(feat), _p(first_idx),
        ctypes.c_float(multiplier), ctypes.c_float(eps), _p(out_feat), _p(out_idx), _p(out_w))
    return out_feat, out_idx, out_w


def rasterize_backward(grad_feat, face_idx, weights, fvi, feat, eps):
    """rasterization.cpp:106-168 (face_idx = original per-mesh face index)."""
    dt = np.asarray(grad_feat).dtype
    sfx = _suffix(dt)
    grad_feat, weights, fvi, feat = (_c(a, dt) for a in (grad_feat, weights, fvi, feat))
    face_idx = _c(face_idx, np.int64)
    B, H, W, D = grad_feat.shape
    F = fvi.shape[1]
    # the reference's float terms summed in double, rounded once (its atomics have no order)
    g_img = np.zeros(fvi.shape, np.float64)
    g_feat = np.zeros(feat.shape, np.float64)
    getattr(lib(), f'or_rasterize_bwd_{sfx}')(
        B, H, W, F, D, _p(grad_feat), _p(face_idx), _p(weights), _p(fvi), _p(feat),
        ctypes.c_float(eps), _p(g_img), _p(g_feat))
    return g_img.astype(dt), g_feat.astype(dt)


def rasterize(height, width, fvz, fvi, feat, valid_faces=None, multiplier=1000, eps=1e-8):
    """Whole rasterize() chain of rasterization.py:290-369 in numpy + the oracle kernel.
    Returns (features, face_idx, weights)."""
    dt = np.asarray(fvz).dtype
    B, F = fvz.shape[:2]
    D = feat.shape[-1]
    if valid_faces is None:
        valid_faces = np.ones((B, F), bool)
    bi, fi = np.nonzero(valid_faces)
    vfvi = fvi[bi, fi] * dt.type(multiplier)
    vfvz = fvz[bi, fi]
    vfeat = feat[bi, fi]
    first = np.zeros(B + 1, np.int64)
    first[1:] = np.cumsum(valid_faces.reshape(B, -1).sum(1))
    bbox = np.concatenate([vfvi.min(1), vfvi.max(1)], 1)
    out_feat, sel, w = packed_rasterize_forward(height, width, vfvz, vfvi, bbox, vfeat.reshape(-1, 3, D),
                                                first, multiplier, eps)
    face_idx = np.where(sel >= 0, fi[np.clip(sel + first[:-1, None, None], 0, max(len(fi) - 1, 0))] if len(fi) else -1, -1)
    return out_feat, face_idx.astype(np.int64), w


# ----------------------------------------------------------------- soft mask
def dibr_soft_mask_forward(fvi_m, bboxes, sel, sigmainv, knum, multiplier):
    """dibr_soft_mask.cpp:48-108 (fvi_m / bboxes already x multiplier)."""
    dt = np.asarray(fvi_m).dtype
    sfx = _suffix(dt)
    fvi_m, bboxes = _c(fvi_m, dt), _c(bboxes, dt)
    sel = _c(sel, np.int64)
    B, F = fvi_m.shape[:2]
    H, W = sel.shape[1:]
    mask = np.zeros((B, H, W), dt)
    prob = np.zeros((B, H, W, knum), dt)
    cidx = np.full((B, H, W, knum), -1, np.int64)
    ctype = np.zeros((B, H, W, knum), np.uint8)
    getattr(lib(), f'or_soft_mask_fwd_{sfx}')(
        B, H, W, F, knum, _p(fvi_m), _p(bboxes), _p(sel), ctypes.c_float(sigmainv),
        ctypes.c_float(multiplier), _p(mask), _p(prob), _p(cidx), _p(ctype))
    return mask, prob, cidx, ctype


def dibr_soft_mask_backward(grad, mask, sel, prob, cidx, ctype, fvi_m, sigmainv, multiplier):
    dt = np.asarray(grad).dtype
    sfx = _suffix(dt)
    grad, mask, prob, fvi_m = (_c(a, dt) for a in (grad, mask, prob, fvi_m))
    sel, cidx = _c(sel, np.int64), _c(cidx, np.int64)
    ctype = _c(ctype, np.uint8)
    B, F = fvi_m.shape[:2]
    H, W = sel.shape[1:]
    K = cidx.shape[-1]
    g = np.zeros(fvi_m.shape, np.float64)  # float terms summed in double, rounded once
    getattr(lib(), f'or_soft_mask_bwd_{sfx}')(
        B, H, W, F, K, _p(grad), _p(mask), _p(sel), _p(prob), _p(cidx), _p(ctype), _p(fvi_m),
        ctypes.c_float(sigmainv), ctypes.c_float(multiplier), _p(g))
    return g.astype(dt)


def soft_mask_bboxes(fvi, boxlen, multiplier):
    """dibr.py:31-39 glue: scale by multiplier and enlarge the bounding boxes."""
    dt = np.asarray(fvi).dtype
    fm = fvi * dt.type(multiplier)
    pmin = fm.min(-2)
    pmax = fm.max(-2)
    bl = dt.type(boxlen * multiplier)
    return fm, np.concatenate([pmin - bl, pmax + bl], -1)


# ----------------------------------------------------------------- distances
def unbatched_triangle_distance_forward(points, face_vertices):
    dt = np.asarray(points).dtype
    sfx = _suffix(dt)
    points, fv = _c(points, dt), _c(face_vertices, dt)
    P, F = points.shape[0], fv.shape[0]
    dist = np.zeros(P, dt)
    idx = np.zeros(P, np.int64)
    typ = np.zeros(P, np.int32)
    getattr(lib(), f'or_p2m_fwd_{sfx}')(P, F, _p(points), _p(fv), _p(dist), _p(idx), _p(typ))
    return dist, idx, typ


def unbatched_triangle_distance_backward(grad, points, face_vertices, idx, typ):
    dt = np.asarray(points).dtype
    sfx = _suffix(dt)
    grad, points, fv = _c(grad, dt), _c(points, dt), _c(face_vertices, dt)
    idx, typ = _c(idx, np.int64), _c(typ, np.int32)
    gp = np.zeros_like(points)
    gf = np.zeros_like(fv)
    getattr(lib(), f'or_p2m_bwd_{sfx}')(points.shape[0], fv.shape[0], _p(grad), _p(points), _p(fv),
                                        _p(idx), _p(typ), _p(gp), _p(gf))
    return gp, gf


def sided_distance_forward(p1, p2):
    dt = np.asarray(p1).dtype
    sfx = _suffix(dt)
    p1, p2 = _c(p1, dt), _c(p2, dt)
    B, N, M = p1.shape[0], p1.shape[1], p2.shape[1]
    dist = np.zeros((B, N), dt)
    idx = np.zeros((B, N), np.int64)
    getattr(lib(), f'or_sided_fwd_{sfx}')(B, N, M, _p(p1), _p(p2), _p(dist), _p(idx))
    return dist, idx


def sided_distance_backward(grad, p1, p2, idx):
    dt = np.asarray(p1).dtype
    sfx = _suffix(dt)
    grad, p1, p2 = _c(grad, dt), _c(p1, dt), _c(p2, dt)
    idx = _c(idx, np.int64)
    B, N, M = p1.shape[0], p1.shape[1], p2.shape[1]
    g1 = np.zeros_like(p1)
    g2 = np.zeros_like(p2)
    getattr(lib(), f'or_sided_bwd_{sfx}')(B, N, M, _p(grad), _p(p1), _p(p2), _p(idx), _p(g1), _p(g2))
    return g1, g2


# ----------------------------------------------------------------------- SPC
def to_morton(points):
    pts = np.asarray(points)
    return np.array([lib().or_to_morton(int(x), int(y), int(z)) for x, y, z in pts], np.uint64)


def morton_to_octree(mortons, level):
    m = _c(mortons, np.uint64)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = lib().or_morton_to_octree(_p(m), m.shape[0], level, ctypes.byref(out))
    res = np.ctypeslib.as_array(out, shape=(max(n, 1),))[:n].copy()
    lib().or_free(out)
    return res


def mesh_to_spc(face_vertices, level):
    """mesh_to_spc.cpp:28-44 -> (octree u8, face_idx i64, bary f32 (N,2)); empty -> (0,),(0,),(0,3)."""
    fv = _c(face_vertices, np.float32)
    pm = ctypes.POINTER(ctypes.c_uint64)()
    pf = ctypes.POINTER(ctypes.c_int64)()
    n = lib().or_mesh_to_spc_leaves(_p(fv), fv.shape[0], level, ctypes.byref(pm), ctypes.byref(pf))
    if n == 0:
        return np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros((0, 3), np.float32)
    mort = np.ctypeslib.as_array(pm, shape=(n,)).copy()
    face = np.ctypeslib.as_array(pf, shape=(n,)).copy()
    lib().or_free(pm)
    lib().or_free(pf)
    bary = np.zeros((n, 2), np.float32)
    lib().or_bary_batch(_p(fv), _p(mort), _p(face), n, level, _p(bary))
    return morton_to_octree(mort, level), face, bary


def m2s_rsqrt_sensitivity(face_vertices, level):
    """Counts of mesh_to_spc SAT decisions sensitive to the edge normalisation's rounding
    (kaolin_oracle.c:or_m2s_rsqrt_sensitivity): proposals, near-threshold proposals, flips
    with every 1/sqrt one ulp up, one ulp down, flips at the leaf level."""
    fv = _c(face_vertices, np.float32)
    out = np.zeros(5, np.int64)
    lib().or_m2s_rsqrt_sensitivity(_p(fv), ctypes.c_int64(fv.shape[0]), ctypes.c_uint(level), _p(out))
    return dict(zip(('proposals', 'near_threshold', 'flips_ulp_up', 'flips_ulp_down', 'flips_at_leaf_level'),
                    (int(x) for x in out)))


def scan_octrees(octrees, lengths):
    o = _c(octrees, np.uint8)
    ln = _c(lengths, np.int32)
    B = ln.shape[0]
    pyr = np.zeros((B, 2, 17), np.int32)
    ex = np.zeros(int(ln.sum()) + B, np.int32)
    level = lib().or_scan_octrees(_p(o), _p(ln), B, _p(pyr), _p(ex))
    return level, np.ascontiguousarray(pyr[:, :, :level + 2]), ex


def generate_points(octrees, pyramids, exsum):
    o = _c(octrees, np.uint8)
    pyr = _c(pyramids, np.int32)
    ex = _c(exsum, np.int32)
    B, L = pyr.shape[0], pyr.shape[2] - 2
    total = int(pyr[:, 1, L + 1].sum())
    pts = np.zeros((total, 3), np.int16)
    lib().or_generate_points(_p(o), _p(pyr), B, L, _p(ex), _p(pts))
    return pts


def raytrace(octree, points, pyramid, exsum, origin, direction, level, return_depth=True, with_exit=False):
    """raytrace.cpp:170-214 -> nuggets (N,2) int32 [, depth (N,1|2) f32]."""
    o = _c(octree, np.uint8)
    pts = _c(points, np.int16)
    ex = _c(exsum, np.int32)
    ro = _c(origin, np.float32)
    rd = _c(direction, np.float32)
    pn = ctypes.POINTER(ctypes.c_int32)()
    pd = ctypes.POINTER(ctypes.c_float)()
    n = lib().or_raytrace(_p(o), _p(pts), _p(ex), _p(ro), _p(rd), ro.shape[0], level,
                          int(return_depth), int(with_exit), ctypes.byref(pn), ctypes.byref(pd))
    dd = 2 if with_exit else 1
    nug = np.ctypeslib.as_array(pn, shape=(max(n, 1) * 2,))[:2 * n].reshape(n, 2).copy()
    lib().or_free(pn)
    if return_depth:
        dep = np.ctypeslib.as_array(pd, shape=(max(n, 1) * dd,))[:n * dd].reshape(n, dd).copy()
        lib().or_free(pd)
        return nug, dep
    return (nug,)


def voxelgrid(vertices, faces, resolution, origin=None, scale=None):
    """trianglemeshes_to_voxelgrids (float32): dense (B,R,R,R) uint8 occupancy."""
    v = _c(vertices, np.float32)
    f = _c(faces, np.int64)
    B, V = v.shape[:2]
    R = int(resolution)
    grid = np.zeros((B, R, R, R), np.uint8)
    o = _c(origin, np.float32) if origin is not None else None
    s = _c(scale, np.float32) if scale is not None else None
    lib().or_voxelgrid_f32(_p(v), B, V, _p(f), f.shape[0], R, _p(o), _p(s), _p(grid))
    return grid


# ---------------------------------------------------------------------------------------------
# Packed ray ops (render/spc/raytrace.py:86-296; kernels raytrace_cuda.cu:309-483).  numpy
# restatement: each pack is walked row by row in the reference kernels' order, operand order
# `in op prev`, arithmetic in the feature dtype (float16 rounds after every step).
def pack_starts(boundaries):
    """torch.nonzero(boundaries)[..., 0] (raytrace.py:176,199)."""
    return np.nonzero(np.asarray(boundaries))[0]


def _pack_ranges(starts, n):
    starts = [int(s) for s in starts]
    ends = starts[1:] + [n]
    return list(zip(starts, ends))


def pack_diff(feats, starts):
    """diff_cuda_kernel (raytrace_cuda.cu:309-325): zeros outside packs and on each pack's last row."""
    feats = np.asarray(feats)
    out = np.zeros_like(feats)
    for b, e in _pack_ranges(starts, feats.shape[0]):
        for i in range(b, e - 1):
            out[i] = feats[i + 1] - feats[i]
    return out


def inclusive_sum(info):
    """cub::DeviceScan::InclusiveSum over int32 (raytrace_cuda.cu:650-663)."""
    return np.cumsum(np.asarray(info, dtype=np.int64)).astype(np.int32)


def sum_reduce(feats, isum):
    """sum_reduce_cuda_kernel (raytrace_cuda.cu:327-346) with the adds in row order (the
    reference's atomics are unordered); out has isum[-1] rows."""
    feats = np.asarray(feats)
    cnt = int(isum[-1]) if len(isum) else 0
    out = np.zeros((cnt,) + feats.shape[1:], dtype=feats.dtype)
    for i in range(feats.shape[0]):
        r = int(isum[i]) - 1
        if 0 <= r < cnt:
            out[r] = out[r] + feats[i]
    return out


def pack_scan(feats, starts, exclusive, reverse, op):
    """cumsum / cumprod kernels (raytrace_cuda.cu:391-483); op 'sum' or 'prod'.  Output
    initialised as the reference's at::zeros / at::ones."""
    feats = np.asarray(feats)
    f = (lambda a, b: a + b) if op == 'sum' else (lambda a, b: a * b)
    out = (np.zeros_like(feats) if op == 'sum' else np.ones_like(feats))
    off = 1 if exclusive else 0
    for b, e in _pack_ranges(starts, feats.shape[0]):
        if b >= e:
            continue
        if not reverse:
            if not off:
                out[b] = feats[b]
            for i in range(b + 1, e):
                out[i] = f(feats[i - off], out[i - 1])
        else:
            if not off:
                out[e - 1] = feats[e - 1]
            for i in range(e - 2, b - 1, -1):
                out[i] = f(feats[i + off], out[i + 1])
    return out


# ---------------------------------------------------------------------------------------------
# DefTet sparse render (render/mesh/deftet.py:269-417; kernels deftet_cuda.cu:32-190, 240-420).
# numpy restatement in the input dtype, no fused multiply-add (every product and sum rounded,
# as the HIP build with -ffp-contract=off).  Loops over pixels, vectorised over faces.
def _copysign_eps_f(eps, v, dtype):
    # copysignf((double)eps, (double)v): both operands rounded to float (deftet_cuda.cu fwd)
    return np.copysign(np.float32(eps), v.astype(np.float32)).astype(dtype)


def deftet_sparse_render_forward(fvz, fvi, bboxes, pix, ranges, knum, eps=1e-8):
    """deftet_sparse_render_forward_cuda (deftet.cpp:49-111): the first knum hits in MESH order.
    bboxes may be None (min / max over the vertices, deftet.py:290-292).
    Returns face_idx (B,P,K) int64 (-1 pad), depth (-inf pad), w0, w1 (0 pad)."""
    with np.errstate(invalid='ignore', divide='ignore'):  # NaN / inf faces give NaN weights, as on the GPU
        return _deftet_sparse_render_forward(fvz, fvi, bboxes, pix, ranges, knum, eps)


def _deftet_sparse_render_forward(fvz, fvi, bboxes, pix, ranges, knum, eps):
    dt = fvz.dtype
    B, F = fvz.shape[:2]
    P = pix.shape[1]
    K = int(knum)
    if bboxes is None:
        bboxes = np.concatenate([fvi.min(axis=2), fvi.max(axis=2)], axis=-1)
    idx = np.full((B, P, K), -1, np.int64)
    depth = np.full((B, P, K), -np.inf, dt)
    w0o = np.zeros((B, P, K), dt)
    w1o = np.zeros((B, P, K), dt)
    for b in range(B):
        ax, ay, bx, by, cx, cy = (fvi[b, :, v // 2, v % 2] for v in range(6))
        az, bz, cz = fvz[b, :, 0], fvz[b, :, 1], fvz[b, :, 2]
        bb = bboxes[b]
        for p in range(P):
            x0, y0 = pix[b, p, 0], pix[b, p, 1]
            lo, hi = ranges[b, p, 0], ranges[b, p, 1]
            f = np.nonzero((x0 >= bb[:, 0]) & (x0 < bb[:, 2]) & (y0 >= bb[:, 1]) & (y0 < bb[:, 3]))[0]
            if f.size == 0:
                continue
            aex, aey = ax[f] - x0, ay[f] - y0
            bex, bey = bx[f] - x0, by[f] - y0
            cex, cey = cx[f] - x0, cy[f] - y0
            _w0 = bex * cey - bey * cex
            _w1 = cex * aey - cey * aex
            _w2 = aex * bey - aey * bex
            norm = _w0 + _w1 + _w2
            den = norm + _copysign_eps_f(eps, norm, dt)
            w0, w1, w2 = _w0 / den, _w1 / den, _w2 / den
            d = w0 * az[f] + w1 * bz[f] + w2 * cz[f]
            ok = (w0 >= 0) & (w1 >= 0) & (w2 >= 0) & (d < hi) & (d >= lo)
            sel = np.nonzero(ok)[0][:K]
            n = sel.size
            idx[b, p, :n] = f[sel]
            depth[b, p, :n] = d[sel]
            w0o[b, p, :n] = w0[sel]
            w1o[b, p, :n] = w1[sel]
    return idx, depth, w0o, w1o


def deftet_resolve(idx, depth, w0, w1, feat):
    """deftet.py:294-306: stable descending depth order, weights (w0, w1, 1 - (w0 + w1)) and
    interpolated features (w0 f0 + w1 f1) + w2 f2.  Returns (sorted_idx, weights, features)."""
    dt = feat.dtype
    B, P, K = idx.shape
    order = np.argsort(-depth, axis=-1, kind='stable')
    sidx = np.take_along_axis(idx, order, -1)
    sw0 = np.take_along_axis(w0, order, -1)
    sw1 = np.take_along_axis(w1, order, -1)
    sw2 = (sidx != -1).astype(dt) - (sw0 + sw1)
    weights = np.stack([sw0, sw1, sw2], axis=-1)
    padded = np.concatenate([np.zeros_like(feat[:, :1]), feat], axis=1)  # (B,F+1,3,D)
    sel = np.stack([padded[b][sidx[b] + 1] for b in range(B)])  # (B,P,K,3,D)
    interp = sw0[..., None] * sel[..., 0, :] + sw1[..., None] * sel[..., 1, :] + sw2[..., None] * sel[..., 2, :]
    return sidx, weights, interp


def deftet_sparse_render(pix, ranges, fvz, fvi, feat, knum=300, eps=1e-8):
    """DeftetSparseRenderer.forward: (interpolated_features, sorted_face_idx, weights)."""
    idx, depth, w0, w1 = deftet_sparse_render_forward(fvz, fvi, None, pix, ranges, knum, eps)
    sidx, weights, interp = deftet_resolve(idx, depth, w0, w1, feat)
    return interp, sidx, weights


def deftet_sparse_render_backward(grad, idx, weights, fvi, feat, eps=1e-8):
    """deftet_sparse_render_backward_cuda (deftet_cuda.cu:240-420), per (pixel, slot) item with a
    face, accumulated in item order (the reference's atomics are unordered)."""
    dt = fvi.dtype
    B, P, K, D = grad.shape
    F = fvi.shape[1]
    g_img = np.zeros_like(fvi)
    g_feat = np.zeros_like(feat)
    bi, pi, ki = np.nonzero(idx >= 0)
    if bi.size == 0:
        return g_img, g_feat
    fid = idx[bi, pi, ki]
    g = grad[bi, pi, ki]  # (N,D)
    w = weights[bi, pi, ki]  # (N,3)
    for ii in range(3):
        np.add.at(g_feat, (bi, fid, ii), g * w[:, ii:ii + 1])
    im = fvi[bi, fid].reshape(-1, 6)
    ax, ay, bx, by, cx, cy = (im[:, c] for c in range(6))
    aw, bw, cw = w[:, 0], w[:, 1], w[:, 2]
    x0 = aw * ax + bw * bx + cw * cx
    y0 = aw * ay + bw * by + cw * cy
    m, p, n, q, s, t = bx - ax, by - ay, cx - ax, cy - ay, x0 - ax, y0 - ay
    k1 = s * q - n * t
    k2 = m * t - s * p
    k3 = m * q - n * p
    k3 = (k3.astype(np.float64) + np.copysign(np.float64(np.float32(eps)), k3.astype(np.float64))).astype(dt)
    z = np.zeros_like(k3)
    dk1 = dict(m=z, n=-t, p=z, q=s, s=q, t=-n)
    dk2 = dict(m=t, n=z, p=-s, q=z, s=-p, t=m)
    dk3 = dict(m=q, n=-p, p=-n, q=m, s=z, t=z)
    dw1 = {v: dk1[v] * k3 - dk3[v] * k1 for v in 'mnpqst'}
    dw2 = {v: dk2[v] * k3 - dk3[v] * k2 for v in 'mnpqst'}
    d1 = [-(dw1['m'] + dw1['n'] + dw1['s']), -(dw1['p'] + dw1['q'] + dw1['t']), dw1['m'], dw1['p'], dw1['n'],
          dw1['q']]
    d2 = [-(dw2['m'] + dw2['n'] + dw2['s']), -(dw2['p'] + dw2['q'] + dw2['t']), dw2['m'], dw2['p'], dw2['n'],
          dw2['q']]
    fa = feat[bi, fid]  # (N,3,D)
    c0, c1, c2 = fa[:, 0], fa[:, 1], fa[:, 2]
    dldI = g / (k3 * k3)[:, None]
    acc = np.zeros((bi.size, 6), dt)
    for c in range(D):
        for v in range(6):
            dI = (c1[:, c] - c0[:, c]) * d1[v] + (c2[:, c] - c0[:, c]) * d2[v]
            acc[:, v] = acc[:, v] + dldI[:, c] * dI
    np.add.at(g_img.reshape(B, F, 6), (bi, fid), acc)
    return g_img, g_feat


# ---------------------------------------------------------------------------------------------
# check_sign (ops/mesh/check_sign.py:25-154; kernel mesh_intersection_cuda.cu:40-210).  numpy
# restatement in the input dtype, per point vectorised over the faces, operations in the
# kernel's order (crossing counts are integers: bit-exact).
def _cs_signed_area(ax, ay, bx, by, cx, cy):
    flip = (cx > bx) | ((bx == cx) & (cy < by))
    a = -((by - cy) * (ax - cx) + (cx - bx) * (ay - cy))
    b = (cy - by) * (ax - bx) + (bx - cx) * (ay - by)
    return np.where(flip, a, b)


def _cs_above(vx, vy, lx, ly, rx, ry):
    v1x, v1y = rx - lx, ry - ly
    v2x, v2y = vx - lx, vy - ly
    return (v1x * v2y - v1y * v2x) > 0


def _cs_signed_volume(ax, ay, az, b, c, d):
    """signed_volume(a, b, c, d) = dot(cross(b - a, c - a), d - a) (mesh_intersection_cuda.cu:60-66)."""
    ux, uy, uz = b[:, 0] - ax, b[:, 1] - ay, b[:, 2] - az
    vx, vy, vz = c[:, 0] - ax, c[:, 1] - ay, c[:, 2] - az
    nx, ny, nz = uy * vz - uz * vy, uz * vx - ux * vz, ux * vy - uy * vx
    return nx * (d[:, 0] - ax) + ny * (d[:, 1] - ay) + nz * (d[:, 2] - az)


def mesh_intersection_counts(points, v1, v2, v3):
    """unbatched_mesh_intersection_cuda: (P,) crossing counts (as int64)."""
    dt = points.dtype
    f32 = np.float32
    ymin = np.minimum(v1[:, 1], np.minimum(v2[:, 1], v3[:, 1])).astype(f32).astype(dt)
    ymax = np.maximum(v1[:, 1], np.maximum(v2[:, 1], v3[:, 1])).astype(f32).astype(dt)
    zmin = np.minimum(v1[:, 2], np.minimum(v2[:, 2], v3[:, 2])).astype(f32).astype(dt)
    zmax = np.maximum(v1[:, 2], np.maximum(v2[:, 2], v3[:, 2])).astype(f32).astype(dt)
    out = np.zeros(points.shape[0], np.int64)
    ten = dt.type(10.)
    for i, (qx, qy, qz) in enumerate(points):
        f = np.nonzero(~((qy < ymin) | (ymax < qy) | (qz < zmin) | (zmax < qz)))[0]
        if f.size == 0:
            continue
        a, b, c = v1[f], v2[f], v3[f]
        c1 = _cs_signed_volume(qx, qy, qz, a, b, c) > 0
        c2 = _cs_signed_volume(qx + ten, qy, qz, a, b, c) > 0
        d1 = _cs_signed_area(qy, qz, a[:, 1], a[:, 2], b[:, 1], b[:, 2])
        d2 = _cs_signed_area(qy, qz, b[:, 1], b[:, 2], c[:, 1], c[:, 2])
        d3 = _cs_signed_area(qy, qz, c[:, 1], c[:, 2], a[:, 1], a[:, 2])
        inside = (c1 != c2) & (d1 * d2 >= 0) & (d3 * d1 >= 0) & (d2 * d3 >= 0)
        cnt = 0
        for j in np.nonzero(inside)[0]:
            p = [(a[j, 1], a[j, 2]), (b[j, 1], b[j, 2]), (c[j, 1], c[j, 2])]
            on_v = on_e = False
            if (qy, qz) == p[0]:
                on_v, v1_, v2_ = True, p[1], p[2]
            elif (qy, qz) == p[1]:
                on_v, v1_, v2_ = True, p[0], p[2]
            elif (qy, qz) == p[2]:
                on_v, v1_, v2_ = True, p[0], p[1]
            elif d1[j] == 0:
                on_e, v1_, v2_, o = True, p[0], p[1], p[2]
            elif d2[j] == 0:
                on_e, v1_, v2_, o = True, p[1], p[2], p[0]
            elif d3[j] == 0:
                on_e, v1_, v2_, o = True, p[2], p[0], p[1]
            if not (on_v or on_e):
                cnt += 1
                continue
            if v1_[0] > v2_[0] or (v1_[0] == v2_[0] and v1_[1] > v2_[1]):
                v1_, v2_ = v2_, v1_
            if on_e:
                cnt += 0 if _cs_above(o[0], o[1], v1_[0], v1_[1], v2_[0], v2_[1]) else 1
            else:
                cnt += 1 if (_cs_above(qy, qz, v1_[0], v1_[1], v2_[0], v2_[1]) and v1_[0] < qy
                             and v2_[0] >= qy) else 0
        out[i] = cnt
    return out


def check_sign(verts, faces, points):
    """check_sign.py:140-154 (GPU branch): (B,P) bool."""
    res = []
    for b in range(verts.shape[0]):
        maxlen = (verts[b].max(0) - verts[b].min(0)).max()
        v = verts[b] / maxlen
        p = points[b] / maxlen
        cnt = mesh_intersection_counts(p, v[faces[:, 0]], v[faces[:, 1]], v[faces[:, 2]])
        res.append(cnt % 2 == 1)
    return np.stack(res)


# ------------------------------------------------------------ compact soft-mask state (GPU)
# The checker's view of the GPU forward's saved state (softtile.hip layout, kaolin_hip.h):
# decode_compact() rebuilds the reference's (B,H,W,K) slot tensors from it, so that the oracle's
# soft-mask backward can run on the GPU forward's own saved values.
def decode_compact(hits, rec_face, rec_prob, K, rows=None):
    """(hits (B,H,W) u8, rec_face u32, rec_prob) -> idx (B,H,W,K) int64 (-1 pad), type u8 (0 pad),
    prob (0 pad), for all rows or only `rows` (the others left as padding)."""
    hits = np.asarray(hits).astype(np.int64)
    rf = np.asarray(rec_face).view(np.uint32)
    rp = np.asarray(rec_prob)
    B, H, W = hits.shape
    tx = (W + 63) // 64
    rows = np.arange(H) if rows is None else np.asarray(rows)
    idx = np.full((B, H, W, K), -1, np.int64)
    typ = np.zeros((B, H, W, K), np.uint8)
    prob = np.zeros((B, H, W, K), rp.dtype)
    if K == 0 or len(rows) == 0:
        return idx, typ, prob
    h = np.zeros((B, len(rows), tx * 64), np.int64)
    h[:, :, :W] = hits[:, rows]
    h = h.reshape(B, len(rows), tx, 64)
    pre = np.cumsum(h, -1) - h                                  # filled slots before the pixel
    seg = (np.arange(B)[:, None, None] * H + rows[None, :, None]) * tx + np.arange(tx)[None, None, :]
    base = (seg * 64 * K)[..., None] + pre                      # (B, R, tx, 64)
    R = len(rows)
    bi = np.full((B, R, W, K), -1, np.int64)
    bt = np.zeros((B, R, W, K), np.uint8)
    bp = np.zeros((B, R, W, K), rp.dtype)
    for k in range(K):
        sel = k < h
        pos = np.where(sel, base + k, 0)
        f = np.where(sel, rf[pos], 0).reshape(B, R, tx * 64)[:, :, :W]
        p = np.where(sel, rp[pos], 0).reshape(B, R, tx * 64)[:, :, :W]
        s = sel.reshape(B, R, tx * 64)[:, :, :W]
        bi[..., k] = np.where(s, (f & 0x0fffffff).astype(np.int64), -1)
        bt[..., k] = np.where(s, (f >> 28).astype(np.uint8), 0)
        bp[..., k] = np.where(s, p, 0)
    idx[:, rows] = bi
    typ[:, rows] = bt
    prob[:, rows] = bp
    return idx, typ, prob


# ------------------------------------------------------------ prepare_vertices (§8f rank 3)
def prepare_vertices(vertices, faces, camera_proj, camera_rot=None, camera_trans=None, camera_transform=None):
    """numpy restatement of render/mesh/utils.py:128-175 (float64 arithmetic on the given values):
    camera/legacy.py:35-36 (P - T) @ R^T or utils.py:163-167 [P, 1] @ M; legacy.py:136-137
    projection; ops/mesh/mesh.py:44-46 gather; ops/mesh/trianglemesh.py:328-334 unit normals.
    Broadcasts a batch of 1 as torch does.  -> (fvc (B,F,3,3), fvi (B,F,3,2), fn (B,F,3))."""
    v = np.asarray(vertices, np.float64)
    if camera_transform is None:
        t = np.asarray(camera_trans, np.float64).reshape(-1, 1, 3)
        r = np.asarray(camera_rot, np.float64)
        vc = np.matmul(v - t, np.transpose(r, (0, 2, 1)))
    else:
        m = np.asarray(camera_transform, np.float64)
        vc = np.matmul(np.concatenate([v, np.ones(v.shape[:-1] + (1,))], -1), m)
    pp = vc * np.asarray(camera_proj, np.float64).reshape(-1, 1, 3)
    vi = pp[:, :, :2] / pp[:, :, 2:3]
    f = np.asarray(faces, np.int64)
    fvc = vc[:, f]
    fvi = vi[:, f]
    n = np.cross(fvc[:, :, 1] - fvc[:, :, 0], fvc[:, :, 2] - fvc[:, :, 0])
    fn = n / (np.linalg.norm(n, axis=2, keepdims=True) + 1e-10)
    return fvc, fvi, fn
