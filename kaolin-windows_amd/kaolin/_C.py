"""``kaolin._C`` for MI355X: the reference's pybind registry (bindings.cpp:37-99),
restricted to the hot path, re-implemented over the C ABI of libkaolin_hip.so.

Same submodule paths, function names, argument order, dtypes, output containers
(lists, or a tuple for scan_octrees_cuda), in/out-parameter conventions and
argument-check messages as the reference dispatchers cited on each function.
Outputs are allocated here with torch (caching allocator, current stream);
kernels run on ``torch.cuda.current_stream()`` of the input's device.
"""
import ctypes
import types

import torch

from . import _native as N
from ._checks import (Arg, check_all_same_gpu, check_contiguous, check_dim, check_same_size, check_same_type,
                      check_size, check_size_dim)

_FLOATS = (torch.float32, torch.float64)


def _float_only(func, t):
    if t.dtype not in _FLOATS:
        raise RuntimeError(f'"{func}" not implemented for \'{_tname(t.dtype)}\'')


def _tname(dtype):
    return {torch.float16: 'Half', torch.float32: 'Float', torch.float64: 'Double', torch.uint8: 'Byte',
            torch.int8: 'Char', torch.int16: 'Short', torch.int32: 'Int', torch.int64: 'Long'}.get(dtype, str(dtype))


# --------------------------------------------------------------------------- render.mesh
def packed_rasterize_forward_cuda(height, width, face_vertices_z, face_vertices_image, face_bboxes, face_features,
                                  first_idx_face_per_mesh, multiplier, eps, max_faces_per_mesh=None):
    """rasterization.cpp:49-104.  ``max_faces_per_mesh`` (extension, optional) bounds
    the per-mesh face count for the screen-space bins; default = total packed faces."""
    func = 'packed_rasterize_forward_cuda'
    args = [Arg(face_vertices_z, 'face_vertices_z', 3), Arg(face_vertices_image, 'face_vertices_image', 4),
            Arg(face_bboxes, 'face_bboxes', 5), Arg(face_features, 'face_features', 6),
            Arg(first_idx_face_per_mesh, 'first_idx_face_per_mesh', 7)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    num_faces = face_vertices_z.shape[0]
    batch_size = first_idx_face_per_mesh.shape[0] - 1
    feat_dim = face_features.shape[2]
    check_size(func, args[0], (num_faces, 3))
    check_size(func, args[1], (num_faces, 3, 2))
    check_size(func, args[2], (num_faces, 4))
    check_size(func, args[3], (num_faces, 3, feat_dim))
    check_size(func, args[4], (batch_size + 1,))
    _float_only(func, face_vertices_z)
    N.require_gpu(func, face_vertices_z)
    dev = face_vertices_z.device
    dtype = face_vertices_z.dtype
    feats = torch.empty((batch_size, height, width, feat_dim), dtype=dtype, device=dev)
    idx = torch.empty((batch_size, height, width), dtype=torch.long, device=dev)
    w = torch.empty((batch_size, height, width, 3), dtype=dtype, device=dev)
    maxf = int(max_faces_per_mesh) if max_faces_per_mesh is not None else max(int(num_faces), 1)
    lib = N.lib()
    ws_bytes = lib.kl_rasterize_workspace_bytes(batch_size, height, width, maxf)
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_packed_rasterize_forward(
            N.dtype_code(dtype), height, width, batch_size, num_faces, feat_dim, maxf,
            N.ptr(face_vertices_z), N.ptr(face_vertices_image), N.ptr(face_bboxes), N.ptr(face_features),
            N.ptr(first_idx_face_per_mesh), float(multiplier), float(eps), N.ptr(feats), N.ptr(idx), N.ptr(w),
            N.ptr(ws), ws_bytes, N.stream_of(dev)), func)
    return [feats, idx, w]


def rasterize_backward_cuda(grad_interpolated_features, interpolated_features, selected_face_idx, output_weights,
                            face_vertices_image, face_features, eps):
    """rasterization.cpp:106-168."""
    func = 'rasterize_backward_cuda'
    args = [Arg(grad_interpolated_features, 'grad_interpolated_features', 1),
            Arg(interpolated_features, 'interpolated_features', 2), Arg(selected_face_idx, 'selected_face_idx', 3),
            Arg(output_weights, 'output_weights', 4), Arg(face_vertices_image, 'face_vertices_image', 5),
            Arg(face_features, 'face_features', 6)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    B, H, W, D = grad_interpolated_features.shape
    F = face_vertices_image.shape[1]
    check_size(func, args[0], (B, H, W, D))
    check_size(func, args[1], (B, H, W, D))
    check_size(func, args[2], (B, H, W))
    check_size(func, args[3], (B, H, W, 3))
    check_size(func, args[4], (B, F, 3, 2))
    check_size(func, args[5], (B, F, 3, D))
    _float_only(func, grad_interpolated_features)
    N.require_gpu(func, grad_interpolated_features)
    dev = face_vertices_image.device
    g_img = torch.empty_like(face_vertices_image)
    g_feat = torch.empty_like(face_features)
    nbytes = N.lib().kl_rasterize_backward_workspace_bytes(B, F, D)
    ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(N.lib().kl_rasterize_backward(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, D, N.ptr(grad_interpolated_features),
            N.ptr(selected_face_idx), N.ptr(output_weights), N.ptr(face_vertices_image), N.ptr(face_features),
            float(eps), N.ptr(g_img), N.ptr(g_feat), N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return [g_img, g_feat]


def dibr_soft_mask_forward_cuda(face_vertices_image, face_large_bboxes, selected_face_idx, sigmainv, knum,
                                multiplier):
    """dibr_soft_mask.cpp:48-108."""
    func = 'dibr_soft_mask_forward_cuda'
    args = [Arg(face_vertices_image, 'face_vertices_image', 1), Arg(face_large_bboxes, 'face_bboxes', 2),
            Arg(selected_face_idx, 'selected_face_idx', 3)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:]
    check_size(func, args[0], (B, F, 3, 2))
    check_size(func, args[1], (B, F, 4))
    check_size(func, args[2], (B, H, W))
    _float_only(func, face_vertices_image)
    N.require_gpu(func, face_vertices_image)
    dev = face_vertices_image.device
    dtype = face_vertices_image.dtype
    K = int(knum)
    soft_mask = torch.empty((B, H, W), dtype=dtype, device=dev)
    prob = torch.empty((B, H, W, K), dtype=dtype, device=dev)
    cidx = torch.empty((B, H, W, K), dtype=torch.long, device=dev)
    ctype = torch.empty((B, H, W, K), dtype=torch.uint8, device=dev)
    lib = N.lib()
    ws_bytes = lib.kl_soft_mask_workspace_bytes(B, H, W, F)
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_dibr_soft_mask_forward(
            N.dtype_code(dtype), B, H, W, F, K, N.ptr(face_vertices_image), N.ptr(face_large_bboxes),
            N.ptr(selected_face_idx), float(sigmainv), float(multiplier), N.ptr(soft_mask), N.ptr(prob),
            N.ptr(cidx), N.ptr(ctype), N.ptr(ws), ws_bytes, N.stream_of(dev)), func)
    return [soft_mask, prob, cidx, ctype]


def dibr_soft_mask_backward_cuda(grad_soft_mask, soft_mask, selected_face_idx, close_face_prob, close_face_idx,
                                 close_face_dist_type, face_vertices_image, sigmainv, multiplier):
    """dibr_soft_mask.cpp:110-183."""
    func = 'dibr_soft_mask_backward_cuda'
    args = [Arg(grad_soft_mask, 'grad_soft_mask', 1), Arg(soft_mask, 'soft_mask', 2),
            Arg(selected_face_idx, 'selected_face_idx', 3), Arg(close_face_prob, 'close_face_prob', 4),
            Arg(close_face_idx, 'close_face_idx', 5), Arg(close_face_dist_type, 'close_face_dist_type', 6),
            Arg(face_vertices_image, 'face_vertices_image', 7)]
    check_all_same_gpu(func, [args[i] for i in (0, 1, 4, 5, 3, 6)])
    check_contiguous(func, [args[i] for i in (0, 1, 3, 4, 5, 6)])
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:]
    K = close_face_idx.shape[-1]
    check_size(func, args[0], (B, H, W))
    check_size(func, args[1], (B, H, W))
    check_size(func, args[2], (B, H, W))
    check_size(func, args[3], (B, H, W, K))
    check_size(func, args[4], (B, H, W, K))
    check_size(func, args[5], (B, H, W, K))
    check_size(func, args[6], (B, F, 3, 2))
    _float_only(func, face_vertices_image)
    N.require_gpu(func, face_vertices_image)
    dev = face_vertices_image.device
    g = torch.empty_like(face_vertices_image)
    nbytes = N.lib().kl_soft_mask_backward_workspace_bytes(B, F)
    ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(N.lib().kl_dibr_soft_mask_backward(
            N.dtype_code(face_vertices_image.dtype), B, H, W, F, K, N.ptr(grad_soft_mask), N.ptr(soft_mask),
            N.ptr(selected_face_idx.contiguous()), N.ptr(close_face_prob), N.ptr(close_face_idx),
            N.ptr(close_face_dist_type), N.ptr(face_vertices_image), float(sigmainv), float(multiplier), N.ptr(g),
            N.ptr(ws), nbytes, N.stream_of(dev)), func)
    return g


# ------------------------------------------------------------------------ render.mesh.deftet
def deftet_sparse_render_forward_cuda(face_vertices_z, face_vertices_image, face_bboxes, pixel_coords,
                                      pixel_depth_ranges, knum, eps):
    """deftet.cpp:49-111: [face_idx (B,P,K) i64 (mesh order, -1 pad), pixel_depths (-inf pad), w0, w1]."""
    func = 'deftet_sparse_render_forward_cuda'
    args = [Arg(face_vertices_z, 'face_vertices_z', 1), Arg(face_vertices_image, 'face_vertices_image', 2),
            Arg(face_bboxes, 'face_bboxes', 3), Arg(pixel_coords, 'pixel_coords', 4),
            Arg(pixel_depth_ranges, 'pixel_depth_ranges', 5)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    B, F = face_vertices_z.shape[:2]
    P = pixel_coords.shape[1]
    check_size(func, args[0], (B, F, 3))
    check_size(func, args[1], (B, F, 3, 2))
    check_size(func, args[2], (B, F, 4))
    check_size(func, args[3], (B, P, 2))
    check_size(func, args[4], (B, P, 2))
    _float_only(func, face_vertices_z)
    N.require_gpu(func, face_vertices_z)
    return deftet_forward(func, face_vertices_z, face_vertices_image, face_bboxes, pixel_coords, pixel_depth_ranges,
                          knum, eps)


def deftet_forward(func, fvz, fvi, bboxes, pix, ranges, knum, eps, binned=False):
    """The forward kernel on checked, contiguous inputs; ``bboxes`` may be None (computed in-kernel
    with the same min / max as deftet.py:290-292).  ``binned`` selects the screen-grid path
    (faster kernel, but one host synchronisation to size the lists); the default tile walk needs
    none and is faster end to end at the bench sizes.  Same outputs."""
    B, F = fvz.shape[:2]
    P = pix.shape[1]
    K = int(knum)
    dev, dtype = fvz.device, fvz.dtype
    idx = torch.empty((B, P, K), dtype=torch.long, device=dev)
    depth = torch.empty((B, P, K), dtype=dtype, device=dev)
    w0 = torch.empty((B, P, K), dtype=dtype, device=dev)
    w1 = torch.empty((B, P, K), dtype=dtype, device=dev)
    lib = N.lib()
    ws_bytes = lib.kl_deftet_workspace_bytes(B, F)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    arena = N.Arena(dev)
    alloc = arena.fn if binned else N.ALLOC_FN()
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_deftet_sparse_render_forward(
            N.dtype_code(dtype), B, F, P, K, N.ptr(fvz), N.ptr(fvi), N.ptr(bboxes), N.ptr(pix), N.ptr(ranges),
            float(eps), N.ptr(idx), N.ptr(depth), N.ptr(w0), N.ptr(w1), N.ptr(ws), ws_bytes, alloc, None,
            N.stream_of(dev)), func)
    return [idx, depth, w0, w1]


def deftet_resolve(face_idx, pixel_depths, w0, w1, face_features):
    """deftet.py:294-306 (DeftetSparseRenderer.forward's torch glue) as one kernel (not a reference
    _C name): (sorted_face_idx (B,P,K), weights (B,P,K,3), interpolated_features (B,P,K,D))."""
    func = 'deftet_sparse_render_resolve'
    B, P, K = face_idx.shape
    F, D = face_features.shape[1], face_features.shape[3]
    dev, dtype = face_features.device, face_features.dtype
    sidx = torch.empty((B, P, K), dtype=torch.long, device=dev)
    weights = torch.empty((B, P, K, 3), dtype=dtype, device=dev)
    interp = torch.empty((B, P, K, D), dtype=dtype, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(N.lib().kl_deftet_sparse_render_resolve(
            N.dtype_code(dtype), B, F, P, K, D, N.ptr(face_idx), N.ptr(pixel_depths), N.ptr(w0), N.ptr(w1),
            N.ptr(face_features), N.ptr(sidx), N.ptr(weights), N.ptr(interp), N.stream_of(dev)), func)
    return sidx, weights, interp


def deftet_sparse_render_backward_cuda(grad_interpolated_features, face_idx, weights, face_vertices_image,
                                       face_features, eps):
    """deftet.cpp:113-163: [grad_face_vertices_image, grad_face_features]."""
    func = 'deftet_sparse_render_backward_cuda'
    args = [Arg(grad_interpolated_features, 'grad_interpolated_features', 1), Arg(face_idx, 'face_idx', 2),
            Arg(weights, 'weights', 3), Arg(face_vertices_image, 'face_vertices_image', 4),
            Arg(face_features, 'face_features', 5)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    B, P, K, D = grad_interpolated_features.shape
    F = face_vertices_image.shape[1]
    check_size(func, args[0], (B, P, K, D))
    check_size(func, args[1], (B, P, K))
    check_size(func, args[2], (B, P, K, 3))
    check_size(func, args[3], (B, F, 3, 2))
    check_size(func, args[4], (B, F, 3, D))
    _float_only(func, grad_interpolated_features)
    N.require_gpu(func, grad_interpolated_features)
    dev = face_vertices_image.device
    g_img = torch.empty_like(face_vertices_image)
    g_feat = torch.empty_like(face_features)
    lib = N.lib()
    ws_bytes = lib.kl_deftet_bwd_workspace_bytes(B, F, P, K)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_deftet_sparse_render_backward(
            N.dtype_code(face_vertices_image.dtype), B, F, P, K, D, N.ptr(grad_interpolated_features),
            N.ptr(face_idx), N.ptr(weights), N.ptr(face_vertices_image), N.ptr(face_features), float(eps),
            N.ptr(g_img), N.ptr(g_feat), N.ptr(ws), ws_bytes, N.stream_of(dev)), func)
    return [g_img, g_feat]


# ------------------------------------------------------------------------------ metrics
def unbatched_triangle_distance_forward_cuda(points, face_vertices, dist, face_idx, dist_type):
    """unbatched_triangle_distance.cpp:43-72 (writes into the caller's tensors)."""
    func = 'unbatched_triangle_distance_forward_cuda'
    args = [Arg(points, 'points', 1), Arg(face_vertices, 'face_vertices', 2), Arg(dist, 'dist', 3),
            Arg(face_idx, 'face_idx', 4), Arg(dist_type, 'dist_type', 5)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    P, F = points.shape[0], face_vertices.shape[0]
    check_size(func, args[0], (P, 3))
    check_size(func, args[1], (F, 3, 3))
    check_size(func, args[2], (P,))
    check_size(func, args[3], (P,))
    check_size(func, args[4], (P,))
    _float_only(func, points)
    N.require_gpu(func, points)
    dev = points.device
    lib = N.lib()
    nbytes = lib.kl_unbatched_triangle_distance_workspace_bytes(P, F)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_unbatched_triangle_distance_forward(
            N.dtype_code(points.dtype), P, F, N.ptr(points), N.ptr(face_vertices), N.ptr(dist), N.ptr(face_idx),
            N.ptr(dist_type), N.ptr(ws), nbytes, N.stream_of(dev)), func)


def unbatched_triangle_distance_backward_cuda(grad_dist, points, face_vertices, face_idx, dist_type, grad_points,
                                              grad_face_vertices):
    """unbatched_triangle_distance.cpp:74-114 (writes into the caller's tensors)."""
    func = 'unbatched_triangle_distance_backward_cuda'
    args = [Arg(grad_dist, 'grad_dist', 1), Arg(points, 'points', 2), Arg(face_vertices, 'face_vertices', 3),
            Arg(face_idx, 'face_idx', 4), Arg(dist_type, 'dist_type', 5), Arg(grad_points, 'grad_points', 6),
            Arg(grad_face_vertices, 'grad_face_vertices', 7)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    P, F = points.shape[0], face_vertices.shape[0]
    check_size(func, args[0], (P,))
    check_size(func, args[1], (P, 3))
    check_size(func, args[2], (F, 3, 3))
    check_size(func, args[3], (P,))
    check_size(func, args[4], (P,))
    check_size(func, args[5], (P, 3))
    check_size(func, args[6], (F, 3, 3))
    _float_only(func, points)
    N.require_gpu(func, points)
    dev = points.device
    # the per-point terms summed per face coordinate in double, rounded once (deterministic)
    nbytes = N.lib().kl_unbatched_triangle_distance_bwd_workspace_bytes(F)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(N.lib().kl_unbatched_triangle_distance_backward(
            N.dtype_code(points.dtype), P, F, N.ptr(grad_dist), N.ptr(points), N.ptr(face_vertices),
            N.ptr(face_idx), N.ptr(dist_type), N.ptr(grad_points), N.ptr(grad_face_vertices), N.ptr(ws), nbytes,
            N.stream_of(dev)), func)


def sided_distance_forward_cuda(p1, p2):
    """sided_distance.cpp:65-89."""
    func = 'sided_distance_forward_cuda'
    a1, a2 = Arg(p1, 'p1', 1), Arg(p2, 'p2', 2)
    check_all_same_gpu(func, [a1, a2])
    check_contiguous(func, [a1, a2])
    check_same_type(func, a1, a2)
    B, N1 = p1.shape[0], p1.shape[1]
    N2 = p2.shape[1]
    check_size(func, a1, (B, N1, 3))
    check_size(func, a2, (B, N2, 3))
    N.require_gpu(func, p1)
    dev = p1.device
    dist = torch.empty((B, N1), dtype=p1.dtype, device=dev)
    idx = torch.empty((B, N1), dtype=torch.long, device=dev)
    with N.on_device(dev), N.timed(func, dev):
        N.check(N.lib().kl_sided_distance_forward(N.dtype_code(p1.dtype), B, N1, N2, N.ptr(p1), N.ptr(p2),
                                                  N.ptr(dist), N.ptr(idx), N.stream_of(dev)), func)
    return [dist, idx]


def sided_distance_backward_cuda(grad_output, p1, p2, idx):
    """sided_distance.cpp:91-122."""
    func = 'sided_distance_backward_cuda'
    ag, a1, a2, ai = Arg(grad_output, 'grad_output', 1), Arg(p1, 'p1', 2), Arg(p2, 'p2', 3), Arg(idx, 'idx', 4)
    check_all_same_gpu(func, [ag, a1, a2, ai])
    check_contiguous(func, [ag, a1, a2, ai])
    B, N1, N2 = p1.shape[0], p1.shape[1], p2.shape[1]
    check_size(func, ai, (B, N1))
    check_size(func, a1, (B, N1, 3))
    check_size(func, a2, (B, N2, 3))
    check_same_size(func, ai, ag)
    N.require_gpu(func, p1)
    dev = p1.device
    g1 = torch.empty_like(p1)
    g2 = torch.empty_like(p2)
    with N.on_device(dev), N.timed(func, dev):
        if p1.dtype in (torch.float32, torch.float64):
            # grad_p2's terms summed in double and rounded once: deterministic, and what a
            # points-sharded caller reproduces bit for bit (kaolin.distributed.sharded_sided_distance)
            sums = N.workspace(B * N2 * 3 * 8, dev)
            N.check(N.lib().kl_sided_distance_backward_sums(N.dtype_code(p1.dtype), B, N1, N2, N.ptr(grad_output),
                                                            N.ptr(p1), N.ptr(p2), N.ptr(idx), N.ptr(g1), N.ptr(sums),
                                                            N.ptr(g2), N.stream_of(dev)), func)
        else:  # half / integer types: the reference's atomics in the type itself
            N.check(N.lib().kl_sided_distance_backward(N.dtype_code(p1.dtype), B, N1, N2, N.ptr(grad_output),
                                                       N.ptr(p1), N.ptr(p2), N.ptr(idx), N.ptr(g1), N.ptr(g2),
                                                       N.stream_of(dev)), func)
    return [g1, g2]


def sided_distance_backward_sums(grad_output, p1, p2, idx):
    """sided_distance_backward_cuda with grad_p2 left as its (B,M,3) float64 double sums (float32 /
    float64 inputs): the per-rank half of kaolin.distributed.sharded_sided_distance's backward."""
    func = 'sided_distance_backward_cuda'
    if p1.dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f'"{func}" (double sums) not implemented for \'{_tname(p1.dtype)}\'')
    N.require_gpu(func, p1, p2, idx, grad_output)
    dev = p1.device
    B, N1, N2 = p1.shape[0], p1.shape[1], p2.shape[1]
    g1 = torch.empty_like(p1)
    sums = torch.empty((B, N2, 3), dtype=torch.float64, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_sided_distance_backward_sums(N.dtype_code(p1.dtype), B, N1, N2,
                                                        N.ptr(grad_output.contiguous()), N.ptr(p1.contiguous()),
                                                        N.ptr(p2.contiguous()), N.ptr(idx.contiguous()), N.ptr(g1),
                                                        N.ptr(sums), None, N.stream_of(dev)), func)
    return g1, sums


# ----------------------------------------------------------------------------- ops.mesh
def unbatched_mesh_intersection_cuda(points, verts_1, verts_2, verts_3):
    """mesh_intersection.cpp:33-68: crossing counts (P,) in the points dtype."""
    func = 'unbatched_mesh_intersection_cuda'
    args = [Arg(points, 'points', 1), Arg(verts_1, 'verts_1', 2), Arg(verts_2, 'verts_2', 3),
            Arg(verts_3, 'verts_3', 4)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    for a in args[1:]:
        check_same_type(func, args[0], a)
    P = points.shape[0]
    F = verts_1.shape[0]
    check_size(func, args[0], (P, 3))
    for a in args[1:]:
        check_size(func, a, (F, 3))
    if points.dtype not in _FLOATS:
        raise RuntimeError(f'unbatched_mesh_intersection_cuda not implemented for \'{_tname(points.dtype)}\'')
    N.require_gpu(func, points)
    dev = points.device
    out = torch.empty((P,), dtype=points.dtype, device=dev)
    lib = N.lib()
    code = N.dtype_code(points.dtype)
    ws_bytes = lib.kl_check_sign_workspace_bytes(code, 1, F, P)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    # under graph capture: the entry without an allocator, which reads nothing back to the host
    alloc = N.ALLOC_FN() if N.capturing(dev) else N.Arena(dev).fn
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_unbatched_mesh_intersection(code, P, F, N.ptr(points), N.ptr(verts_1), N.ptr(verts_2),
                                                   N.ptr(verts_3), N.ptr(out), N.ptr(ws), ws_bytes, alloc, None,
                                                   N.stream_of(dev)), func)
    return out


def check_sign_batched(verts, faces, points, maxlen):
    """check_sign.py:140-154 for the whole batch in one launch (not a reference _C name):
    contains (B,P) bool, faces gathered and 1 / maxlen applied in-kernel (maxlen None: taken
    from the vertices on the device)."""
    func = 'check_sign'
    B, V = verts.shape[:2]
    F, P = faces.shape[0], points.shape[1]
    dev = points.device
    out = torch.empty((B, P), dtype=torch.bool, device=dev)
    lib = N.lib()
    code = N.dtype_code(verts.dtype)
    ws_bytes = lib.kl_check_sign_workspace_bytes(code, B, F, P)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    alloc = N.ALLOC_FN() if N.capturing(dev) else N.Arena(dev).fn  # as unbatched_mesh_intersection_cuda
    with N.on_device(dev), N.timed(func, dev):
        N.check(lib.kl_check_sign(code, B, V, F, P, N.ptr(verts), N.ptr(faces), N.ptr(points), N.ptr(maxlen),
                                  N.ptr(out), N.ptr(ws), ws_bytes, alloc, None, N.stream_of(dev)), func)
    return out


# ------------------------------------------------------------------- ops.conversions / spc
def _mesh_to_spc_checks(face_vertices):
    if not face_vertices.is_cuda:
        raise RuntimeError('face_vertices must be a CUDA tensor')
    if not face_vertices.is_contiguous():
        raise RuntimeError('face_vertices must be contiguous')
    if face_vertices.dim() != 3 or face_vertices.shape[1] != 3 or face_vertices.shape[2] != 3:
        raise RuntimeError('face_vertices must be of shape (F, 3, 3)')
    if face_vertices.dtype != torch.float32:
        raise RuntimeError('face_vertices must be float')


def mesh_to_spc_cuda(face_vertices, target_level):
    """mesh_to_spc.cpp:28-44."""
    func = 'mesh_to_spc_cuda'
    _mesh_to_spc_checks(face_vertices)
    N.require_gpu(func, face_vertices)
    if N.capturing(face_vertices.device):
        raise RuntimeError(f'{func}: the output size is known only after the levels (one host read); '
                           'under graph capture call kaolin.ops.conversions.unbatched_mesh_to_spc(..., capacity=N)')
    dev = face_vertices.device
    arena = N.Arena(dev)
    oct_p, fidx_p, bary_p = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    nn, nl = ctypes.c_int64(), ctypes.c_int64()
    with N.on_device(dev):
        N.check(N.lib().kl_mesh_to_spc(face_vertices.shape[0], N.ptr(face_vertices), int(target_level), arena.fn,
                                       None, ctypes.byref(oct_p), ctypes.byref(nn), ctypes.byref(fidx_p),
                                       ctypes.byref(bary_p), ctypes.byref(nl), N.stream_of(dev)), func)
    if nl.value == 0:
        return [torch.empty((0,), dtype=torch.uint8, device=dev), torch.empty((0,), dtype=torch.long, device=dev),
                torch.zeros((0, 3), dtype=torch.float32, device=dev)]
    octree = arena.tensor(oct_p.value, nn.value, torch.uint8, (nn.value,))
    face_idx = arena.tensor(fidx_p.value, nl.value, torch.long, (nl.value,))
    bary = arena.tensor(bary_p.value, nl.value * 2, torch.float32, (nl.value, 2))
    return [octree, face_idx, bary]


def mesh_to_spc_fixed_cuda(face_vertices, target_level, capacity):
    """mesh_to_spc_cuda with fixed output sizes (not a reference _C name): nothing is read back to
    the host, so it can be captured into a graph (kl_mesh_to_spc_fixed).  capacity: N (octree bytes
    and leaves alike) or (node_capacity, leaf_capacity).  Returns [octree (node_capacity,) u8,
    face_idx (leaf_capacity,) int64, bary (leaf_capacity, 2) f32, result (3,) int64 = (num_nodes,
    num_leaves, status)]: status 0 = written (octree bytes past num_nodes 0, face_idx past
    num_leaves -1, bary 0), 1 = a capacity too small (nothing written; num_nodes / num_leaves are
    the sizes needed), 2 = the per-level pair buffers (96 per face) overflowed (nothing written:
    call the eager form)."""
    func = 'mesh_to_spc_cuda'
    _mesh_to_spc_checks(face_vertices)
    N.require_gpu(func, face_vertices)
    if int(target_level) < 1:
        raise ValueError(f'level must be >= 1 with a capacity, got {target_level}')
    ncap, lcap = (int(capacity), int(capacity)) if not isinstance(capacity, (tuple, list)) else \
        (int(capacity[0]), int(capacity[1]))
    if ncap < 0 or lcap < 0:
        raise ValueError(f'capacity must be >= 0, got {capacity}')
    dev = face_vertices.device
    octree = torch.empty((ncap,), dtype=torch.uint8, device=dev)
    face_idx = torch.empty((lcap,), dtype=torch.long, device=dev)
    bary = torch.empty((lcap, 2), dtype=torch.float32, device=dev)
    result = torch.empty((3,), dtype=torch.int64, device=dev)
    F = face_vertices.shape[0]
    ws_bytes = N.size('kl_mesh_to_spc_fixed_workspace_bytes', F)
    if ws_bytes == 0:
        raise RuntimeError(f'{func}: too many faces for the fixed-capacity form')
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_mesh_to_spc_fixed(F, N.ptr(face_vertices), int(target_level), ncap, lcap, N.ptr(octree),
                                             N.ptr(face_idx), N.ptr(bary), N.ptr(result), N.ptr(ws), ws_bytes,
                                             N.stream_of(dev)), func)
    return [octree, face_idx, bary, result]


def morton_to_octree(mortons, level):
    """spc.cpp:55-65 (mortons: sorted unique int64 leaf codes)."""
    func = 'morton_to_octree'
    N.require_gpu(func, mortons)
    dev = mortons.device
    mortons = mortons.contiguous()
    arena = N.Arena(dev)
    oct_p, nn = ctypes.c_void_p(), ctypes.c_int64()
    with N.on_device(dev):
        N.check(N.lib().kl_morton_to_octree(mortons.shape[0], N.ptr(mortons), int(level), arena.fn, None,
                                            ctypes.byref(oct_p), ctypes.byref(nn), N.stream_of(dev)), func)
    return arena.tensor(oct_p.value, nn.value, torch.uint8, (nn.value,))


def points_to_octree(points, level):
    """spc.cpp:67-77 -> spc_cuda.cu:166-178: int16 points (N,3), unique and in morton order
    (the caller's contract, as in the reference) -> morton codes -> octree."""
    return morton_to_octree(points_to_morton_cuda(points.contiguous()), level)


def points_to_morton_cuda(points):
    """point_utils.cpp:52-64."""
    func = 'points_to_morton_cuda'
    a = Arg(points, 'points', 1)
    check_all_same_gpu(func, [a])
    check_contiguous(func, [a])
    _check_scalar_types(func, a, (torch.int16,))
    if points.dim() != 2 or points.shape[1] != 3:
        raise RuntimeError('points must be Nx3')
    n = points.shape[0]
    dev = points.device
    morton = torch.empty((n,), dtype=torch.long, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_points_to_morton(n, N.ptr(points), N.ptr(morton), N.stream_of(dev)), func)
    return morton


def morton_to_points_cuda(morton_codes):
    """point_utils.cpp:36-50."""
    func = 'morton_to_points_cuda'
    a = Arg(morton_codes, 'morton_codes', 1)
    check_all_same_gpu(func, [a])
    check_contiguous(func, [a])
    _check_scalar_types(func, a, (torch.int64,))
    n = morton_codes.shape[0]
    dev = morton_codes.device
    points = torch.empty((n, 3), dtype=torch.int16, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_morton_to_points(n, N.ptr(morton_codes), N.ptr(points), N.stream_of(dev)), func)
    return points


def _check_octrees(octrees, name='octrees'):
    if octrees.dtype != torch.uint8:
        raise RuntimeError(f'{name} must be byte')
    if not octrees.is_cuda:
        raise RuntimeError(f'{name} must be a CUDA tensor')
    if not octrees.is_contiguous():
        raise RuntimeError(f'{name} must be contiguous')


def scan_octrees_cuda(octrees, lengths):
    """spc.cpp:79-107 -> (level, pyramid (B,2,level+2) CPU int32, exsum int32)."""
    func = 'scan_octrees_cuda'
    _check_octrees(octrees)
    if lengths.is_cuda:
        raise RuntimeError('lengths must be a cpu tensor')
    if not lengths.is_contiguous():
        raise RuntimeError('lengths must be contiguous')
    N.require_gpu(func, octrees)
    dev = octrees.device
    lengths32 = lengths.to(torch.int32).contiguous()
    B = lengths32.shape[0]
    total = int(lengths32.sum())
    exsum = torch.zeros(total + B, dtype=torch.int32, device=dev)
    pyr = torch.zeros((B, 2, 17), dtype=torch.int32)
    level = ctypes.c_int()
    with N.on_device(dev):
        N.check(N.lib().kl_scan_octrees(B, N.ptr(octrees), ctypes.c_void_p(lengths32.data_ptr()), N.ptr(exsum),
                                        ctypes.c_void_p(pyr.data_ptr()), ctypes.byref(level), N.stream_of(dev)),
                func)
    lv = level.value
    return lv, pyr[:, :, :lv + 2].contiguous(), exsum


def generate_points_cuda(octrees, pyramids, exsum):
    """spc.cpp:109-134."""
    func = 'generate_points_cuda'
    _check_octrees(octrees)
    if pyramids.is_cuda:
        raise RuntimeError('pyramids must be a cpu tensor')
    if not pyramids.is_contiguous():
        raise RuntimeError('pyramids must be contiguous')
    if not exsum.is_cuda:
        raise RuntimeError('exsum must be a CUDA tensor')
    if not exsum.is_contiguous():
        raise RuntimeError('exsum must be contiguous')
    N.require_gpu(func, octrees)
    dev = octrees.device
    pyr = pyramids.to(torch.int32).contiguous()
    level = pyr.shape[2] - 2
    psum = int(pyr[:, 1, level + 1].sum())
    points = torch.empty((psum, 3), dtype=torch.int16, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_generate_points(pyr.shape[0], level, N.ptr(octrees), ctypes.c_void_p(pyr.data_ptr()),
                                           N.ptr(exsum), N.ptr(points), N.stream_of(dev)), func)
    return points


# ------------------------------------------------------------------------------ render.spc
def _raytrace_checks(func, octree, points, pyramid, exclusive_sum, ray_o, ray_d):
    """raytrace.cpp:170-200's argument checks; returns the pyramid's max level."""
    args = [Arg(octree, 'octree', 1), Arg(points, 'points', 2), Arg(exclusive_sum, 'exclusive_sum', 4),
            Arg(ray_o, 'ray_o', 5), Arg(ray_d, 'ray_d', 6)]
    check_all_same_gpu(func, args)
    check_contiguous(func, args)
    if pyramid.is_cuda:
        raise RuntimeError(f'Expected tensor to have cpu DeviceType, but got tensor with {pyramid.device.type} '
                           f'DeviceType (while checking arguments for {func})')
    if points.dtype != torch.int16:
        raise RuntimeError('points must be short')
    check_dim(func, Arg(points, 'points', 2), 2)
    check_size_dim(func, Arg(points, 'points', 2), 1, 3)
    check_dim(func, Arg(pyramid, 'pyramid', 3), 2)
    check_size_dim(func, Arg(pyramid, 'pyramid', 3), 0, 2)
    max_level = pyramid.shape[1] - 2
    if not max_level < 15:
        raise RuntimeError('SPC pyramid too big')
    pyr = pyramid.reshape(-1).tolist()  # (one conversion: four tensor indexings cost ~15 us of host time)
    osize = int(pyr[2 * max_level + 2])
    psize = int(pyr[2 * max_level + 3])
    check_size_dim(func, Arg(octree, 'octree', 1), 0, osize)
    check_size_dim(func, Arg(points, 'points', 2), 0, psize)
    if not (int(pyr[max_level + 1]) == 0 and int(pyr[max_level + 2]) == 0):
        raise RuntimeError('SPC pyramid corrupt, check if the SPC pyramid has been sliced')
    N.require_gpu(func, octree)
    return max_level


def raytrace_cuda(octree, points, pyramid, exclusive_sum, ray_o, ray_d, target_level, return_depth, with_exit):
    """raytrace.cpp:170-214."""
    func = 'raytrace_cuda'
    max_level = _raytrace_checks(func, octree, points, pyramid, exclusive_sum, ray_o, ray_d)
    if N.capturing(octree.device):
        raise RuntimeError(f'{func}: the output size is known only after the march (one host read per level); '
                           'under graph capture call kaolin.render.spc.unbatched_raytrace(..., capacity=N)')
    dev = octree.device
    arena = N.Arena(dev)
    nug_p, dep_p, nh = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
    with N.on_device(dev):
        N.check(N.lib().kl_raytrace(N.ptr(octree), octree.shape[0], N.ptr(points), points.shape[0],
                                    N.ptr(exclusive_sum), max_level, N.ptr(ray_o), N.ptr(ray_d), ray_o.shape[0],
                                    int(target_level), int(bool(return_depth)), int(bool(with_exit)), arena.fn, None,
                                    ctypes.byref(nug_p), ctypes.byref(dep_p), ctypes.byref(nh), N.stream_of(dev)),
                func)
    n = nh.value
    nuggets = arena.tensor(nug_p.value, 2 * n, torch.int32, (n, 2))
    if return_depth:
        dd = 2 if with_exit else 1
        depth = arena.tensor(dep_p.value, n * dd, torch.float32, (n, dd))
        return [nuggets, depth]
    return [nuggets]


def raytrace_fixed_cuda(octree, points, pyramid, exclusive_sum, ray_o, ray_d, target_level, return_depth, with_exit,
                        capacity):
    """raytrace_cuda with a fixed output size (not a reference _C name): nothing is read back to
    the host, so it can be captured into a graph (kl_raytrace_fixed).  Returns [nuggets
    (capacity, 2) int32, depth (capacity, 1|2) f32 if return_depth, result (2,) int64 = (rows
    written, 1 if truncated)]; rows past result[0] hold (-1, -1) and depth 0."""
    func = 'raytrace_cuda'
    _raytrace_checks(func, octree, points, pyramid, exclusive_sum, ray_o, ray_d)
    capacity = int(capacity)
    if capacity < 0:
        raise ValueError(f'capacity must be >= 0, got {capacity}')
    dev = octree.device
    dd = 2 if with_exit else 1
    nuggets = torch.empty((capacity, 2), dtype=torch.int32, device=dev)
    depth = torch.empty((capacity, dd), dtype=torch.float32, device=dev) if return_depth else None
    result = torch.empty((2,), dtype=torch.int64, device=dev)
    lib = N.lib()
    nr = ray_o.shape[0]
    ws_bytes = N.size('kl_raytrace_fixed_workspace_bytes', nr, capacity, int(bool(with_exit)))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with N.on_device(dev):
        N.check(lib.kl_raytrace_fixed(N.ptr(octree), N.ptr(points), N.ptr(exclusive_sum), N.ptr(ray_o), N.ptr(ray_d),
                                      nr, int(target_level), int(bool(return_depth)), int(bool(with_exit)), capacity,
                                      N.ptr(nuggets), N.ptr(depth), N.ptr(result), N.ptr(ws), ws_bytes,
                                      N.stream_of(dev)), func)
    return [nuggets, depth, result] if return_depth else [nuggets, result]


def _host_f32(x, n):
    """A host float array of a CPU tensor's values (the reference reads them through data_ptr)."""
    a = (ctypes.c_float * n)(*x.reshape(-1)[:n].tolist())
    return ctypes.cast(a, ctypes.c_void_p), a


def generate_primary_rays_cuda(height, width, Eye, At, Up, fov, World):
    """raytrace.cpp:111-166 (deprecated upstream, bindings.cpp:86): pinhole rays (origin,
    direction) of a height x width image, (height*width, 3) float32 each on the current device."""
    for name, t in (('Eye', Eye), ('At', At), ('Up', Up)):
        if not t.is_contiguous():
            raise RuntimeError(f'{name} must be contiguous')
        if t.device.type != 'cpu':
            raise RuntimeError(f'{name} must be a cpu tensor')
        if t.dtype != torch.float32:
            raise RuntimeError(f'{name} must be byte')  # the reference's CHECK_FLOAT message
        if not (t.dim() == 1 and t.shape[0] == 3):
            raise RuntimeError(f'{name} must be a triplet')
    if not World.is_contiguous():
        raise RuntimeError('World must be contiguous')
    if World.device.type != 'cpu':
        raise RuntimeError('World must be a cpu tensor')
    if tuple(World.shape) != (4, 4):
        raise RuntimeError('World must of size {4, 4}')
    height, width = int(height), int(width)
    num = height * width
    N.require_gpu('generate_primary_rays_cuda')
    dev = torch.device('cuda', torch.cuda.current_device())
    org = torch.empty((num, 3), dtype=torch.float32, device=dev)
    dirs = torch.empty((num, 3), dtype=torch.float32, device=dev)
    keep = [_host_f32(t.float(), k) for t, k in ((Eye, 3), (At, 3), (Up, 3), (World, 16))]
    with N.on_device(dev):
        N.check(N.lib().kl_generate_primary_rays(height, width, keep[0][0], keep[1][0], keep[2][0], float(fov),
                                                 keep[3][0], N.ptr(org), N.ptr(dirs), N.stream_of(dev)),
                'generate_primary_rays_cuda')
    return [org, dirs]


def generate_shadow_rays_cuda(ray_o, ray_d, light, plane):
    """raytrace.cpp:234-283 (deprecated upstream, bindings.cpp:88): for the rays that meet
    `plane` ahead, rays from `light` to the hit point: [src, dst (normalised), map (ray
    index)], the reference's count of rows (its exclusive scan's last entry)."""
    func = 'generate_shadow_rays_cuda'
    for t in (ray_o, ray_d):
        if t.dtype != torch.float32:
            raise RuntimeError(f'expected scalar type Float but found {_tname(t.dtype)}')
    for name, t, k in (('light', light, 3), ('plane', plane, 4)):
        if t.device.type != 'cpu':
            raise RuntimeError(f'{func}: {name} must be a cpu tensor')
        if t.dtype != torch.float32:
            raise RuntimeError(f'expected scalar type Float but found {_tname(t.dtype)}')
        if t.numel() < k:
            raise RuntimeError(f'{func}: {name} must hold {k} values')
    N.require_gpu(func, ray_o, ray_d)
    dev = ray_o.device
    ray_o, ray_d = ray_o.contiguous(), ray_d.contiguous()
    num = ray_d.shape[0]
    src = torch.empty((num, 3), dtype=torch.float32, device=dev)
    dst = torch.empty((num, 3), dtype=torch.float32, device=dev)
    mp = torch.empty((num,), dtype=torch.int32, device=dev)
    lib = N.lib()
    ws_bytes = lib.kl_generate_shadow_rays_workspace_bytes(num)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    lt, pl = _host_f32(light.contiguous(), 3), _host_f32(plane.contiguous(), 4)
    cnt = ctypes.c_int64()
    with N.on_device(dev):
        N.check(lib.kl_generate_shadow_rays(num, N.ptr(ray_o), N.ptr(ray_d), lt[0], pl[0], N.ptr(src), N.ptr(dst),
                                            N.ptr(mp), ctypes.byref(cnt), N.ptr(ws), ws_bytes, N.stream_of(dev)),
                func)
    c = cnt.value
    return [src[:c], dst[:c], mp[:c]]


def mark_pack_boundaries_cuda(pack_ids):
    """raytrace.cpp:216-232."""
    func = 'mark_pack_boundaries_cuda'
    a = Arg(pack_ids, 'pack_ids', 1)
    check_dim(func, a, 1)
    check_all_same_gpu(func, [a])
    check_contiguous(func, [a])
    if pack_ids.dtype not in (torch.uint8, torch.int8, torch.int32, torch.int64, torch.int16):
        raise RuntimeError(f'Expected scalar type of argument #1 \'pack_ids\' to be one of Byte, Char, Int, Long, '
                           f'Short (while checking arguments for {func})')
    dev = pack_ids.device
    out = torch.empty((pack_ids.shape[0],), dtype=torch.int32, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_mark_pack_boundaries(N.dtype_code(pack_ids.dtype), pack_ids.shape[0], N.ptr(pack_ids),
                                                N.ptr(out), N.stream_of(dev)), func)
    return out


_HALF_FLOATS = (torch.float16, torch.float32, torch.float64)


def _check_scalar_types(func, a, allowed):
    """at::checkScalarTypes / at::checkScalarType message."""
    if a.t.dtype not in allowed:
        names = ', '.join(_tname(d) for d in allowed)
        what = f'one of {names}' if len(allowed) > 1 else names
        raise RuntimeError(f"Expected scalar type of argument #{a.pos} '{a.name}' to be {what}; but got "
                           f"{_tname(a.t.dtype)} (while checking arguments for {func})")


def _pack_args(func, feats, idx, idx_name, idx_dtype):
    a, b = Arg(feats, 'feats', 1), Arg(idx, idx_name, 2)
    check_dim(func, a, 2)
    check_dim(func, b, 1)
    check_all_same_gpu(func, [a, b])
    check_contiguous(func, [a, b])
    _check_scalar_types(func, a, _HALF_FLOATS)
    _check_scalar_types(func, b, (idx_dtype,))


def diff_cuda(feats, pack_indices):
    """raytrace.cpp:285-309."""
    func = 'diff_cuda'
    _pack_args(func, feats, pack_indices, 'pack_indices', torch.int64)
    out = torch.empty_like(feats)
    dev = feats.device
    with N.on_device(dev):
        N.check(N.lib().kl_pack_diff(N.dtype_code(feats.dtype), feats.shape[0], feats.shape[1], N.ptr(feats),
                                     N.ptr(pack_indices), pack_indices.shape[0], N.ptr(out), N.stream_of(dev)), func)
    return out


def inclusive_sum_cuda(info):
    """raytrace.cpp:311-325."""
    func = 'inclusive_sum_cuda'
    a = Arg(info, 'info', 1)
    check_dim(func, a, 1)
    check_all_same_gpu(func, [a])
    check_contiguous(func, [a])
    _check_scalar_types(func, a, (torch.int32,))
    n = info.shape[0]
    dev = info.device
    out = torch.empty((n,), dtype=torch.int32, device=dev)
    with N.on_device(dev):
        ws = torch.empty((N.lib().kl_inclusive_sum_workspace_bytes(n),), dtype=torch.uint8, device=dev)
        N.check(N.lib().kl_inclusive_sum_i32(n, N.ptr(info), N.ptr(out), N.ptr(ws), ws.numel(), N.stream_of(dev)),
                func)
    return out


def sum_reduce_cuda(feats, inclusive_sum):
    """raytrace.cpp:328-351: (cnt, feat_dim) with cnt = inclusive_sum[-1] (a device->host read,
    as the reference's cudaMemcpyAsync at raytrace_cuda.cu:677)."""
    func = 'sum_reduce_cuda'
    _pack_args(func, feats, inclusive_sum, 'inclusive_sum', torch.int32)
    nf, dim = feats.shape
    dev = feats.device
    cnt = int(inclusive_sum[-1]) if nf > 0 else 0
    cnt = max(0, min(cnt, nf))  # the reference allocated num_feats rows and sliced [:cnt]
    out = torch.empty((cnt, dim), dtype=feats.dtype, device=dev)
    with N.on_device(dev):
        N.check(N.lib().kl_sum_reduce(N.dtype_code(feats.dtype), nf, dim, N.ptr(feats), N.ptr(inclusive_sum), cnt,
                                      N.ptr(out), N.stream_of(dev)), func)
    return out


def _pack_scan(func, entry, feats, pack_indices, exclusive, reverse):
    _pack_args(func, feats, pack_indices, 'pack_indices', torch.int32)
    out = torch.empty_like(feats)
    dev = feats.device
    with N.on_device(dev):
        N.check(getattr(N.lib(), entry)(N.dtype_code(feats.dtype), feats.shape[0], feats.shape[1], N.ptr(feats),
                                        N.ptr(pack_indices), pack_indices.shape[0], int(bool(exclusive)),
                                        int(bool(reverse)), N.ptr(out), N.stream_of(dev)), func)
    return out


def cumsum_cuda(feats, pack_indices, exclusive, reverse):
    """raytrace.cpp:354-377."""
    return _pack_scan('cumsum_cuda', 'kl_pack_cumsum', feats, pack_indices, exclusive, reverse)


def cumprod_cuda(feats, pack_indices, exclusive, reverse):
    """raytrace.cpp:380-402."""
    return _pack_scan('cumprod_cuda', 'kl_pack_cumprod', feats, pack_indices, exclusive, reverse)


# ----------------------------------------------------------------------- module layout
def _module(name, **fns):
    m = types.ModuleType(name)
    for k, v in fns.items():
        setattr(m, k, v)
    return m


render = _module('kaolin._C.render')
render.mesh = _module('kaolin._C.render.mesh', packed_rasterize_forward_cuda=packed_rasterize_forward_cuda,
                      rasterize_backward_cuda=rasterize_backward_cuda,
                      dibr_soft_mask_forward_cuda=dibr_soft_mask_forward_cuda,
                      dibr_soft_mask_backward_cuda=dibr_soft_mask_backward_cuda,
                      deftet_sparse_render_forward_cuda=deftet_sparse_render_forward_cuda,
                      deftet_sparse_render_backward_cuda=deftet_sparse_render_backward_cuda)
render.spc = _module('kaolin._C.render.spc', raytrace_cuda=raytrace_cuda, raytrace_fixed_cuda=raytrace_fixed_cuda,
                     generate_primary_rays_cuda=generate_primary_rays_cuda,
                     generate_shadow_rays_cuda=generate_shadow_rays_cuda,
                     mark_pack_boundaries_cuda=mark_pack_boundaries_cuda, diff_cuda=diff_cuda,
                     inclusive_sum_cuda=inclusive_sum_cuda, sum_reduce_cuda=sum_reduce_cuda,
                     cumsum_cuda=cumsum_cuda, cumprod_cuda=cumprod_cuda)
metrics = _module('kaolin._C.metrics', sided_distance_forward_cuda=sided_distance_forward_cuda,
                  sided_distance_backward_cuda=sided_distance_backward_cuda,
                  unbatched_triangle_distance_forward_cuda=unbatched_triangle_distance_forward_cuda,
                  unbatched_triangle_distance_backward_cuda=unbatched_triangle_distance_backward_cuda)
ops = _module('kaolin._C.ops')
ops.mesh = _module('kaolin._C.ops.mesh', unbatched_mesh_intersection_cuda=unbatched_mesh_intersection_cuda)
ops.conversions = _module('kaolin._C.ops.conversions', mesh_to_spc_cuda=mesh_to_spc_cuda,
                          mesh_to_spc_fixed_cuda=mesh_to_spc_fixed_cuda)
ops.spc = _module('kaolin._C.ops.spc', morton_to_octree=morton_to_octree, points_to_octree=points_to_octree,
                  points_to_morton_cuda=points_to_morton_cuda, morton_to_points_cuda=morton_to_points_cuda,
                  scan_octrees_cuda=scan_octrees_cuda, generate_points_cuda=generate_points_cuda)
