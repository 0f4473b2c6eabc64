"""HIP path (through kaolin._C and the front-ends) vs the CPU oracle and the reference goldens.

All tests need an MI355X.  Integer outputs (face indices, distance types, octrees,
nuggets, voxels) must be bit-identical to the oracle; floating outputs of the forward
kernels are bit-identical too where no transcendental is involved (same operation
order, no contraction, IEEE div/sqrt); soft-mask probabilities differ only by expf
ulps (tolerance 1e-6 relative).  f32 gradients are the reference's float terms summed in
double and rounded once, so they are bit-equal to the oracle's ordered double sum
(dibr_util.assert_grads_equal: at most 1 element in 10^4 one ulp off, where a face's terms span
more than ~2^29); f64 gradients that go through double atomics agree to ~1e-15 relative.
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from dibr_util import assert_grads_equal

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module')
def kal():
    import kaolin
    return kaolin


def T(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t.to(dtype) if dtype is not None else t


def A(t):
    return t.detach().cpu().numpy()


def _uv_sphere(n_lat, n_lon, radius=1.0):
    lat = np.linspace(0, math.pi, n_lat + 1)[1:-1]
    lon = np.arange(n_lon) * (2 * math.pi / n_lon)
    ring = np.stack([np.sin(lat)[:, None] * np.cos(lon)[None], np.repeat(np.cos(lat)[:, None], n_lon, 1),
                     np.sin(lat)[:, None] * np.sin(lon)[None]], -1).reshape(-1, 3)
    verts = np.concatenate([[[0., 1., 0.]], ring, [[0., -1., 0.]]]) * radius
    faces = []
    nr = n_lat - 1
    for j in range(n_lon):
        faces.append([0, 1 + (j + 1) % n_lon, 1 + j])
    for i in range(nr - 1):
        for j in range(n_lon):
            a, b = 1 + i * n_lon + j, 1 + i * n_lon + (j + 1) % n_lon
            c, d = 1 + (i + 1) * n_lon + j, 1 + (i + 1) * n_lon + (j + 1) % n_lon
            faces += [[a, b, d], [a, d, c]]
    last = 1 + nr * n_lon
    for j in range(n_lon):
        faces.append([1 + (nr - 1) * n_lon + j, 1 + (nr - 1) * n_lon + (j + 1) % n_lon, last])
    return verts, np.array(faces, np.int64)


def _render_inputs(kal, n_lat, n_lon, B, dtype=torch.float32, seed=0):
    v, f = _uv_sphere(n_lat, n_lon, 0.9)
    g = np.random.default_rng(seed)
    v = v * (1 + 0.01 * g.standard_normal((v.shape[0], 1)))
    verts = T(v, dtype).unsqueeze(0).repeat(B, 1, 1)
    faces = T(f)
    az = torch.arange(B, dtype=dtype, device=DEV) * (2 * math.pi / B)
    cam = torch.stack([3 * torch.sin(az), torch.zeros_like(az) + 0.3, 3 * torch.cos(az)], -1)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(
        cam, torch.zeros_like(cam), torch.tensor([[0., 1., 0.]], dtype=dtype, device=DEV).repeat(B, 1))
    vc = kal.render.camera.rotate_translate_points(verts, rot, trans)
    proj = kal.render.camera.generate_perspective_projection(math.pi / 4, dtype=dtype).to(DEV)
    vi = kal.render.camera.perspective_camera(vc, proj)
    fvc = kal.ops.mesh.index_vertices_by_faces(vc, faces)
    fvz = fvc[..., -1].contiguous()
    fvi = kal.ops.mesh.index_vertices_by_faces(vi, faces).contiguous()
    fnz = kal.ops.mesh.face_normals(fvc, unit=True)[..., -1]
    uv = torch.stack([torch.atan2(verts[..., 2], verts[..., 0]), verts[..., 1]], -1)
    feat = kal.ops.mesh.index_vertices_by_faces(torch.cat([uv, torch.ones_like(uv[..., :1])], -1), faces)
    return fvz, fvi, feat.contiguous(), fnz


# ------------------------------------------------------------------ rasterize
@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('valid', [0, 1])
def test_rasterize_sphere_fixture(kal, golden, dname, flip, valid):
    g = golden('dibr_sphere.npz')
    p = f'{dname}_flip{flip}_'
    q = p + f'valid{valid}_'
    fvz, fvi, uv = T(g[p + 'face_vertices_z']), T(g[p + 'face_vertices_image']), T(g[p + 'face_uvs'])
    vf = T(g[p + 'valid_faces']) if valid else None
    fvi_r = fvi.clone().requires_grad_(True)
    uv_r = uv.clone().requires_grad_(True)
    feats, fidx = kal.render.mesh.rasterize(35, 31, fvz, fvi_r, uv_r, valid_faces=vf)
    # reference golden (naive oracle of the reference) with the reference test tolerances
    assert np.array_equal(A(fidx), g[q + 'face_idx'])
    np.testing.assert_allclose(A(feats), g[q + 'features'], rtol=1e-5, atol=1e-5)
    feats.backward(T(g[q + 'grad_out']))
    np.testing.assert_allclose(A(fvi_r.grad), g[q + 'grad_face_vertices_image'], rtol=1e-3, atol=1e-2)
    np.testing.assert_allclose(A(uv_r.grad), g[q + 'grad_face_uvs'], rtol=1e-3, atol=1e-3)
    # our oracle: bit-exact forward, 1e-5 backward
    of, oi, ow = orc.rasterize(35, 31, g[p + 'face_vertices_z'], g[p + 'face_vertices_image'], g[p + 'face_uvs'],
                               valid_faces=g[p + 'valid_faces'] if valid else None)
    assert np.array_equal(A(fidx), oi)
    assert np.array_equal(A(feats), of)
    gi, gf = orc.rasterize_backward(g[q + 'grad_out'], oi, ow, g[p + 'face_vertices_image'], g[p + 'face_uvs'], 1e-8)
    assert_grads_equal(A(fvi_r.grad), gi)
    assert_grads_equal(A(uv_r.grad), gf)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('valid', [0, 1])
@pytest.mark.parametrize('backend', ['cuda', 'cuda_packed'])
def test_rasterize_list_sphere_fixture(kal, golden, dname, flip, valid, backend):
    """test_rasterization.py:158-200,240-290 (test_cuda_{forward,backward}_with_list): features
    as the list [face_uvs, face_mask]; the outputs are a tuple of per-element views and each
    element gets its own gradient.  Golden features at the reference tolerance, the oracle
    bit-exact on the concatenated features."""
    g = golden('dibr_sphere.npz')
    p = f'{dname}_flip{flip}_'
    q = p + f'valid{valid}_'
    fvz, fvi, uv = T(g[p + 'face_vertices_z']), T(g[p + 'face_vertices_image']), T(g[p + 'face_uvs'])
    vf = T(g[p + 'valid_faces']) if valid else None
    fvi_r = fvi.clone().requires_grad_(True)
    uv_r = uv.clone().requires_grad_(True)
    mask_r = torch.ones_like(uv[..., :1]).requires_grad_(True)
    (uvs_map, mask_map), fidx = kal.render.mesh.rasterize(35, 31, fvz, fvi_r, [uv_r, mask_r], valid_faces=vf,
                                                          backend=backend)
    assert uvs_map.shape == uv.shape[:1] + (35, 31, 2) and mask_map.shape == uv.shape[:1] + (35, 31, 1)
    assert np.array_equal(A(fidx), g[q + 'face_idx'])
    np.testing.assert_allclose(A(uvs_map), g[q + 'features'], rtol=1e-5, atol=1e-5)
    cat = np.concatenate([g[p + 'face_uvs'], np.ones_like(g[p + 'face_uvs'][..., :1])], -1)
    of, oi, ow = orc.rasterize(35, 31, g[p + 'face_vertices_z'], g[p + 'face_vertices_image'], cat,
                               valid_faces=g[p + 'valid_faces'] if valid else None)
    assert np.array_equal(A(fidx), oi)
    assert np.array_equal(A(uvs_map), of[..., :2]) and np.array_equal(A(mask_map), of[..., 2:])
    go = np.concatenate([g[q + 'grad_out'], np.random.default_rng(2).uniform(size=of[..., 2:].shape)], -1)
    go = go.astype(of.dtype)
    torch.autograd.backward([uvs_map, mask_map], [T(go[..., :2]), T(go[..., 2:])])
    gi, gf = orc.rasterize_backward(go, oi, ow, g[p + 'face_vertices_image'], cat, 1e-8)
    assert_grads_equal(A(fvi_r.grad), gi)
    assert_grads_equal(A(uv_r.grad), gf[..., :2])
    assert_grads_equal(A(mask_r.grad), gf[..., 2:])


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_dibr_rasterization_list_vs_oracle(kal, dtype):
    """dibr_rasterization with the tutorial's feature list [face_uvs, ones] (dibr_tutorial.ipynb
    cell 12) runs the single fused node: outputs and per-element gradients equal the tensor
    call's bit for bit, and the oracle's (rasterize + soft-mask backward on the same values)."""
    fvz, fvi, feat, fnz = _render_inputs(kal, 30, 50, 3, dtype)
    H, W = 72, 100
    uv, ones = feat[..., :2].contiguous(), torch.ones_like(feat[..., 2:])
    a = fvi.clone().requires_grad_(True)
    u = uv.clone().requires_grad_(True)
    o = ones.clone().requires_grad_(True)
    (fu, fo), mask, idx = kal.render.mesh.dibr_rasterization(H, W, fvz, a, [u, o], fnz)
    assert fu.shape == (3, H, W, 2) and fo.shape == (3, H, W, 1)
    gu, go, gm = torch.rand_like(fu), torch.rand_like(fo), torch.rand_like(mask)
    torch.autograd.backward([fu, fo, mask], [gu, go, gm])
    # the tensor call on the concatenated features
    a2 = fvi.clone().requires_grad_(True)
    f2 = torch.cat([uv, ones], -1).requires_grad_(True)
    ft, mask2, idx2 = kal.render.mesh.dibr_rasterization(H, W, fvz, a2, f2, fnz)
    torch.autograd.backward([ft, mask2], [torch.cat([gu, go], -1), gm])
    assert torch.equal(idx, idx2) and torch.equal(mask, mask2)
    assert torch.equal(fu, ft[..., :2]) and torch.equal(fo, ft[..., 2:])
    # f32: the terms sum exactly in double, bit-equal run to run; f64: the soft-mask hash adds
    # double terms in LDS-atomic order, equal to ~1e-15 relative
    assert_grads_equal(A(a.grad), A(a2.grad))
    assert_grads_equal(A(u.grad), A(f2.grad[..., :2].contiguous()))
    assert_grads_equal(A(o.grad), A(f2.grad[..., 2:].contiguous()))
    # the oracle
    cat = A(torch.cat([uv, ones], -1))
    of, oi, ow = orc.rasterize(H, W, A(fvz), A(fvi), cat, valid_faces=A(fnz >= 0))
    assert np.array_equal(A(idx), oi) and np.array_equal(A(fu), of[..., :2]) and np.array_equal(A(fo), of[..., 2:])
    fm = A(fvi) * A(fvi).dtype.type(1000.)
    pad = fm.dtype.type(0.02 * 1000.)
    bb = np.concatenate([fm.min(-2) - pad, fm.max(-2) + pad], -1)
    om, op, oci, oct_ = orc.dibr_soft_mask_forward(fm, bb, oi, 7000., 30, 1000.)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    from kaolin import _fused
    _, state = _fused.soft_mask_forward_compact(fvi, idx, 7000., 0.02, 30, 1000.)
    _, _, gp = _decode_compact(state, H, W, 30)
    gi_r, gfe = orc.rasterize_backward(A(torch.cat([gu, go], -1)), oi, ow, A(fvi), cat, 1e-8)
    gi = gi_r + orc.dibr_soft_mask_backward(A(gm), A(mask), oi, gp, oci, oct_, fm, 7000., 1000.)
    assert_grads_equal(A(a.grad), gi)
    assert_grads_equal(A(u.grad), gfe[..., :2])
    assert_grads_equal(A(o.grad), gfe[..., 2:])


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('H,W', [(96, 128), (67, 45)])
def test_packed_rasterize_vs_oracle(kal, dtype, H, W):
    fvz, fvi, feat, fnz = _render_inputs(kal, 30, 50, 3, dtype)
    valid = fnz >= 0
    feats, fidx = kal.render.mesh.rasterize(H, W, fvz, fvi, feat, valid_faces=valid)
    of, oi, ow = orc.rasterize(H, W, A(fvz), A(fvi), A(feat), valid_faces=A(valid))
    assert np.array_equal(A(fidx), oi)
    assert np.array_equal(A(feats), of)
    assert (oi >= 0).mean() > 0.2


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('use_valid', [False, True])
def test_fused_path_matches_packed_C_chain(kal, dtype, use_valid):
    """The fused front-end path (in-kernel packing / bbox / remap, gather backward) equals
    the reference's torch-glue + packed _C chain: forward and gradients bit-exact."""
    fvz, fvi, feat, fnz = _render_inputs(kal, 30, 50, 3, dtype)
    valid = (fnz >= 0) if use_valid else None
    outs = []
    for backend in ('cuda', 'cuda_packed'):
        a = fvi.clone().requires_grad_(True)
        b = feat.clone().requires_grad_(True)
        f, i = kal.render.mesh.rasterize(70, 90, fvz, a, b, valid_faces=valid, backend=backend)
        g = torch.Generator(device='cpu').manual_seed(3)
        f.backward(torch.rand(f.shape, generator=g, dtype=dtype).to(DEV))
        outs.append((f, i, a.grad, b.grad))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert_grads_equal(A(outs[0][2]), A(outs[1][2]))
    assert_grads_equal(A(outs[0][3]), A(outs[1][3]))
    # soft mask: fused (unscaled input, in-kernel bbox) vs the _C contract
    m, box = 1000., 0.02
    fm = (fvi * m).contiguous()
    bb = torch.cat([fm.min(-2)[0] - box * m, fm.max(-2)[0] + box * m], -1).contiguous()
    r1 = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, outs[0][1], 7000., 30, m)
    from kaolin import _fused
    r2 = _fused.soft_mask_forward(fvi, outs[0][1], 7000., box, 30, m)
    for x, y in zip(r1, r2):
        assert torch.equal(x, y)


def _adversarial_faces(dtype, seed=5):
    """Small random faces on a coarse depth grid (exact depth ties between overlapping
    faces), exact duplicates (same depth -> lowest index must win), -0.0/+0.0 depth ties,
    faces far larger than 64 pixels, a NaN depth, an infinite and a NaN coordinate, a
    zero-area face and faces straddling the screen border."""
    g = np.random.default_rng(seed)
    n = 400
    c = g.uniform(-1.1, 1.1, (n, 1, 2))
    fvi = c + g.uniform(-0.12, 0.12, (n, 3, 2))
    fvz = -np.round(g.uniform(1, 3, (n, 1)) * 2) / 2 + np.zeros((n, 3))
    fvi = np.concatenate([fvi, fvi[:60]])                      # duplicates
    fvz = np.concatenate([fvz, fvz[:60]])
    big = np.array([[[-0.9, -0.9], [0.9, -0.8], [0.0, 0.95]], [[-1.5, 1.5], [1.5, 1.5], [0.0, -1.5]]])
    fvi = np.concatenate([fvi, big, big[:1], big[:1]])         # big faces, then a +0/-0 depth pair
    fvz = np.concatenate([fvz, np.full((2, 3), -1.0), np.zeros((1, 3)), -np.zeros((1, 3))])
    fvz[7, 0] = np.nan                                         # NaN depth
    fvi[11, 1, 0] = np.inf                                     # infinite coordinate
    fvi[13, 2, 1] = np.nan                                     # NaN coordinate
    fvi[17] = fvi[17, :1]                                      # zero-area face
    feat = g.uniform(-1, 1, (fvi.shape[0], 3, 2))
    np_dt = np.float32 if dtype == torch.float32 else np.float64
    return fvz[None].astype(np_dt), fvi[None].astype(np_dt), feat[None].astype(np_dt)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('backend', ['cuda', 'cuda_packed'])
def test_rasterize_adversarial_vs_oracle(kal, dtype, backend):
    z, v, f = _adversarial_faces(dtype)
    z, v, f = np.concatenate([z, z[:, ::-1]]), np.concatenate([v, v[:, ::-1]]), np.concatenate([f, f[:, ::-1]])
    valid = np.random.default_rng(1).uniform(size=z.shape[:2]) > 0.1
    for vf in (None, valid):
        feats, fidx = kal.render.mesh.rasterize(97, 130, T(z), T(v), T(f), None if vf is None else T(vf),
                                                backend=backend)
        of, oi, ow = orc.rasterize(97, 130, z, v, f, valid_faces=vf)
        assert np.array_equal(A(fidx), oi)
        assert np.array_equal(A(feats), of, equal_nan=True)
        assert (oi >= 0).mean() > 0.5


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('K', [30, 8])
def test_soft_mask_adversarial_vs_oracle(kal, dtype, K):
    from kaolin import _fused
    z, v, f = _adversarial_faces(dtype, seed=6)
    _, sel = kal.render.mesh.rasterize(97, 130, T(z), T(v), T(f))
    m, box, sig = 1000., 0.03, 7000.
    mask, prob, cidx, ctype, hits = _fused.soft_mask_forward(T(v), sel, sig, box, K, m, with_hits=True)
    assert np.array_equal(A(hits), (A(cidx) >= 0).sum(-1))
    fm = v * v.dtype.type(m)
    pad = v.dtype.type(box * m)
    bb = np.concatenate([fm.min(-2) - pad, fm.max(-2) + pad], -1)
    om, op, oi, ot = orc.dibr_soft_mask_forward(fm, bb, A(sel), sig, K, m)
    assert np.array_equal(A(cidx), oi)
    assert np.array_equal(A(ctype), ot)
    np.testing.assert_allclose(A(prob), op, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    assert (oi[..., -1] >= 0).sum() > (100 if K == 8 else -1)  # K=8: many pixels saturate knum
    grad = torch.rand_like(mask)
    # the backward on identical saved values: the GPU forward's mask and probabilities
    ogi = orc.dibr_soft_mask_backward(A(grad), A(mask), A(sel), A(prob), oi, ot, fm, sig, m)
    g1 = _fused.soft_mask_backward(grad, mask, sel, prob, cidx, ctype, T(v), sig, m, hits)
    g2 = kal._C.render.mesh.dibr_soft_mask_backward_cuda(grad, mask, sel, prob, cidx, ctype, T(fm), sig, m)
    assert np.isfinite(ogi).mean() > 0.9
    assert_grads_equal(A(g1), ogi)
    assert_grads_equal(A(g2), ogi)


def test_dibr_bench_sphere_vs_oracle(kal):
    """The bench workload's mesh (50k-face UV sphere, heavy pole tiles) at 128x128:
    rasterizer and soft mask bit-exact / 1e-6 against the oracle."""
    import bench
    inp = bench.dibr_inputs([0.3], DEV, H=128, W=128)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    feats, mask, idx = kal.render.mesh.dibr_rasterization(128, 128, fvz, fvi, feat, fnz, 7000, 0.02, 30, 1000, 1e-8)
    of, oi, ow = orc.rasterize(128, 128, A(fvz), A(fvi), A(feat), valid_faces=A(fnz >= 0))
    assert np.array_equal(A(idx), oi)
    assert np.array_equal(A(feats), of)
    fm = A(fvi) * np.float32(1000.)
    bb = np.concatenate([fm.min(-2) - np.float32(20.), fm.max(-2) + np.float32(20.)], -1)
    om, op, oi2, ot = orc.dibr_soft_mask_forward(fm, bb, oi, 7000., 30, 1000.)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)


def test_rasterize_backward_vs_oracle(kal):
    fvz, fvi, feat, fnz = _render_inputs(kal, 30, 50, 2)
    fvi_r = fvi.clone().requires_grad_(True)
    feat_r = feat.clone().requires_grad_(True)
    feats, fidx = kal.render.mesh.rasterize(80, 80, fvz, fvi_r, feat_r, valid_faces=fnz >= 0)
    go = torch.rand_like(feats)
    feats.backward(go)
    of, oi, ow = orc.rasterize(80, 80, A(fvz), A(fvi), A(feat), valid_faces=A(fnz >= 0))
    gi, gf = orc.rasterize_backward(A(go), oi, ow, A(fvi), A(feat), 1e-8)
    assert_grads_equal(A(fvi_r.grad), gi)
    assert_grads_equal(A(feat_r.grad), gf)
    # the _C contract's scatter backward (rasterize_backward_cuda), directly against the oracle
    w = torch.from_numpy(ow).to(DEV)
    g_img, g_feat = kal._C.render.mesh.rasterize_backward_cuda(go, feats, fidx, w, fvi, feat, 1e-8)
    assert_grads_equal(A(g_img), gi)
    assert_grads_equal(A(g_feat), gf)


def test_packed_rasterize_C_direct(kal):
    """_C entry point with packed inputs (rasterization.cpp:49-104): packed (per-mesh) index."""
    fvz, fvi, feat, fnz = _render_inputs(kal, 12, 20, 2)
    B, F = fvz.shape[:2]
    m = 1000.
    vfvi = (fvi * m).reshape(B * F, 3, 2).contiguous()
    bbox = torch.cat([vfvi.min(1)[0], vfvi.max(1)[0]], 1).contiguous()
    first = torch.tensor([0, F, 2 * F], dtype=torch.long, device=DEV)
    out = kal._C.render.mesh.packed_rasterize_forward_cuda(40, 33, fvz.reshape(-1, 3).contiguous(), vfvi, bbox,
                                                           feat.reshape(-1, 3, 3).contiguous(), first, m, 1e-8)
    assert isinstance(out, list) and len(out) == 3
    of, oi, ow = orc.packed_rasterize_forward(40, 33, A(fvz.reshape(-1, 3)), A(vfvi), A(bbox),
                                              A(feat.reshape(-1, 3, 3)), A(first), m, 1e-8)
    assert np.array_equal(A(out[1]), oi)
    assert np.array_equal(A(out[0]), of)
    assert np.array_equal(A(out[2]), ow)


# ------------------------------------------------------------------ soft mask
def _mask_iou_target(sel):
    mask = sel != -1
    return torch.nn.functional.pad(mask, (0, 5))[..., 5:]


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('sig,box', [(7000, 0.02), (7000, 0.2), (70, 0.02), (70, 0.2)])
@pytest.mark.parametrize('knum', [30, 20])
@pytest.mark.parametrize('multiplier', [1000, 100, 1])
def test_soft_mask_simple_golden(kal, golden, dtype, sig, box, knum, multiplier):
    """test_dibr.py:108-191 on the HIP path."""
    g = golden('dibr_simple.npz')
    fvi = T(g['face_vertices_image'], dtype)
    fvz = T(g['face_vertices_z'], dtype)
    _, sel = kal.render.mesh.rasterize(35, 31, fvz, fvi, torch.zeros(fvz.shape + (1,), dtype=dtype, device=DEV))
    assert np.array_equal(A(sel), g['selected_face_idx'])
    fm = fvi * multiplier
    bb = torch.cat([fm.min(-2)[0] - box * multiplier, fm.max(-2)[0] + box * multiplier], -1)
    mask, prob, cidx, ctype = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb.contiguous(), sel, sig, knum,
                                                                             multiplier)
    np.testing.assert_allclose(A(mask), g[f'soft_mask_{sig}_{box}'], atol=1e-5, rtol=1e-5)
    assert np.array_equal(A(cidx), g[f'close_face_idx_{sig}_{box}'][..., :knum])
    np.testing.assert_allclose(A(prob), g[f'close_face_prob_{sig}_{box}'][..., :knum], atol=1e-5, rtol=1e-5)
    assert np.array_equal(A(ctype), g[f'close_face_dist_type_{sig}_{box}'][..., :knum])
    fvi_r = fvi.clone().requires_grad_(True)
    sm = kal.render.mesh.dibr_soft_mask(fvi_r, sel, sig, box, knum, multiplier)
    loss = kal.metrics.render.mask_iou(sm, _mask_iou_target(sel))
    loss.backward()
    np.testing.assert_allclose(A(fvi_r.grad), g[f'grad_{sig}_{box}'], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('sig,box', [(7000, 0.02), (70, 0.01)])
@pytest.mark.parametrize('knum', [30, 40])
def test_soft_mask_sphere_golden(kal, golden, dname, flip, sig, box, knum):
    """test_dibr.py:297-394 on the HIP path (type <=1% mismatch, grads 1e-1 as the reference)."""
    g = golden('dibr_sphere.npz')
    p = f'{dname}_flip{flip}_'
    fvi, fvz = T(g[p + 'face_vertices_image']), T(g[p + 'face_vertices_z'])
    _, sel = kal.render.mesh.rasterize(35, 31, fvz, fvi, torch.zeros(fvz.shape + (1,), dtype=fvz.dtype, device=DEV))
    for multiplier in (1000, 100):
        fm = fvi * multiplier
        bb = torch.cat([fm.min(-2)[0] - box * multiplier, fm.max(-2)[0] + box * multiplier], -1).contiguous()
        mask, prob, cidx, ctype = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, sig, knum, multiplier)
        np.testing.assert_allclose(A(mask), g[f'soft_mask_{sig}_{box}'], atol=1e-5, rtol=1e-5)
        assert np.array_equal(A(cidx), g[f'close_face_idx_{sig}_{box}'][..., :knum])
        np.testing.assert_allclose(A(prob), g[f'close_face_prob_{sig}_{box}'][..., :knum], atol=1e-5, rtol=1e-5)
        assert np.mean(A(ctype) != g[f'close_face_dist_type_{sig}_{box}'][..., :knum]) <= 0.01
        fvi_r = fvi.clone().requires_grad_(True)
        sm = kal.render.mesh.dibr_soft_mask(fvi_r, sel, sig, box, knum, multiplier)
        kal.metrics.render.mask_iou(sm, _mask_iou_target(sel)).backward()
        np.testing.assert_allclose(A(fvi_r.grad), g[f'grad_{sig}_{box}'], rtol=1e-1, atol=1e-1)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('knum', [30, 7])
def test_soft_mask_vs_oracle(kal, dtype, knum):
    fvz, fvi, feat, fnz = _render_inputs(kal, 30, 50, 3, dtype)
    H, W = 72, 100
    _, sel = kal.render.mesh.rasterize(H, W, fvz, fvi, feat, valid_faces=fnz >= 0)
    m, box, sig = 1000., 0.04, 7000.
    fm = (fvi * m).contiguous()
    bb = torch.cat([fm.min(-2)[0] - box * m, fm.max(-2)[0] + box * m], -1).contiguous()
    mask, prob, cidx, ctype = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, sig, knum, m)
    om, op, oi, ot = orc.dibr_soft_mask_forward(A(fm), A(bb), A(sel), sig, knum, m)
    assert np.array_equal(A(cidx), oi)
    assert np.array_equal(A(ctype), ot)
    np.testing.assert_allclose(A(prob), op, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    assert (oi[..., 0] >= 0).sum() > 100  # the band is exercised
    if knum == 7:
        assert (oi[..., -1] >= 0).sum() > 0  # some pixels saturate knum
    grad = torch.rand_like(mask)
    gi = kal._C.render.mesh.dibr_soft_mask_backward_cuda(grad, mask, sel, prob, cidx, ctype, fm, sig, m)
    ogi = orc.dibr_soft_mask_backward(A(grad), A(mask), A(sel), A(prob), oi, ot, A(fm), sig, m)
    assert_grads_equal(A(gi), ogi)


def test_dibr_rasterization_composition(kal):
    """test_dibr.py:486-529: dibr_rasterization == rasterize + dibr_soft_mask, exactly."""
    fvz, fvi, feat, fnz = _render_inputs(kal, 20, 30, 2)
    f1, sm1, i1 = kal.render.mesh.dibr_rasterization(64, 48, fvz, fvi, feat, fnz, 7000, 0.02, 30, 1000)
    f2, i2 = kal.render.mesh.rasterize(64, 48, fvz, fvi, feat, fnz >= 0., 1000)
    sm2 = kal.render.mesh.dibr_soft_mask(fvi, i2, 7000, 0.02, 30, 1000.)
    assert torch.equal(f1, f2) and torch.equal(i1, i2) and torch.equal(sm1, sm2)


def test_dibr_deterministic_forward(kal):
    fvz, fvi, feat, fnz = _render_inputs(kal, 40, 60, 2)
    r1 = kal.render.mesh.dibr_rasterization(128, 128, fvz, fvi, feat, fnz)
    r2 = kal.render.mesh.dibr_rasterization(128, 128, fvz, fvi, feat, fnz)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


# ------------------------------------------------- compact soft-mask state (fused path)
def _decode_compact(state, H, W, K):
    """The compact records back into the reference's (B,H,W,K) slot tensors."""
    from dibr_util import decode_compact, state_arrays
    return decode_compact(*state_arrays(state), K)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('K', [30, 8, 1])
def test_soft_mask_compact_vs_oracle(kal, dtype, K):
    """Compact fused state: mask bit-exact to the _C path, the records decode to the
    oracle's slots exactly (idx, type) / 1e-6 (prob), gradients 1e-5 -- on adversarial faces."""
    from kaolin import _fused
    z, v, f = _adversarial_faces(dtype, seed=6)
    _, sel = kal.render.mesh.rasterize(97, 130, T(z), T(v), T(f))
    m, box, sig = 1000., 0.03, 7000.
    mask, state = _fused.soft_mask_forward_compact(T(v), sel, sig, box, K, m)
    fm = v * v.dtype.type(m)
    pad = v.dtype.type(box * m)
    bb = np.concatenate([fm.min(-2) - pad, fm.max(-2) + pad], -1)
    om, op, oi, ot = orc.dibr_soft_mask_forward(fm, bb, A(sel), sig, K, m)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    r1 = kal._C.render.mesh.dibr_soft_mask_forward_cuda(T(fm), T(bb), sel, sig, K, m)
    assert np.array_equal(A(mask), A(r1[0]), equal_nan=True)  # NaN where a face has a NaN vertex
    assert np.array_equal(A(state.hits), (oi >= 0).sum(-1))
    idx, typ, prob = _decode_compact(state, 97, 130, K)
    assert np.array_equal(idx, oi)
    assert np.array_equal(typ, ot)
    np.testing.assert_allclose(prob, op, rtol=1e-6, atol=1e-7)
    grad = torch.rand_like(mask)
    ogi = orc.dibr_soft_mask_backward(A(grad), A(mask), A(sel), prob, oi, ot, fm, sig, m)  # GPU's saved values
    g1 = _fused.soft_mask_backward_compact(grad, mask, state, T(v), sig, m)
    assert_grads_equal(A(g1), ogi)
    assert int(state.scratch.item()) == 0


@pytest.mark.parametrize('dname', ['float32', 'float64'])
def test_soft_mask_backward_pinned_bench_mesh(kal, dname):
    """The GPU soft-mask backward (compact state) on the bench's 50k-face UV sphere (2 views at
    96x128) against the independent numpy restatement of dibr_soft_mask_cuda.cu:230-353
    (tests/golden/make_soft_bwd_pin.py:soft_bwd_ref) run on the GPU forward's own saved slots:
    f32 bit-equal to its float terms summed in double and rounded once; f64 within 1e-12 of each
    entry's sum of |terms|."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), 'golden'))
    import make_soft_bwd_pin as M
    from kaolin import _fused
    (name, fvi, fvz, H, W, sig, box, knum, mult, fnz), = [c for c in M.bench_cases() if c[0].endswith(dname)]
    _, sel = kal.render.mesh.rasterize(H, W, T(fvz), T(fvi), T(np.zeros(fvz.shape + (1,), fvz.dtype)),
                                       valid_faces=T(fnz >= 0))
    mask, state = _fused.soft_mask_forward_compact(T(fvi), sel, sig, box, knum, mult)
    up = np.random.RandomState(5).uniform(0, 1, mask.shape).astype(fvi.dtype)
    g = A(_fused.soft_mask_backward_compact(T(up), mask, state, T(fvi), sig, mult)).reshape(-1)
    idx, typ, prob = _decode_compact(state, H, W, knum)
    fm = fvi * fvi.dtype.type(mult)
    exp, ab, n = M.soft_bwd_ref(up, A(mask), A(sel), prob, idx, typ, fm, sig, mult)
    assert n > 10000
    exp, ab = exp.reshape(-1), ab.reshape(-1)
    if g.dtype == np.float32:
        assert_grads_equal(g, exp.astype(np.float32))
    else:
        assert np.all(np.abs(g - exp) <= 1e-12 * ab)


@pytest.mark.parametrize('which', ['both', 'features', 'mask'])
def test_dibr_rasterization_fused_grads_vs_oracle(kal, which):
    """The single-node dibr_rasterization backward (gather + soft terms added in place)
    against the oracle's rasterize_backward + dibr_soft_mask_backward, on the bench mesh."""
    import bench
    inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    a = fvi.clone().requires_grad_(True)
    b = feat.clone().requires_grad_(True)
    feats, mask, idx = kal.render.mesh.dibr_rasterization(96, 128, fvz, a, b, fnz, 7000, 0.02, 30, 1000, 1e-8)
    gf = torch.rand_like(feats)
    gm = torch.rand_like(mask)
    outs, grads = ([feats, mask], [gf, gm]) if which == 'both' else \
        (([feats], [gf]) if which == 'features' else ([mask], [gm]))
    torch.autograd.backward(outs, grads, retain_graph=True)
    of, oi, ow = orc.rasterize(96, 128, A(fvz), A(fvi), A(feat), valid_faces=A(fnz >= 0))
    assert np.array_equal(A(idx), oi) and np.array_equal(A(feats), of)
    fm = A(fvi) * np.float32(1000.)
    bb = np.concatenate([fm.min(-2) - np.float32(20.), fm.max(-2) + np.float32(20.)], -1)
    om, op, oci, oct_ = orc.dibr_soft_mask_forward(fm, bb, oi, 7000., 30, 1000.)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    gi = np.zeros(fm.shape, np.float32)
    gfe = np.zeros(A(feat).shape, np.float32)
    if which in ('both', 'features'):
        gi_r, gfe = orc.rasterize_backward(A(gf), oi, ow, A(fvi), A(feat), 1e-8)
        gi = gi + gi_r
    if which in ('both', 'mask'):
        # the soft-mask backward on the GPU forward's saved values (its mask and probabilities,
        # which equal the oracle's to expf ulps)
        from kaolin import _fused
        _, state = _fused.soft_mask_forward_compact(fvi, idx, 7000., 0.02, 30, 1000.)
        _, _, gp = _decode_compact(state, 96, 128, 30)
        gi = gi + orc.dibr_soft_mask_backward(A(gm), A(mask), oi, gp, oci, oct_, fm, 7000., 1000.)
    assert_grads_equal(A(a.grad), gi)
    assert_grads_equal(A(b.grad), gfe)
    # a second backward through the retained graph gives the same gradients again
    g1 = a.grad.clone()
    a.grad = None
    torch.autograd.backward(outs, grads)
    assert torch.equal(a.grad, g1)


def _dev_param(idx, val):
    from dibr_util import dev_param
    dev_param(idx, val)


def _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, K, box=0.02):
    from kaolin import _fused
    f, i, w, m, st, rg = _fused.dibr_forward(H, W, fvz, fvi, feat, fnz, 7000., box, K, 1000., 1e-8)
    from dibr_util import state_arrays
    hits, rf, rp = state_arrays(st)
    seg = A(st.seg_tot)
    # the records of each row segment up to its hit total (the rest of a segment is unwritten)
    R = 64 * K
    keep = (np.arange(R)[None, :] < seg[:, None]).reshape(-1) if K > 0 else np.zeros(0, bool)
    return [A(f), A(i), A(w), A(m), hits, seg, rf[:keep.size][keep], rp[:keep.size][keep], A(rg)]


@pytest.mark.devlib
@pytest.mark.parametrize('case', ['bench', 'adversarial', 'bigbox'])
def test_dibr_bin_marks_equal_atomic_binning(kal, case):
    """kl_dibr_forward's binning (raster_bin_word_kernel): the r05 per-wave byte marks against the LDS
    atomicOr marking (dev param 22 = 1) -- every output and the compact state equal."""
    import bench
    if case == 'adversarial':
        z, v, f = _adversarial_faces(torch.float32)
        fvz, fvi, feat = T(z), T(v), T(f)
        fnz = T(np.random.default_rng(2).uniform(-0.3, 1, fvz.shape[:2]).astype(np.float32))
        H, W, box = 97, 130, 0.02
    else:
        inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
        fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
        H, W, box = 96, 128, (0.2 if case == 'bigbox' else 0.02)
    marks = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, 30, box)
    try:
        _dev_param(22, 1)
        atomic = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, 30, box)
    finally:
        _dev_param(22, 0)
    names = ['features', 'face_idx', 'weights', 'soft_mask', 'hits', 'seg_tot', 'rec_face', 'rec_prob', 'ranges']
    for n, x, y in zip(names, marks, atomic):
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), n


@pytest.mark.devlib
@pytest.mark.parametrize('case', ['bench', 'adversarial', 'knum255', 'tiny'])
def test_soft_live_flags_equal(kal, case):
    """The soft forward's work items flagged live by the rasterizer (r05: an item whose rows hold no
    uncovered pixel is done after one load) against the unflagged kernel (dev param 26 = 1) -- every
    output and the compact state equal; knum 255 (1-row items), and a 40x24 image (fewer flags than
    the launch's item bound)."""
    import bench
    K, H, W = 30, 96, 128
    if case == 'adversarial':
        z, v, f = _adversarial_faces(torch.float32)
        fvz, fvi, feat = T(z), T(v), T(f)
        fnz = T(np.random.default_rng(2).uniform(-0.3, 1, fvz.shape[:2]).astype(np.float32))
        H, W = 97, 130
    else:
        if case == 'tiny':
            H, W = 40, 24
        inp = bench.dibr_inputs([0.3, 2.0], DEV, H=H, W=W)
        fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
        K = 255 if case == 'knum255' else 30
    flagged = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, K, 0.02)
    try:
        _dev_param(26, 1)
        plain = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, K, 0.02)
    finally:
        _dev_param(26, 0)
    names = ['features', 'face_idx', 'weights', 'soft_mask', 'hits', 'seg_tot', 'rec_face', 'rec_prob', 'ranges']
    for n, x, y in zip(names, flagged, plain):
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), n


@pytest.mark.devlib
@pytest.mark.parametrize('case', ['bench', 'cfg3_views', 'tiny'])
def test_chip_order_barrier_fallback_equal(kal, case):
    """r06: the chip-wide order kernel's grid barrier has a bounded wait; a workgroup that gives up
    counts every tile of its bitmap itself.  Dev param 16 = 1 makes every workgroup take that path at
    once: every output and the compact state equal the barrier's (cfg3's 4 views at 512^2: 4 count
    workgroups per bitmap; 96x128: one)."""
    import bench
    H, W = {'bench': (96, 128), 'cfg3_views': (512, 512), 'tiny': (40, 24)}[case]
    views = [0.0, 1.5707963, 3.1415927, 4.712389] if case == 'cfg3_views' else [0.3, 2.0]
    inp = bench.dibr_inputs(views, DEV, H=H, W=W)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    base = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, 30, 0.02)
    try:
        _dev_param(16, 1)
        fb = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, 30, 0.02)
    finally:
        _dev_param(16, 0)
    names = ['features', 'face_idx', 'weights', 'soft_mask', 'hits', 'seg_tot', 'rec_face', 'rec_prob', 'ranges']
    for n, x, y in zip(names, base, fb):
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), n


@pytest.mark.devlib
@pytest.mark.parametrize('knum,alt', [(30, 2), (30, 3), (8, 2)])
def test_soft_item_rows_equal(kal, knum, alt):
    """The soft forward's rows per work item (4 where the slot lists fit 64 KB of LDS) against
    another split (dev param 20 = alt halvings: 2 or 1 rows) -- every output and the compact
    state equal."""
    import bench
    inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    base = _dibr_fused_forward(fvz, fvi, feat, fnz, 96, 128, knum, 0.02)
    try:
        _dev_param(20, alt)
        other = _dibr_fused_forward(fvz, fvi, feat, fnz, 96, 128, knum, 0.02)
    finally:
        _dev_param(20, 0)
    names = ['features', 'face_idx', 'weights', 'soft_mask', 'hits', 'seg_tot', 'rec_face', 'rec_prob', 'ranges']
    for n, x, y in zip(names, base, other):
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), n


@pytest.mark.devlib
@pytest.mark.parametrize('case', ['bench', 'adversarial', 'knum64', 'knum255', 'bigbox'])
def test_dibr_fused_tile_kernel_equals_two_kernel_path(kal, case):
    """kl_dibr_forward's fused tile kernel (dibrtile.hip: the rasterizer and the soft mask in one
    kernel over one chunk expansion; dev param 10 = 2) against the default two-kernel path
    (raster_tile_kernel then soft_tile_fwd_kernel): face_idx, weights, features, soft mask, the compact state's hits /
    row totals / records, face ranges -- bit for bit; on the bench mesh, adversarial faces (NaN /
    inf / ties / duplicates / big faces), knum 64 and 255 (1-2 rows per work item), and a large
    boxlen whose enlarged bboxes overflow the kernel's LDS soft list (its second expansion)."""
    import bench
    if case in ('adversarial',):
        z, v, f = _adversarial_faces(torch.float32)
        fvz, fvi, feat = T(np.concatenate([z, z[:, ::-1]])), T(np.concatenate([v, v[:, ::-1]])), \
            T(np.concatenate([f, f[:, ::-1]]))
        fnz = T(np.random.default_rng(2).uniform(-0.3, 1, fvz.shape[:2]).astype(np.float32))
        H, W, K, box = 97, 130, 30, 0.02
    else:
        inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
        fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
        H, W = 96, 128
        K = {'knum64': 64, 'knum255': 255}.get(case, 30)
        box = 0.2 if case == 'bigbox' else 0.02
    try:
        two = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, K, box)
        _dev_param(10, 2)
        fused = _dibr_fused_forward(fvz, fvi, feat, fnz, H, W, K, box)
    finally:
        _dev_param(10, 0)
    names = ['features', 'face_idx', 'weights', 'soft_mask', 'hits', 'seg_tot', 'rec_face', 'rec_prob', 'ranges']
    for n, x, y in zip(names, fused, two):
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), n
    assert fused[4].max() > 0  # the soft mask has hits


def test_soft_mask_compact_knum_over_55(kal):
    """knum > 55 puts at most 2 rows in a soft-mask work item (softtile.hip soft_lp_min), so
    every row is walked by 2-4 waves: the compact standalone soft mask against the oracle there."""
    from kaolin import _fused
    import bench
    inp = bench.dibr_inputs([0.3], DEV, H=64, W=96)
    fvi = inp['fvi']
    _, sel = kal.render.mesh.rasterize(64, 96, inp['fvz'], fvi, inp['feat'], valid_faces=inp['fnz'] >= 0)
    for K in (64, 200):
        mask, state = _fused.soft_mask_forward_compact(fvi, sel, 7000., 0.05, K, 1000.)
        fm = A(fvi) * np.float32(1000.)
        pad = np.float32(0.05 * 1000.)
        bb = np.concatenate([fm.min(-2) - pad, fm.max(-2) + pad], -1)
        om, op, oi, ot = orc.dibr_soft_mask_forward(fm, bb, A(sel), 7000., K, 1000.)
        np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
        idx, typ, prob = _decode_compact(state, 64, 96, K)
        assert np.array_equal(idx, oi) and np.array_equal(typ, ot)
        assert (oi >= 0).sum(-1).max() > 30  # deep slot lists


def test_compiled_node_equals_python_node(kal, monkeypatch):
    """csrc/torch_ops.cpp's compiled autograd node (the eager default) against the ctypes / Python
    node (kaolin/_fused.py): forward and gradients bit-equal, features as a list, a retained
    second backward included."""
    from kaolin import _ext
    assert _ext.get() is not None, 'the compiled node is not built (kaolin/_lib/ext)'
    import bench
    inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    runs = []
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(_ext, '_mod', None)
        a = fvi.clone().requires_grad_(True)
        u = feat[..., :2].contiguous().requires_grad_(True)
        o = feat[..., 2:].contiguous().requires_grad_(True)
        (fu, fo), mask, idx = kal.render.mesh.dibr_rasterization(96, 128, fvz, a, [u, o], fnz)
        # a C++ custom Function's node shows as CppFunction in Python; its name() is CppNode<...>
        name = type(mask.grad_fn).__name__ + ' ' + mask.grad_fn.name()
        assert ('CppNode' in name and 'DibrRasterization' in name) if use_ext else 'DibrRasterizationCuda' in name, name
        g = torch.Generator(device='cpu').manual_seed(5)
        grads = [torch.rand(t.shape, generator=g).to(DEV) for t in (fu, fo, mask)]
        torch.autograd.backward([fu, fo, mask], grads, retain_graph=True)
        first = (a.grad.clone(), u.grad.clone(), o.grad.clone())
        a.grad = u.grad = o.grad = None
        torch.autograd.backward([fu, fo, mask], grads)
        assert torch.equal(a.grad, first[0]) and torch.equal(u.grad, first[1]) and torch.equal(o.grad, first[2])
        runs.append((fu, fo, mask, idx) + first)
    for x, y in zip(runs[0], runs[1]):
        assert torch.equal(x, y)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('cams', ['rot_trans', 'transform'])
def test_compiled_tutorial_nodes_equal_python_nodes(kal, monkeypatch, dtype, cams):
    """The tutorial loop's other library ops as compiled nodes (csrc/torch_ops.cpp: prepare_vertices,
    mask_iou, texture_mapping) against their Python / ctypes nodes: outputs and every gradient
    (vertices, cameras, projection, texture, coordinates, both masks) bit-equal."""
    from kaolin import _ext
    assert _ext.get() is not None, 'the compiled nodes are not built (kaolin/_lib/ext)'
    g = torch.Generator(device='cpu').manual_seed(3)
    B = 2
    sv, sf = _uv_sphere(6, 8, 0.5)  # a well-conditioned mesh (random faces make f64 sums ill-conditioned)
    verts = (torch.from_numpy(sv)[None] + (torch.rand((1, len(sv), 3), generator=g, dtype=torch.float64) - 0.5)
             * 0.05).to(dtype)
    faces = torch.from_numpy(np.asarray(sf, dtype=np.int64))
    proj = torch.tensor([[2.0], [2.0], [-1.0]], dtype=dtype)
    rot = torch.linalg.qr(torch.rand((B, 3, 3), generator=g, dtype=torch.float64))[0].to(dtype)
    trans = torch.rand((B, 3), generator=g, dtype=dtype) * 0.1 + torch.tensor([0, 0, 3.], dtype=dtype)
    xf = torch.cat([rot, trans[:, None]], 1)
    tex = torch.rand((B, 3, 16, 24), generator=g, dtype=dtype)
    uv = torch.rand((B, 12, 10, 2), generator=g, dtype=dtype) * 1.2 - 0.1
    m1 = torch.rand((B, 12, 10), generator=g, dtype=dtype)
    m2 = (torch.rand((B, 12, 10), generator=g) > 0.5).to(dtype)
    runs = []
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(_ext, '_mod', None)
        leaves = [t.to(DEV).requires_grad_(True) for t in (verts, proj, rot, trans, xf, tex, uv, m1, m2)]
        v_, p_, r_, t_, x_, tx_, uv_, a_, b_ = leaves
        if cams == 'rot_trans':
            fvc, fvi, fn = kal.render.mesh.prepare_vertices(v_, faces.to(DEV), p_, camera_rot=r_, camera_trans=t_)
        else:
            fvc, fvi, fn = kal.render.mesh.prepare_vertices(v_, faces.to(DEV), p_, camera_transform=x_)
        img = kal.render.mesh.texture_mapping(uv_, tx_, mode='bilinear')
        loss = kal.metrics.render.mask_iou(a_, b_)
        def node(t):  # the op's own node under any view / reshape nodes
            n = t.grad_fn
            while 'View' in n.name() or 'Reshape' in n.name():
                n = n.next_functions[0][0]
            return n.name()
        names = [node(fvc), node(img), node(loss)]
        assert all('CppNode' in n for n in names) if use_ext else not any('CppNode' in n for n in names), names
        gg = torch.Generator(device='cpu').manual_seed(9)
        outs = [fvc, fvi, fn, img]
        ups = [torch.rand(o.shape, generator=gg, dtype=dtype).to(DEV) for o in outs]
        torch.autograd.backward(outs + [loss], ups + [torch.tensor(0.7, dtype=dtype, device=DEV)])
        runs.append([o.detach() for o in outs + [loss]] + [t.grad if t.grad is not None else torch.zeros(())
                                                           for t in leaves])
    for k, (x, y) in enumerate(zip(runs[0], runs[1])):
        if dtype == torch.float64 and k >= 5:
            # f64 gradient terms are summed with double atomics (order-dependent last bits)
            d = (x - y).abs().max().item() if x.numel() else 0.0
            assert torch.allclose(x, y, rtol=1e-12, atol=1e-12), (k, d)
        else:
            assert torch.equal(x, y), k


def test_compiled_nodes_refuse_double_backward(kal):
    """dibr_rasterization's backward is one HIP call (as the reference's CUDA backward):
    backward(create_graph=True) raises instead of returning gradients that silently drop the op's
    second-order term."""
    from kaolin import _ext
    assert _ext.get() is not None
    import bench
    inp = bench.dibr_inputs([0.3], DEV, H=32, W=48)
    fvi = inp['fvi'].clone().requires_grad_(True)
    f, m, _ = kal.render.mesh.dibr_rasterization(32, 48, inp['fvz'], fvi, inp['feat'], inp['fnz'])
    with pytest.raises(RuntimeError, match='create_graph'):
        torch.autograd.grad(m.sum() + f.sum(), fvi, create_graph=True)


@pytest.mark.parametrize('route', ['compiled', 'python'])
def test_torch_reference_nodes_double_backward(kal, monkeypatch, route):
    """mask_iou, prepare_vertices and texture_mapping are plain torch in the reference, so their
    gradients are differentiable there.  Under create_graph the HIP nodes take the
    reference chain's gradient (csrc/torch_ops.cpp *_chain; kaolin/_double_backward.py for the
    Python nodes): first derivatives equal the reference chain's own, bit for bit, and second
    derivatives to the engine's summation order (texture_mapping: grid_sample's backward has no
    derivative in torch, so its second derivative raises in both); an ordinary backward stays on
    the HIP path."""
    from kaolin import _ext
    from kaolin.metrics.render import _mask_iou_torch
    from kaolin.render.mesh.utils import _prepare_vertices_torch, _texture_mapping_torch
    if route == 'python':
        monkeypatch.setattr(_ext, 'get', lambda: None)
    else:
        assert _ext.get() is not None

    def derivs(f, inputs, second=True):
        xs = [x.detach().clone().requires_grad_(True) for x in inputs]
        ys = f(*xs)
        ys = list(ys) if isinstance(ys, (list, tuple)) else [ys]
        loss = sum((y * (k + 1.5)).sum() for k, y in enumerate(ys))
        d1 = torch.autograd.grad(loss, xs, create_graph=True, allow_unused=True)
        out = [d.detach() for d in d1 if d is not None]
        sec = []
        if second:
            sec = [d for d in torch.autograd.grad(sum((d * d).sum() for d in d1 if d is not None), xs,
                                                  allow_unused=True) if d is not None]
        return [y.detach() for y in ys], out, sec

    def check(f1, f2, inputs, second=True):
        (ya, a, a2), (yb, b, b2) = derivs(f1, inputs, second), derivs(f2, inputs, second)
        for x, y in zip(ya, yb):  # the HIP forward: within float rounding of torch's (not bit-equal)
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-5)
        assert len(a) == len(b) and len(a2) == len(b2)
        for x, y in zip(a, b):  # first derivatives: the reference chain's, bit for bit
            assert torch.equal(x, y)
        # second derivatives: the chain's, up to the order the autograd engine adds a tensor's
        # gradient contributions in (node creation order: the chain is rebuilt inside the backward)
        for x, y in zip(a2, b2):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)

    gen = torch.Generator().manual_seed(4)
    a = torch.rand((2, 8, 8), generator=gen).to(DEV)
    b = torch.rand((2, 8, 8), generator=gen).to(DEV)
    check(kal.metrics.render.mask_iou, _mask_iou_torch, [a, b])
    verts = torch.rand((2, 30, 3), generator=gen).to(DEV)
    faces = torch.stack([torch.randperm(30, generator=gen)[:3] for _ in range(40)]).to(DEV)
    proj = torch.tensor([[1.8], [1.8], [-1.]], device=DEV)
    rot = torch.linalg.qr(torch.randn((2, 3, 3), generator=gen))[0].to(DEV)
    trans = torch.tensor([[0., 0., 3.], [0.1, 0., 3.2]], device=DEV)
    check(lambda *x: kal.render.mesh.prepare_vertices(x[0], faces, x[1], x[2], x[3]),
          lambda *x: _prepare_vertices_torch(x[0], faces, x[1], x[2], x[3], None), [verts, proj, rot, trans])
    uv = torch.rand((2, 5, 7, 2), generator=gen).to(DEV)
    tex = torch.rand((2, 3, 16, 16), generator=gen).to(DEV)
    for mode in ('bilinear', 'nearest'):
        f1 = lambda c, t: kal.render.mesh.texture_mapping(c, t, mode)  # noqa: E731
        f2 = lambda c, t: _texture_mapping_torch(c, t, mode)  # noqa: E731
        check(f1, f2, [uv, tex], second=False)
        for fn in (f1, f2):
            with pytest.raises(RuntimeError, match='grid_sampler_2d_backward is not implemented'):
                derivs(fn, [uv, tex])
    # an ordinary backward stays on the HIP node
    x = a.clone().requires_grad_(True)
    torch.autograd.grad(kal.metrics.render.mask_iou(x, b), x)


def test_dibr_mixed_dtypes_raise(kal, monkeypatch):
    """A float input of another dtype than face_vertices_image raises (the reference's
    data_ptr<scalar_t>() check) on the compiled node and on the Python node alike -- it is
    never read as the wrong type."""
    from kaolin import _ext
    import bench
    inp = bench.dibr_inputs([0.3], DEV, H=32, W=48)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(_ext, '_mod', None)
        for args in ((fvz, fvi, feat.double(), fnz), (fvz.double(), fvi, feat, fnz),
                     (fvz, fvi, [feat[..., :2].double(), feat[..., 2:].double()], fnz)):
            with pytest.raises(RuntimeError):
                kal.render.mesh.dibr_rasterization(32, 48, *args)
        # and on the direct compiled entry point, past the front-end's routing
        if use_ext and _ext.get() is not None:
            from kaolin import _native as N
            with pytest.raises(RuntimeError):
                _ext.get().dibr_rasterization(32, 48, fvz, fvi, feat.double(), fnz, 7000., 0.02, 30, 1000., 1e-8,
                                              N.stream_of(fvi.device))


def test_dibr_bench_full_size_fused_equals_C_chain(kal):
    """cfg3 at full size (4 views, 512^2, 50k faces): the fused single-node path's
    outputs equal the reference-contract chain (packed _C rasterizer + _C soft mask)
    exactly; gradients agree to float summation order."""
    import bench
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], DEV)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    a1, b1 = fvi.clone().requires_grad_(True), feat.clone().requires_grad_(True)
    f1, m1, i1 = kal.render.mesh.dibr_rasterization(512, 512, fvz, a1, b1, fnz)
    (f1 * inp['g_feat']).sum().add((m1 * inp['g_mask']).sum()).backward()
    a2, b2 = fvi.clone().requires_grad_(True), feat.clone().requires_grad_(True)
    f2, i2 = kal.render.mesh.rasterize(512, 512, fvz, a2, b2, fnz >= 0, backend='cuda_packed')
    fm = (a2 * 1000.)
    bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
    m2 = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm.detach().contiguous(), bb.detach(), i2, 7000., 30,
                                                        1000.)[0]
    assert torch.equal(f1, f2) and torch.equal(i1, i2) and torch.equal(m1, m2)
    sm = kal.render.mesh.dibr_soft_mask(a2, i2, 7000, 0.02, 30, 1000.)
    assert torch.equal(sm, m2)
    (f2 * inp['g_feat']).sum().add((sm * inp['g_mask']).sum()).backward()
    assert torch.equal(a1.grad, a2.grad)  # both sum in double and round once
    assert torch.equal(b1.grad, b2.grad)


# ------------------------------------------------------------ point_to_mesh
def test_p2m_kat(kal, golden):
    g = golden('p2m.npz')
    for dtype in (torch.float32, torch.float64):
        d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(T(g['kat_points'], dtype).unsqueeze(0),
                                                                  T(g['kat_face_vertices'], dtype).unsqueeze(0))
        np.testing.assert_allclose(A(d[0]), g['kat_dist'], rtol=1e-5, atol=1e-8)
        assert np.array_equal(A(i[0]), g['kat_face_idx'])
        assert np.array_equal(A(t[0]), g['kat_dist_type'])


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_p2m_random_fixture(kal, golden, dname):
    g = golden('p2m.npz')
    p = f'rand_{dname}_'
    P = T(g[p + 'points']).requires_grad_(True)
    FV = T(g[p + 'face_vertices']).requires_grad_(True)
    d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(P.unsqueeze(0), FV.unsqueeze(0))
    np.testing.assert_allclose(A(d[0]), g[p + 'dist'], rtol=1e-5, atol=1e-8)
    assert np.array_equal(A(i[0]), g[p + 'face_idx'])
    assert np.array_equal(A(t[0]), g[p + 'dist_type'])
    od, oi, ot = orc.unbatched_triangle_distance_forward(g[p + 'points'], g[p + 'face_vertices'])
    assert np.array_equal(A(d[0]), od) and np.array_equal(A(i[0]), oi) and np.array_equal(A(t[0]), ot)
    d.backward(T(g[p + 'grad_out']).unsqueeze(0))
    np.testing.assert_allclose(A(P.grad), g[p + 'grad_points'], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(A(FV.grad), g[p + 'grad_face_vertices'], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('P,F', [(3000, 1800), (700, 513), (64, 1)])
def test_p2m_vs_oracle(kal, P, F):
    g = torch.Generator(device='cpu').manual_seed(P + F)
    pts = torch.randn((P, 3), generator=g)
    fv = torch.randn((F, 3, 3), generator=g)
    d = torch.empty(P, device=DEV)
    i = torch.empty(P, dtype=torch.long, device=DEV)
    t = torch.empty(P, dtype=torch.int32, device=DEV)
    kal._C.metrics.unbatched_triangle_distance_forward_cuda(pts.to(DEV), fv.to(DEV), d, i, t)
    od, oi, ot = orc.unbatched_triangle_distance_forward(pts.numpy(), fv.numpy())
    assert np.array_equal(A(d), od) and np.array_equal(A(i), oi) and np.array_equal(A(t), ot)
    gr = torch.rand(P, generator=g)
    gp = torch.empty((P, 3), device=DEV)
    gf = torch.empty((F, 3, 3), device=DEV)
    kal._C.metrics.unbatched_triangle_distance_backward_cuda(gr.to(DEV), pts.to(DEV), fv.to(DEV), i, t, gp, gf)
    ogp, ogf = orc.unbatched_triangle_distance_backward(gr.numpy(), pts.numpy(), fv.numpy(), oi, ot)
    # grad_points per point: bit-exact; the face gradient summed in double on both sides, rounded once
    assert np.array_equal(A(gp), ogp)
    assert_grads_equal(A(gf), ogf)


def _p2m_stress(kind, dtype):
    g = np.random.default_rng({'cfg2': 0, 'slivers': 1, 'scaled': 2, 'onsurface': 3, 'dups': 4}[kind])
    if kind == 'cfg2':  # the bench distribution at a smaller size
        pts, fv = g.standard_normal((20000, 3)), g.standard_normal((1100, 3, 3))
    elif kind == 'dups':  # proper faces duplicated within and across the face splits (distance ties)
        fv = g.standard_normal((1100, 3, 3))
        fv[600:700] = fv[0:100]
        fv[1050:1100] = fv[20:70]
        fv[300:310] = fv[290:300]
        pts = g.standard_normal((20000, 3))
        pts[:3000] = fv[g.integers(0, 100, 3000), 1]  # on duplicated vertices: distance-0 ties
    elif kind == 'slivers':  # needle / collinear / zero-area faces, duplicates across 512-tiles
        fv = g.standard_normal((1200, 3, 3))
        fv[::7, 2] = fv[::7, 0] + 1e-4 * g.standard_normal((len(fv[::7]), 3))       # needles
        fv[1::7, 2] = 0.5 * (fv[1::7, 0] + fv[1::7, 1])                                # collinear
        fv[2::11, 1] = fv[2::11, 0]                                                    # zero-length edge
        fv[600:700] = fv[0:100]                                                        # duplicates
        fv[[512, 1024]] = fv[[512, 1024], :1]                                          # degenerate tile starts
        pts = g.standard_normal((15000, 3)) * 0.5
    elif kind == 'scaled':  # large offsets and scales
        fv = g.standard_normal((1100, 3, 3)) * 300 + 2000
        pts = g.standard_normal((16000, 3)) * 300 + 2000
    else:  # points exactly on faces / vertices (distance 0 ties) + a NaN point
        fv = g.standard_normal((1100, 3, 3))
        w = g.dirichlet([1, 1, 1], 16000)
        pick = g.integers(0, 1100, 16000)
        pts = np.einsum('pk,pkc->pc', w, fv[pick])
        pts[::5] = fv[pick[::5], 0]
        pts[77] = np.nan
    np_dt = np.float32 if dtype == torch.float32 else np.float64
    return pts.astype(np_dt), fv.astype(np_dt)


@pytest.mark.devlib
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('kind', ['cfg2', 'slivers', 'scaled', 'onsurface', 'dups'])
@pytest.mark.parametrize('walk', ['pairs', 'wave', 'pairs_r05'])
def test_p2m_face_skipping_is_exact(kal, kind, dtype, walk):
    """P*F >= 2^24 takes the Morton-ordered path whose waves skip faces that provably cannot
    be nearest; results must stay bit-identical to the oracle's full scan -- with the per-point pair
    queue (default, r06: per-point tests only for the (face, 8-point sub-cluster) pairs a sub-cluster
    bound keeps; proper faces and finite waves), with the r05 pair queue (every kept face's per-point
    test, dev param 11 = 5) and with the wave-level walk alone (dev param 11 = 4).  'dups': duplicated proper faces within and across the face splits, points on their
    vertices (distance-0 ties: the earliest face wins)."""
    pts, fv = _p2m_stress(kind, dtype)
    P, F = len(pts), len(fv)
    assert P * F >= 1 << 24
    d = torch.empty(P, dtype=dtype, device=DEV)
    i = torch.empty(P, dtype=torch.long, device=DEV)
    t = torch.empty(P, dtype=torch.int32, device=DEV)
    try:
        _dev_param(11, {'wave': 4, 'pairs_r05': 5}.get(walk, 0))
        kal._C.metrics.unbatched_triangle_distance_forward_cuda(T(pts), T(fv), d, i, t)
    finally:
        _dev_param(11, 0)
    od, oi, ot = orc.unbatched_triangle_distance_forward(pts, fv)
    assert np.array_equal(A(d), od, equal_nan=True)
    assert np.array_equal(A(i), oi) and np.array_equal(A(t), ot)


# ------------------------------------------------------------ sided distance
def test_sided_kat_and_ties(kal, golden):
    g = golden('sided.npz')
    for dtype in (torch.float16, torch.float32, torch.float64):
        d, i = kal.metrics.pointcloud.sided_distance(T(g['kat_p1'], dtype), T(g['kat_p2'], dtype))
        tol = 1e-3 if dtype == torch.float16 else 1e-4
        np.testing.assert_allclose(A(d.double()), g['kat_dist'], rtol=tol, atol=tol * 10 if dtype == torch.float16 else 1e-5)
        assert np.array_equal(A(i), g['kat_idx'])
    d, i = kal.metrics.pointcloud.sided_distance(T(g['large_p1']), T(g['large_p2']))
    od, oi = orc.sided_distance_forward(g['large_p1'], g['large_p2'])
    assert np.array_equal(A(d), od) and np.array_equal(A(i), oi)
    np.testing.assert_allclose(A(d), g['large_dist'])


@pytest.mark.devlib
@pytest.mark.parametrize('dtype', [torch.float16, torch.float32, torch.float64, torch.int32, torch.uint8])
def test_sided_tile_splits_equal_one_pass(kal, dtype):
    """sided_distance's forward with p2's 512-point tiles split over workgroups (default when the
    point blocks are few) against one pass over all tiles (dev param 23 = 1): distances and indices
    bit-equal, with duplicated p2 points across tiles (ties: the earliest index), NaN p2 points at
    tile starts and inside tiles (f32), and p2 sizes not a multiple of 512; f32 also against the
    oracle."""
    rng = np.random.default_rng(7)
    for (B, N, M) in ((1, 300, 2600), (2, 77, 1537), (1, 2048, 2048)):
        p1 = rng.random((B, N, 3)) * 4
        p2 = rng.random((B, M, 3)) * 4
        p2[:, 1024:1100] = p2[:, 0:76]   # ties across tiles
        if M >= 1612:
            p2[:, 1600:1612] = p2[:, 520:532]
        if dtype.is_floating_point:
            if dtype == torch.float32:
                p2[0, 512] = np.nan      # a tile's first point
                p2[0, 1030] = np.nan     # inside a tile
        else:
            p1, p2 = np.floor(p1 * 3), np.floor(p2 * 3)
        a, b = T(p1, dtype), T(p2, dtype)
        d, i = kal.metrics.pointcloud.sided_distance(a, b)
        try:
            _dev_param(23, 1)
            d1, i1 = kal.metrics.pointcloud.sided_distance(a, b)
        finally:
            _dev_param(23, 0)
        assert torch.equal(i, i1) and np.array_equal(A(d), A(d1), equal_nan=True), (B, N, M)
        if dtype == torch.float32:
            for k in range(B):
                od, oi = orc.sided_distance_forward(A(a[k:k + 1]), A(b[k:k + 1]))
                assert np.array_equal(A(d[k:k + 1]), od, equal_nan=True) and np.array_equal(A(i[k:k + 1]), oi)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_sided_vs_oracle_and_grad(kal, golden, dtype):
    g = golden('sided.npz')
    p1 = T(g['rand_p1'], dtype).requires_grad_(True)
    p2 = T(g['rand_p2'], dtype).requires_grad_(True)
    d, i = kal.metrics.pointcloud.sided_distance(p1, p2)
    od, oi = orc.sided_distance_forward(A(p1), A(p2))
    assert np.array_equal(A(d), od) and np.array_equal(A(i), oi)
    np.testing.assert_allclose(A(d), g['rand_dist'], rtol=1e-5, atol=1e-6)
    gr = torch.rand_like(d)
    d.backward(gr)
    og1, og2 = orc.sided_distance_backward(A(gr), A(p1), A(p2), oi)
    np.testing.assert_allclose(A(p1.grad), og1, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(A(p2.grad), og2, rtol=1e-5, atol=1e-5)


def test_sided_gradcheck(kal):
    g = torch.Generator().manual_seed(0)
    p1 = torch.randn((5, 20, 3), generator=g, dtype=torch.double).to(DEV).requires_grad_(True)
    p2 = torch.randn((5, 15, 3), generator=g, dtype=torch.double).to(DEV).requires_grad_(True)
    assert torch.autograd.gradcheck(kal.metrics.pointcloud.sided_distance, (p1, p2), eps=1e-6, atol=1e-6)


def test_sided_error_messages(kal):
    """test_pointcloud.py:124-152: messages matched verbatim."""
    with pytest.raises(RuntimeError, match=r"Expected tensor of size \[3, 3, 3\], but got tensor of size \[2, 3, 3\] "
                                           r"for argument #2 'p2' \(while checking arguments for "
                                           r"sided_distance_forward_cuda\)"):
        kal.metrics.pointcloud.sided_distance(torch.randint(0, 10, (3, 2, 3), device=DEV).float(),
                                              torch.randint(0, 10, (2, 3, 3), device=DEV).float())
    with pytest.raises(RuntimeError, match="Expected 3-dimensional tensor, but got 4-dimensional tensor for "
                                           r"argument #1 'p1' \(while checking arguments for "
                                           r"sided_distance_forward_cuda\)"):
        kal.metrics.pointcloud.sided_distance(torch.rand((3, 2, 3, 4), device=DEV), torch.rand((2, 3, 3), device=DEV))


def test_chamfer_and_fscore(kal, golden):
    g = golden('sided.npz')
    p1, p2 = T(g['rand_p1']), T(g['rand_p2'])
    ch = kal.metrics.pointcloud.chamfer_distance(p1, p2)
    d1, _ = orc.sided_distance_forward(g['rand_p1'], g['rand_p2'])
    d2, _ = orc.sided_distance_forward(g['rand_p2'], g['rand_p1'])
    np.testing.assert_allclose(A(ch), d1.mean(-1) + d2.mean(-1), rtol=1e-5)
    fs = kal.metrics.pointcloud.f_score(p1, p2, radius=0.05)
    assert fs.shape == (2,) and torch.all((fs >= 0) & (fs <= 1))


# reference tests/python/kaolin/metrics/test_pointcloud.py:305-346 (TestFScore) and the
# f_score docstring example (metrics/pointcloud.py:158-169): inputs and expected values as data
_FS_GT = [[[8.8977, 4.1709, 1.2839], [8.5640, 7.7767, 9.4214]],
          [[0.5431, 6.4495, 11.4914], [3.2126, 8.0865, 3.1018]]]
_FS_PRED = [[[8.8914, 4.1788, 1.2176], [8.5291, 7.5513, 9.5412]],
            [[0.4010, 6.4602, 11.5183], [3.2977, 8.0325, 3.1180]]]
_FS_PRED3 = [[[8.8914, 4.1788, 1.2176], [8.5291, 7.5513, 9.5412], [3.7831, 6.0182, 4.1208]],
             [[0.4010, 6.4602, 11.5183], [3.2977, 8.0325, 3.1180], [2.4987, 5.8763, 3.1987]]]
_FS_TOL = {torch.half: (1e-3, 1e-3), torch.float32: (1e-5, 1e-4), torch.float64: (1e-6, 1e-5)}


@pytest.mark.parametrize('dtype', [torch.half, torch.float32, torch.float64])
def test_fscore_reference_kats(kal, dtype):
    atol, rtol = _FS_TOL[dtype]
    gt = torch.tensor(_FS_GT, dtype=dtype, device=DEV)
    for pred, e1, e2 in ((_FS_PRED, [0.5, 1.0], [0.5, 0.5]), (_FS_PRED3, [0.4, 0.8], [0.4, 0.4])):
        pr = torch.tensor(pred, dtype=dtype, device=DEV)
        o1 = kal.metrics.pointcloud.f_score(gt, pr, radius=0.2)
        o2 = kal.metrics.pointcloud.f_score(gt, pr, radius=0.12)
        assert o1.dtype == dtype
        assert torch.allclose(o1, torch.tensor(e1, dtype=dtype, device=DEV), atol=atol, rtol=rtol)
        assert torch.allclose(o2, torch.tensor(e2, dtype=dtype, device=DEV), atol=atol, rtol=rtol)
    if dtype == torch.half:  # the docstring example is f32; in half eps=1e-8 underflows (0/0 in both)
        return
    p1 = torch.tensor([[[8.8977, 4.1709, 1.2839], [8.5640, 7.7767, 9.4214]],
                       [[0.5431, 6.4495, 11.4914], [3.2126, 8.0865, 3.1018]]], device=DEV, dtype=dtype)
    p2 = torch.tensor([[[9.4863, 4.2249, 0.1712], [8.1783, 8.5310, 8.5119]],
                       [[-0.0020699, 6.4429, 12.3], [3.8386, 8.3585, 4.7662]]], device=DEV, dtype=dtype)
    assert torch.allclose(kal.metrics.pointcloud.f_score(p1, p2, radius=1),
                          torch.tensor([0.0, 0.5], device=DEV, dtype=dtype), atol=atol, rtol=rtol)
    assert torch.allclose(kal.metrics.pointcloud.f_score(p1, p2, radius=1.5),
                          torch.tensor([1.0, 0.5], device=DEV, dtype=dtype), atol=atol, rtol=rtol)


# ------------------------------------------------------------ voxelgrid
@pytest.mark.parametrize('name', ['batched', 'origins', 'scale', 'res7', 'default_os', 'sphere32', 'random24'])
def test_voxelgrid_golden(kal, golden, name):
    g = golden('voxelgrid.npz')
    o = T(g[f'{name}_origin']) if f'{name}_origin' in g else None
    s = T(g[f'{name}_scale']) if f'{name}_scale' in g else None
    vg = kal.ops.conversions.trianglemeshes_to_voxelgrids(T(g[f'{name}_vertices']), T(g[f'{name}_faces']),
                                                          int(g[f'{name}_resolution']), o, s)
    assert np.array_equal(np.argwhere(A(vg)).astype(np.int32), g[f'{name}_occupied'])
    assert set(np.unique(A(vg))) <= {0.0, 1.0}


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_voxelgrid_default_bounds_equal_torch(kal, dtype):
    """kl_voxelgrid_bounds: the default origin / scale (trianglemesh.py:74-77) equal torch's
    min / max reductions exactly, NaN propagated per coordinate."""
    from kaolin import _native as N
    g = torch.Generator().manual_seed(11)
    v = (torch.randn((3, 5000, 3), generator=g, dtype=torch.float64) * 3 - 1).to(dtype)
    v[1, 17, 2] = float('nan')
    v[2, :, 0] = -0.0
    vd = v.to(DEV)
    o = torch.empty((3, 3), dtype=dtype, device=DEV)
    sc = torch.empty((3,), dtype=dtype, device=DEV)
    nb = N.lib().kl_voxelgrid_bounds_workspace_bytes(3)
    ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
    N.check(N.lib().kl_voxelgrid_bounds(N.dtype_code(dtype), 3, 5000, N.ptr(vd), N.ptr(o), N.ptr(sc), N.ptr(ws), nb,
                                        N.stream_of(vd.device)), 'bounds')
    ro = torch.min(v, dim=1)[0]
    rs = torch.max(torch.max(v, dim=1)[0] - ro, dim=1)[0]
    assert torch.equal(torch.isnan(o.cpu()), torch.isnan(ro)) and torch.equal(torch.isnan(sc.cpu()), torch.isnan(rs))
    fin = ~torch.isnan(ro)
    assert torch.equal(o.cpu()[fin], ro[fin])
    assert torch.equal(sc.cpu()[~torch.isnan(rs)], rs[~torch.isnan(rs)])


def test_voxelgrid_sparse(kal, golden):
    g = golden('voxelgrid.npz')
    vg = kal.ops.conversions.trianglemeshes_to_voxelgrids(T(g['batched_vertices']), T(g['batched_faces']), 3,
                                                          T(g['batched_origin']), T(g['batched_scale']),
                                                          return_sparse=True)
    assert vg.is_sparse
    assert np.array_equal(np.argwhere(A(vg.to_dense())).astype(np.int32), g['batched_occupied'])


def test_voxelgrid_vs_oracle_sphere(kal):
    v, f = _uv_sphere(40, 64, 0.95)
    vg = kal.ops.conversions.trianglemeshes_to_voxelgrids(T(v, torch.float32).unsqueeze(0), T(f), 96)
    ov = orc.voxelgrid(v[None].astype(np.float32), f, 96)
    assert np.array_equal(A(vg).astype(np.uint8), ov)


def _voxel_async(points, faces, R, cap, grid_dtype=torch.float32):
    """kl_voxelgrid_mark_async on one mesh at an explicit capacity -> (grid, status)."""
    from kaolin import _native as N
    lib = N.lib()
    code = N.dtype_code(points.dtype)
    nb = lib.kl_voxelgrid_mark_async_workspace_bytes(code, cap)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=DEV)
    grid = torch.zeros((R, R, R), dtype=grid_dtype, device=DEV)
    status = torch.full((1,), -1, dtype=torch.int32, device=DEV)
    N.check(lib.kl_voxelgrid_mark_async(code, points.shape[0], N.ptr(points), faces.shape[0], N.ptr(faces), R,
                                        N.dtype_code(grid_dtype), N.ptr(grid), cap, N.ptr(status), N.ptr(ws), nb,
                                        N.stream_of(points.device)), 'voxel async')
    return grid, int(status.item())


@pytest.mark.devlib
@pytest.mark.parametrize('R', [64, 300])
def test_voxelgrid_tail_kernel_levels_equal(kal, R):
    """r06: the subdivision's later levels in one persistent launch (grid barriers between levels)
    against every level its own launch (dev param 21 = 1) and against the persistent kernel from level
    1 on (21 = 3), at capacities that overflow some level and that hold every level: grids equal."""
    from dibr_util import require_dev
    require_dev()
    v, f = _uv_sphere(20, 32, 0.95)
    vt, ft = T(v, torch.float32).unsqueeze(0), T(f)
    o = torch.min(vt, dim=1)[0]
    sc = torch.max(torch.max(vt, dim=1)[0] - o, dim=1)[0]
    pts = ((vt - o.unsqueeze(1)) / sc.view(-1, 1, 1))[0].contiguous()
    for cap in (300, 1 << 20):
        grids = {}
        try:
            for dp in (0, 1, 3):
                _dev_param(21, dp)
                grids[dp] = _voxel_async(pts, ft, R, cap)
        finally:
            _dev_param(21, 0)
        for dp in (1, 3):
            assert torch.equal(grids[dp][0], grids[0][0]), (cap, dp)
            assert grids[dp][1] & 5 == 0
        assert int(grids[0][0].sum()) > 0


def test_voxelgrid_front_end_normalises_in_kernel(kal):
    """r06: the front-end's kl_voxelgrid_async (vertices normalised in the kernels, grid zero-filled by
    the call) equals kl_voxelgrid_mark_async on the torch-normalised points and a zeroed grid, with
    caller origin / scale (f64 scale for f32 vertices: converted first, as the reference's tensor ops)
    and a batch of two meshes."""
    v, f = _uv_sphere(20, 32, 0.95)
    vt = torch.stack([T(v, torch.float32), T(v * 0.5 + 0.1, torch.float32)])
    ft = T(f)
    for o, sc in ((None, None), (torch.tensor([[-1., -1., -1.], [-0.2, -0.3, -0.1]], device=DEV),
                                 torch.tensor([2.0, 1.5], dtype=torch.float64, device=DEV))):
        got = kal.ops.conversions.trianglemeshes_to_voxelgrids(vt, ft, 48, o, sc)
        oo = torch.min(vt, dim=1)[0] if o is None else o
        ss = torch.max(torch.max(vt, dim=1)[0] - oo, dim=1)[0] if sc is None else sc
        pts = ((vt - oo.to(vt.dtype).unsqueeze(1)) / ss.to(vt.dtype).view(-1, 1, 1)).contiguous()
        for b in range(2):
            ref, st = _voxel_async(pts[b], ft, 48, 1 << 20)
            assert torch.equal(got[b], ref) and st == 0, b


def _voxel_host_sized(kal, v, f, R, o=None, s=None):
    from kaolin.ops.conversions import trianglemesh as tm
    tm.HOST_SIZED = True
    try:
        return kal.ops.conversions.trianglemeshes_to_voxelgrids(v, f, R, o, s)
    finally:
        tm.HOST_SIZED = False


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_voxelgrid_async_equals_host_sized_any_capacity(kal, dtype):
    """The device-counted subdivision (no host reads) marks the host-sized path's grid for every
    capacity: 0 (every triangle finished depth-first at level 0), capacities that overflow some
    level part-way, and one that holds every level."""
    v, f = _uv_sphere(20, 32, 0.95)
    vt, ft = T(v, dtype).unsqueeze(0), T(f)
    R = 64
    ref = _voxel_host_sized(kal, vt, ft, R)
    if dtype == torch.float32:
        assert np.array_equal(A(ref[0]).astype(np.uint8), orc.voxelgrid(v[None].astype(np.float32), f, R)[0])
    o = torch.min(vt, dim=1)[0]
    s = torch.max(torch.max(vt, dim=1)[0] - o, dim=1)[0]
    pts = ((vt - o.unsqueeze(1)) / s.view(-1, 1, 1))[0].contiguous()
    for cap in (0, 1, 300, 5000, 1 << 20):
        grid, status = _voxel_async(pts, ft, R, cap)
        assert torch.equal(grid, ref[0].float()), cap
        assert status & 1 == 0
        if cap == 0:
            assert status == 2  # the first level overflowed
        if cap == 1 << 20:
            assert status == 0


@pytest.mark.parametrize('grid_dtype', [torch.float64, torch.float16, torch.uint8])
def test_voxelgrid_async_grid_dtypes_and_outside_unit_cube(kal, grid_dtype):
    """An origin / scale that leaves the unit cube needs more levels than are launched: the last
    level finishes those subtrees depth-first; the grid still equals the host-sized path's."""
    v, f = _uv_sphere(6, 8, 0.95)
    vt, ft = T(v, torch.float32).unsqueeze(0), T(f)
    R = 16
    # the unit cube around the pole (0, 0.95, 0); the rest of the sphere reaches ~19: ~2 levels
    # more than are launched
    o = torch.tensor([[-0.05, 0.9, -0.05]], device=DEV)
    s = torch.tensor([0.1], device=DEV)
    ref = _voxel_host_sized(kal, vt, ft, R, o, s)
    pts = ((vt - o.unsqueeze(1)) / s.view(-1, 1, 1))[0].contiguous()
    grid, status = _voxel_async(pts, ft, R, 1 << 16, grid_dtype)
    assert status & 1 == 0
    assert torch.equal(grid.float(), ref[0].float())
    assert int(ref.sum()) > 0


def test_voxelgrid_async_budget_exceeded_raises(kal):
    """A triangle whose subtree exceeds the depth-first budget stops (all threads) and the
    eager call raises, where the host-sized path would fail its allocation."""
    v = torch.tensor([[[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]]], device=DEV)
    f = torch.tensor([[0, 1, 2]], device=DEV)
    with pytest.raises(RuntimeError, match='2\\^20'):
        kal.ops.conversions.trianglemeshes_to_voxelgrids(v, f, 8, torch.zeros((1, 3), device=DEV),
                                                         torch.tensor([1e-5], device=DEV))


def test_voxelgrid_graph_capture(kal):
    """trianglemeshes_to_voxelgrids (default origin / scale) captured into a HIP graph: nothing
    is read back, and replays over new vertices give the eager grids."""
    v, f = _uv_sphere(20, 32, 0.9)
    vt, ft = T(v, torch.float32).unsqueeze(0), T(f)
    R = 48
    static_v = vt.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kal.ops.conversions.trianglemeshes_to_voxelgrids(static_v, ft, R)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = kal.ops.conversions.trianglemeshes_to_voxelgrids(static_v, ft, R)
    for k, scale in enumerate((1.0, 0.7)):
        newv = vt * scale + 0.01 * k
        static_v.copy_(newv)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, _voxel_host_sized(kal, newv, ft, R)), k


# ------------------------------------------------------------------ SPC
def test_mesh_to_spc_kat(kal, golden):
    g = golden('spc.npz')
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(T(g['m2s_face_vertices']), int(g['m2s_level']))
    assert np.array_equal(A(octree), g['m2s_octree'])
    assert np.array_equal(A(fidx), g['m2s_face_idx'])
    np.testing.assert_allclose(A(bary), g['m2s_bary'], atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize('level', [1, 4, 6])
def test_mesh_to_spc_vs_oracle(kal, level):
    v, f = _uv_sphere(16, 24, 0.9)
    fv = v[f].astype(np.float32)
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level)
    oo, of, ob = orc.mesh_to_spc(fv, level)
    assert np.array_equal(A(octree), oo)
    assert np.array_equal(A(fidx), of)
    np.testing.assert_array_equal(A(bary), ob)


def _grazing_triangles(level, seed=3):
    """Triangles that sit on the SAT's decision boundaries at `level`: axis-aligned on voxel
    planes (box-axis ties), planes through voxel corners (normal-axis ties, x + y + z = c and
    x - y = c), near-collinear slivers and tiny triangles at corners, plus random ones."""
    rng = np.random.RandomState(seed)
    n = 2 ** level
    g = lambda k: -1.0 + 2.0 * k / n  # noqa: E731  (voxel plane k, exact in float)
    tris = []
    for _ in range(200):
        k = rng.randint(1, n)
        a, b = np.sort(rng.uniform(-1, 1, 2)), np.sort(rng.uniform(-1, 1, 2))
        ax = rng.randint(3)
        t = np.array([[g(k), a[0], b[0]], [g(k), a[1], b[0]], [g(k), a[0], b[1]]])
        tris.append(np.roll(t, ax, axis=1))
    for _ in range(200):  # plane x + y + z = corner sum
        c = g(rng.randint(0, n + 1)) + g(rng.randint(0, n + 1)) + g(rng.randint(0, n + 1))
        p = rng.uniform(-1, 1, (3, 2))
        tris.append(np.stack([p[:, 0], p[:, 1], c - p[:, 0] - p[:, 1]], 1))
    for _ in range(200):  # plane x - y = corner difference, z free
        c = g(rng.randint(0, n + 1)) - g(rng.randint(0, n + 1))
        p = rng.uniform(-1, 1, (3, 2))
        tris.append(np.stack([p[:, 0], p[:, 0] - c, p[:, 1]], 1))
    for _ in range(200):  # slivers
        a, d = rng.uniform(-0.9, 0.9, 3), rng.uniform(-0.5, 0.5, 3)
        tris.append(np.stack([a, a + d, a + d * rng.uniform(0, 1) + rng.uniform(-1, 1, 3) * 1e-6]))
    for _ in range(200):  # tiny, at a voxel corner
        c = np.array([g(rng.randint(1, n)) for _ in range(3)])
        tris.append(c + rng.uniform(-1, 1, (3, 3)) * 2.0 ** -(level + 4))
    tris.extend(rng.uniform(-1, 1, (200, 3, 3)))
    fv = np.clip(np.stack(tris), -1, 1).astype(np.float32)
    return fv


@pytest.mark.parametrize('level', [3, 5, 7])
def test_mesh_to_spc_decision_boundaries_vs_oracle(kal, level):
    """The level kernel's float pre-test (tri_voxel_maybe) only skips proposals the full fp64 SAT
    rejects: grazing, coplanar-on-a-voxel-face and sliver triangles agree with the oracle bit for bit."""
    fv = _grazing_triangles(level)
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level)
    oo, of, ob = orc.mesh_to_spc(fv, level)
    assert np.array_equal(A(octree), oo)
    assert np.array_equal(A(fidx), of)
    np.testing.assert_array_equal(A(bary), ob)


def test_mesh_to_spc_empty(kal):
    fv = torch.tensor([[[5., 5., 5.], [6., 5., 5.], [5., 6., 5.]]], device=DEV)
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(fv, 3)
    assert octree.shape == (0,) and fidx.shape == (0,) and tuple(bary.shape) == (0, 3)


@pytest.mark.parametrize('level', [10, 12, 14])
def test_mesh_to_spc_deep_levels_vs_oracle(kal, level):
    """Deep levels (nodes kept as packed 16-bit points up to 2^14 - 1; keys past the 32 bits the
    old sorted-pairs path needed): small random triangles, octree / face_idx / bary vs the oracle,
    and the fixed-capacity form equal to it."""
    rng = np.random.RandomState(level)
    c = rng.uniform(-0.9, 0.9, (24, 1, 3))
    fv = (c + rng.normal(0, 2.0 ** -(level - 5), (24, 3, 3))).astype(np.float32)
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level)
    oo, of, ob = orc.mesh_to_spc(fv, level)
    assert np.array_equal(A(octree), oo)
    assert np.array_equal(A(fidx), of)
    np.testing.assert_array_equal(A(bary), ob)
    assert _m2s_fixed_check(kal, T(fv), level, octree.shape[0], fidx.shape[0]) == 0


def _m2s_fixed_check(kal, fv, level, ncap, lcap):
    """unbatched_mesh_to_spc(..., capacity) against the eager call: the written prefix bit-equal,
    padding (0, -1, 0) after it, or status 1 with the sizes needed and nothing written."""
    octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(fv, level)
    fo, ff, fb, res = kal.ops.conversions.unbatched_mesh_to_spc(fv, level, capacity=(ncap, lcap))
    nn, nl, status = (int(x) for x in res.cpu())
    leaves = fidx.shape[0]
    nodes = octree.shape[0] if leaves else 0
    assert (nn, nl) == (nodes, leaves)
    assert fo.shape == (ncap,) and ff.shape == (lcap,) and tuple(fb.shape) == (lcap, 2)
    if nodes > ncap or leaves > lcap:
        assert status == 1
        assert not fo.any() and bool((ff == -1).all()) and not fb.any()
        return status
    assert status == 0
    assert torch.equal(fo[:nodes], octree[:nodes]) and not fo[nodes:].any()
    assert torch.equal(ff[:leaves], fidx) and bool((ff[leaves:] == -1).all())
    assert torch.equal(fb[:leaves], bary[:, :2] if leaves else fb[:0]) and not fb[leaves:].any()
    return status


@pytest.mark.devlib
@pytest.mark.parametrize('cap', [2048, 16384])
def test_mesh_to_spc_pair_overflow_fallback(kal, cap):
    """The node-rank path's pair buffers (96 pairs per face and level) overflowing -- the branch of
    r04's GPU fault.  With the capacity shrunk (dev param 14: 2048 pairs overflow at the root, 16384
    at a later level's node scan), the eager call takes the per-level fallback (kl_dev_get_stat) and
    equals the oracle; the fixed-capacity form returns status 2 with nothing written; with the
    capacity restored the node-rank path runs again and gives the same octree."""
    from dibr_util import require_dev
    from kaolin import _native as N
    lib = require_dev()
    level = 6
    v, f = _uv_sphere(16, 24, 0.9)
    fv = v[f].astype(np.float32)
    oo, of, ob = orc.mesh_to_spc(fv, level)
    N._SIZES.clear()  # workspace sizes follow the capacity
    lib.kl_dev_set_param(14, cap)
    try:
        octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level)
        torch.cuda.synchronize()
        assert lib.kl_dev_get_stat(0) == 1  # the per-level fallback ran
        assert np.array_equal(A(octree), oo) and np.array_equal(A(fidx), of)
        np.testing.assert_array_equal(A(bary), ob)
        fo, ff, fb, res = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level, capacity=(100000, 100000))
        nn, nl, status = (int(x) for x in res.cpu())
        assert (nn, nl, status) == (0, 0, 2)
        assert not fo.any() and bool((ff == -1).all()) and not fb.any()
    finally:
        lib.kl_dev_set_param(14, 0)
        N._SIZES.clear()
    octree2, fidx2, _ = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), level)
    torch.cuda.synchronize()
    assert lib.kl_dev_get_stat(0) == 0
    assert torch.equal(octree2, octree) and torch.equal(fidx2, fidx)


@pytest.mark.parametrize('level', [1, 3, 6])
def test_mesh_to_spc_fixed_capacity_equals_eager(kal, level):
    """kl_mesh_to_spc_fixed (nothing read back): exact, generous and too-small capacities on a
    sphere and on the grazing-triangle set, and the empty mesh."""
    v, f = _uv_sphere(16, 24, 0.9)
    for fv in (T(v[f].astype(np.float32)), T(_grazing_triangles(level))):
        octree, fidx, _ = kal.ops.conversions.unbatched_mesh_to_spc(fv, level)
        nodes, leaves = octree.shape[0], fidx.shape[0]
        assert _m2s_fixed_check(kal, fv, level, nodes, leaves) == 0
        assert _m2s_fixed_check(kal, fv, level, nodes + 100, leaves + 77) == 0
        assert _m2s_fixed_check(kal, fv, level, nodes - 1, leaves) == 1
        assert _m2s_fixed_check(kal, fv, level, nodes, max(leaves - 1, 0)) == 1
    empty = torch.tensor([[[5., 5., 5.], [6., 5., 5.], [5., 6., 5.]]], device=DEV)
    assert _m2s_fixed_check(kal, empty, level, 16, 16) == 0


def test_mesh_to_spc_fixed_capacity_graph_replay(kal):
    """The fixed-capacity call captured into a graph and replayed on new vertices (the same input
    buffer) answers the new mesh; the eager call refuses to be captured."""
    v, f = _uv_sphere(20, 30, 0.9)
    fv0 = T(v[f].astype(np.float32))
    buf = fv0.clone()
    cap = 40000
    for _ in range(2):  # warm-up (allocations) outside the capture
        kal.ops.conversions.unbatched_mesh_to_spc(buf, 6, capacity=cap)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = kal.ops.conversions.unbatched_mesh_to_spc(buf, 6, capacity=cap)
    for k, (scale, shift) in enumerate([(1.0, 0.0), (0.7, 0.1), (0.5, -0.3)]):
        newfv = (fv0 * scale + shift).contiguous()
        buf.copy_(newfv)
        graph.replay()
        torch.cuda.synchronize()
        octree, fidx, bary = kal.ops.conversions.unbatched_mesh_to_spc(newfv, 6)
        nn, nl, status = (int(x) for x in out[3].cpu())
        assert (nn, nl, status) == (octree.shape[0], fidx.shape[0], 0), k
        assert torch.equal(out[0][:nn], octree) and torch.equal(out[1][:nl], fidx), k
        assert torch.equal(out[2][:nl], bary), k
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match='capacity'):
        with torch.cuda.graph(g2):
            kal.ops.conversions.unbatched_mesh_to_spc(buf, 6)


def test_scan_generate_kat(kal, golden):
    g = golden('spc.npz')
    level, pyr, ex = kal.ops.spc.scan_octrees(T(g['scan_octrees']), torch.from_numpy(g['scan_lengths']))
    assert level == int(g['scan_max_level'])
    assert not pyr.is_cuda and np.array_equal(pyr.numpy(), g['scan_pyramids'])
    assert np.array_equal(A(ex), g['scan_exsum'])
    pts = kal.ops.spc.generate_points(T(g['scan_octrees']), pyr, ex)
    assert np.array_equal(A(pts), g['scan_points'])


def _rt_setup(kal, octree_np):
    octree = T(octree_np)
    level, pyr, ex = kal.ops.spc.scan_octrees(octree, torch.tensor([len(octree_np)], dtype=torch.int32))
    pts = kal.ops.spc.generate_points(octree, pyr, ex)
    return octree, pyr[0], ex, pts


@pytest.mark.parametrize('name', ['positive', 'negative', 'none', 'coarser', 'depth', 'depth_exit',
                                  'inside_nodepth', 'inside_depth', 'inside_exit'])
def test_raytrace_kat(kal, golden, name):
    g = golden('spc.npz')
    octree, pyr, ex, pts = _rt_setup(kal, g['rt_octree'])
    lv, rd, we = (int(x) for x in g[f'rt_{name}_cfg'])
    out = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(g[f'rt_{name}_origin']),
                                            T(g[f'rt_{name}_direction']), lv, return_depth=bool(rd),
                                            with_exit=bool(we))
    nug = np.stack([A(out[0]), A(out[1])], -1).reshape(-1, 2)
    assert np.array_equal(nug, g[f'rt_{name}_nuggets'])
    if rd:
        np.testing.assert_allclose(A(out[2]), g[f'rt_{name}_depth'], rtol=1e-5, atol=1e-6)


def test_raytrace_ambiguous(kal, golden):
    g = golden('spc.npz')
    octree, pyr, ex, pts = _rt_setup(kal, g['rt_ambiguous_octree'])
    r, p, d = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(g['rt_ambiguous_origin']),
                                                T(g['rt_ambiguous_direction']), 1, return_depth=True)
    assert np.array_equal(np.stack([A(r), A(p)], -1), g['rt_ambiguous_nuggets'])


def test_mark_pack_boundaries_kat(kal, golden):
    g = golden('spc.npz')
    octree, pyr, ex, pts = _rt_setup(kal, g['rt_octree'])
    r, p = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(g['rt_positive_origin']),
                                             T(g['rt_positive_direction']), 2, return_depth=False)
    assert np.array_equal(A(kal.render.spc.mark_pack_boundaries(r)), g['rt_positive_first_hits'])


@pytest.mark.parametrize('with_exit', [False, True])
def test_raytrace_vs_oracle_mesh_spc(kal, with_exit):
    v, f = _uv_sphere(24, 36, 0.8)
    fv = v[f].astype(np.float32)
    L = 6
    octree, _, _ = kal.ops.conversions.unbatched_mesh_to_spc(T(fv), L)
    octree_np = A(octree)
    octree, pyr, ex, pts = _rt_setup(kal, octree_np)
    n = 48
    ii, jj = np.meshgrid(np.linspace(-0.9, 0.9, n), np.linspace(-0.9, 0.9, n), indexing='ij')
    origin = np.stack([ii, jj, np.full_like(ii, 3.)], -1).reshape(-1, 3).astype(np.float32)
    d = np.stack([0.05 * ii, 0.03 * jj, -np.ones_like(ii)], -1).reshape(-1, 3)
    d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)
    r, p, dep = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(origin), T(d), L, return_depth=True,
                                                  with_exit=with_exit)
    onug, odep = orc.raytrace(octree_np, A(pts), pyr.numpy(), A(ex), origin, d, L, True, with_exit)
    assert np.array_equal(np.stack([A(r), A(p)], -1), onug)
    assert np.array_equal(A(dep), odep)
    assert len(onug) > 1000


@pytest.mark.parametrize('name', ['positive', 'negative', 'none', 'depth_exit', 'inside_nodepth', 'inside_exit'])
def test_raytrace_fixed_kat(kal, golden, name):
    """unbatched_raytrace(..., capacity=N) (kl_raytrace_fixed): the KAT rows, then padding."""
    g = golden('spc.npz')
    octree, pyr, ex, pts = _rt_setup(kal, g['rt_octree'])
    lv, rd, we = (int(x) for x in g[f'rt_{name}_cfg'])
    ref = g[f'rt_{name}_nuggets']
    # capacity bounds every level's candidates (a hit node's children, up to 8, before their own
    # test), not only the last level's nuggets: 8 x the largest level count (oracle) + 5
    o_np, d_np = g[f'rt_{name}_origin'].astype(np.float32), g[f'rt_{name}_direction'].astype(np.float32)
    per_level = [len(orc.raytrace(g['rt_octree'], A(pts), pyr.numpy(), A(ex), o_np, d_np, lvl, False, False)[0])
                 for lvl in range(lv + 1)]
    assert per_level[-1] == len(ref)
    cap = 8 * max(per_level) + 5
    out = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(g[f'rt_{name}_origin']),
                                            T(g[f'rt_{name}_direction']), lv, return_depth=bool(rd),
                                            with_exit=bool(we), capacity=cap)
    res = A(out[-1])
    assert res.tolist() == [len(ref), 0]
    nug = np.stack([A(out[0]), A(out[1])], -1)
    assert np.array_equal(nug[:len(ref)], ref) and (nug[len(ref):] == -1).all()
    if rd:
        dep = A(out[2])
        np.testing.assert_allclose(dep[:len(ref)], g[f'rt_{name}_depth'], rtol=1e-5, atol=1e-6)
        assert (dep[len(ref):] == 0).all()


@pytest.mark.devlib
def test_raytrace_fixed_capture_and_truncation(kal):
    """The fixed-capacity march equals the host-sized one (nuggets and depth bit-equal); captured
    into a graph and replayed with new rays it answers the new rays; with a capacity below the
    intermediate levels' counts it returns the first `capacity` rows of the full answer and flags
    the truncation."""
    v, f = _uv_sphere(24, 36, 0.8)
    L = 6
    octree, _, _ = kal.ops.conversions.unbatched_mesh_to_spc(T(v[f].astype(np.float32)), L)
    octree, pyr, ex, pts = _rt_setup(kal, A(octree))

    def rays(shift):
        n = 40
        ii, jj = np.meshgrid(np.linspace(-0.9, 0.9, n) + shift, np.linspace(-0.9, 0.9, n), indexing='ij')
        o = np.stack([ii, jj, np.full_like(ii, 3.)], -1).reshape(-1, 3).astype(np.float32)
        d = np.stack([0.05 * ii, 0.03 * jj, -np.ones_like(ii)], -1).reshape(-1, 3)
        return o, (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)

    o1, d1 = rays(0.0)
    to, td = T(o1), T(d1)
    r, p, dep = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True)
    n1 = len(r)
    cap = 16 * n1 + 4096  # above every level's candidates (a hit node's untested children)
    fr, fp, fd, res = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True,
                                                        capacity=cap)
    assert A(res).tolist() == [n1, 0]
    assert torch.equal(fr[:n1], r) and torch.equal(fp[:n1], p) and torch.equal(fd[:n1], dep)
    # captured
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True, capacity=cap)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gr, gp, gd, gres = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True,
                                                             capacity=cap)
        with pytest.raises(RuntimeError, match='capacity'):
            kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True)
    o2, d2 = rays(0.05)
    to.copy_(T(o2))
    td.copy_(T(d2))
    graph.replay()
    torch.cuda.synchronize()
    r2, p2, dep2 = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True)
    n2 = len(r2)
    assert A(gres).tolist() == [n2, 0] and not (n2 == n1 and torch.equal(p2, p))
    assert torch.equal(gr[:n2], r2) and torch.equal(gp[:n2], p2) and torch.equal(gd[:n2], dep2)
    # truncated: fewer rows than the intermediate levels hold
    small = n2 // 3
    tr, tp, tdp, tres = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True,
                                                          capacity=small)
    k, flag = A(tres).tolist()
    # the kept rows are a prefix of the full answer (possibly empty: an earlier level's kept
    # candidates may all miss at the target level)
    assert flag == 1 and 0 <= k <= small
    assert torch.equal(tr[:k], r2[:k]) and torch.equal(tp[:k], p2[:k]) and torch.equal(tdp[:k], dep2[:k])
    # the default (hit-list) march truncates exactly as the per-level march does (dev param 15 = 2),
    # every row and the result, at capacities below and around the intermediate levels' counts
    for c in (small, n2 // 2, n2, 2 * n2, 4 * n2):
        got = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True, capacity=c)
        try:
            _dev_param(15, 2)
            ref = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, to, td, L, with_exit=True, capacity=c)
        finally:
            _dev_param(15, 0)
        assert all(torch.equal(x, y) for x, y in zip(got, ref)), c


@pytest.mark.devlib
@pytest.mark.parametrize('level,nrays', [(4, 1000), (6, 1000), (6, 5), (0, 64), (3, 130)])
def test_raytrace_marches_agree(kal, level, nrays):
    """The four marches of kl_raytrace, nuggets and depths (entry and exit) bit-equal to the per-level
    march (dev param 15 = 2, kl_dev_get_stat(1) == 0): the hit-list march (default, stat 4; level 0
    and lists past its buffers fall back to the per-level march, stat 5), the fused level march
    (dev param 15 = 3: one launch per level, counts on the device, one host read) and the per-ray
    depth-first march (dev param 15 = 4, stat 3), on a dense level-6 octree: level 4 fits the hit-list
    and fused buffers (16 nuggets per ray, at least 65,536), level 6 with 1,000 rays does not (~100
    nuggets per ray): both report it and the per-level march answers (stat 0 / 2).  Levels 0 and 3:
    the root alone, and ray counts that are not a multiple of the 64-ray workgroups.  The
    fixed-capacity entry's hit-list march (default) and fused march (dev param 15 = 3) against its
    per-level march (dev param 15 = 2) too."""
    from dibr_util import require_dev
    lib = require_dev()
    n_oct = sum(8 ** k for k in range(6))
    octree, pyr, ex, pts = _rt_setup(kal, np.full(n_oct, 255, np.uint8))
    rng = np.random.RandomState(level + nrays)
    o = rng.normal(size=(nrays, 3))
    o = (3.0 * o / np.linalg.norm(o, axis=1, keepdims=True)).astype(np.float32)
    d = -o + 0.3 * rng.normal(size=(nrays, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    outs, fixed = {}, {}
    for mode in (2, 0, 3, 4):
        lib.kl_dev_set_param(15, mode)
        try:
            outs[mode] = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(o), T(d), level, with_exit=True)
            torch.cuda.synchronize()
            outs[mode] += (lib.kl_dev_get_stat(1),)
            if mode in (2, 0, 3):
                fixed[mode] = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(o), T(d), level,
                                                                with_exit=True, capacity=1000 * nrays + 64)
        finally:
            lib.kl_dev_set_param(15, 0)
    (r2, p2, d2, s2), (r0, p0, d0, s0) = outs[2], outs[0]
    (r3, p3, d3, s3), (r4, p4, d4, s4) = outs[3], outs[4]
    fits = (level, nrays) != (6, 1000)
    assert s2 == 0 and s4 == 3 and s0 == (4 if level > 0 and fits else 5)
    # 2 = a level's candidates (its parents' children) exceeded the fused march's buffers
    assert s3 in (1, 2) and (s3 == 2 or len(r2) <= max(16 * nrays, 65536)) and (fits or s3 == 2)
    assert (level, nrays) != (6, 5) or s3 == 1
    for r, p, dp in ((r0, p0, d0), (r3, p3, d3), (r4, p4, d4)):
        assert torch.equal(r, r2) and torch.equal(p, p2) and torch.equal(dp, d2)
    assert len(r2) > (1000 if nrays > 5 and level >= 4 else 0)
    k = len(r2)
    for mode in (2, 0, 3):
        fr, fp, fd, fres = fixed[mode]
        assert A(fres).tolist() == [k, 0]
        assert torch.equal(fr[:k], r2) and torch.equal(fp[:k], p2) and torch.equal(fd[:k], d2)
    # without depth, and depth without exit: the default and the depth-first march against the per-level
    for kw in ({'return_depth': False}, {}):
        got = {}
        for mode in (2, 0, 4):
            lib.kl_dev_set_param(15, mode)
            try:
                got[mode] = kal.render.spc.unbatched_raytrace(octree, pts, pyr, ex, T(o), T(d), level, **kw)
            finally:
                lib.kl_dev_set_param(15, 0)
        for mode in (0, 4):
            assert len(got[mode]) == len(got[2]) and all(torch.equal(x, y) for x, y in zip(got[mode], got[2]))


@pytest.mark.parametrize('na,nb,off', [(0, 5, 0), (7, 0, 0), (3145728, 1048576, 0), (1001, 333, 0),
                                       (3145728, 1048576, 1), (4000001, 77, 2)])
def test_loss_dot2(kal, na, nb, off):
    """bench.py's fused loss helper (kl_loss_dot2) vs an fp64 torch dot; replays reuse the workspace.
    off > 0: views starting off floats into their storage (the scalar path for a misaligned pair)."""
    from kaolin import _native
    g = torch.Generator(device='cpu').manual_seed(3)
    a, ga, b, gb = (torch.rand(n + off, generator=g).to(DEV)[off:] for n in (na, na, nb, nb))
    ws = torch.zeros(_native.lib().kl_loss_dot2_workspace_bytes(), dtype=torch.uint8, device=DEV)
    ref = float(a.double() @ ga.double() + b.double() @ gb.double())
    seen = set()
    for _ in range(3):  # deterministic: the last workgroup adds the partials in block order
        out = torch.full((1,), float('nan'), device=DEV)
        _native.check(_native.lib().kl_loss_dot2(_native.ptr(a), _native.ptr(ga), na, _native.ptr(b), _native.ptr(gb),
                                                 nb, _native.ptr(ws), _native.ptr(out), _native.stream_of(a.device)),
                      'kl_loss_dot2')
        assert abs(float(out) - ref) <= 1e-6 * max(1.0, abs(ref))
        seen.add(float(out))
    assert len(seen) == 1


# ---------------------------------------------------------------- packed ray ops (§8f rank 1)
def _rand_packs(rng, n, dim, dtype, lead_gap=True):
    """n rows in random packs (lengths 1..40); with lead_gap the first rows belong to no pack."""
    b = np.zeros(n, dtype=bool)
    i = int(rng.integers(1, 5)) if lead_gap else 0
    while i < n:
        b[i] = True
        i += int(rng.integers(1, 41))
    x = (rng.random((n, dim)) * 1.5 + 0.25).astype(dtype)
    return x, b


def test_rayops_kat(kal, golden):
    g = golden('rayops.npz')
    spc = kal.render.spc
    f, bnd, tau = T(g['feats']), T(g['boundaries']), T(g['tau'])
    assert torch.equal(spc.mark_pack_boundaries(T(g['ridx'])).cpu(), torch.from_numpy(g['ridx_boundaries']))
    assert np.array_equal(A(spc.diff(f, bnd)), g['diff'])
    assert np.array_equal(A(spc.sum_reduce(f, bnd)), g['sum_reduce'])
    for op, fn in (('sum', spc.cumsum), ('prod', spc.cumprod)):
        for ex in (False, True):
            for rev in (False, True):
                key = 'cum' + op + ('_exclusive' if ex else '') + ('_reverse' if rev else '')
                assert np.array_equal(A(fn(f, bnd, exclusive=ex, reverse=rev)), g[key]), key
    feats_out, trans = spc.exponential_integration(f, tau, bnd, exclusive=False)
    assert np.allclose(A(feats_out), g['expint_feats'], atol=1e-4)
    assert np.allclose(A(trans), g['expint_transmittance'], atol=1e-4)


@pytest.mark.parametrize('dtype', [np.float32, np.float64, np.float16])
@pytest.mark.parametrize('dim', [1, 3, 32])
def test_rayops_vs_oracle(kal, dtype, dim):
    """Bit-exact vs the oracle's sequential walks, rows before the first pack included."""
    rng = np.random.default_rng(dim)
    x, b = _rand_packs(rng, 3000, dim, dtype)
    spc = kal.render.spc
    xt, bt = T(x), T(b)
    st = orc.pack_starts(b)
    for ex in (False, True):
        for rev in (False, True):
            assert np.array_equal(A(spc.cumsum(xt, bt, exclusive=ex, reverse=rev)),
                                  orc.pack_scan(x, st, ex, rev, 'sum')), (ex, rev)
            assert np.array_equal(A(spc.cumprod(xt, bt, exclusive=ex, reverse=rev)),
                                  orc.pack_scan(x, st, ex, rev, 'prod')), (ex, rev)
    assert np.array_equal(A(spc.diff(xt, bt)), orc.pack_diff(x, st))
    isum = orc.inclusive_sum(b)
    assert np.array_equal(A(kal._C.render.spc.inclusive_sum_cuda(bt.int())), isum)
    assert np.array_equal(A(spc.sum_reduce(xt, bt)), orc.sum_reduce(x, isum))


def test_rayops_edge_cases(kal):
    spc = kal.render.spc
    x = T(np.arange(12, dtype=np.float32).reshape(6, 2))
    none = T(np.zeros(6, dtype=bool))
    assert torch.equal(spc.cumsum(x, none), torch.zeros_like(x))      # no pack: at::zeros untouched
    assert torch.equal(spc.cumprod(x, none), torch.ones_like(x))      # at::ones untouched
    assert torch.equal(spc.diff(x, none), torch.zeros_like(x))
    assert spc.sum_reduce(x, none).shape == (0, 2)
    one = T(np.array([1, 0, 0, 0, 0, 0], dtype=bool))
    assert torch.equal(spc.sum_reduce(x, one), x.sum(0, keepdim=True))
    empty = torch.zeros((0, 2), device=DEV)
    eb = torch.zeros((0,), dtype=torch.bool, device=DEV)
    assert spc.cumsum(empty, eb).shape == (0, 2)
    assert spc.sum_reduce(empty, eb).shape == (0, 2)


def test_rayops_big_and_backward(kal):
    """test_rayops.py's big cases: 10000 packs x 100 rows x 32 features vs torch along dim 1."""
    spc = kal.render.spc
    g = torch.Generator(device='cpu').manual_seed(0)
    fb = torch.rand((10000, 100, 32), generator=g).to(DEV)
    bnd = torch.zeros((10000, 100), dtype=torch.bool, device=DEV)
    bnd[:, 0] = True
    bnd = bnd.reshape(-1)
    flat = fb.reshape(-1, 32)
    assert torch.allclose(spc.sum_reduce(flat, bnd), fb.sum(1), atol=1e-5)
    assert torch.allclose(spc.cumsum(flat, bnd), torch.cumsum(fb, 1).reshape(-1, 32), atol=1e-5)
    assert torch.allclose(spc.cumprod(flat, bnd), torch.cumprod(fb, 1).reshape(-1, 32), atol=1e-4)
    for fn, ref, atol in ((spc.sum_reduce, lambda t: t.sum(1), 1e-5), (spc.cumsum, lambda t: torch.cumsum(t, 1), 1e-4),
                          (spc.cumprod, lambda t: torch.cumprod(t, 1), 1e-2)):
        x = (fb + 1e-3).detach().requires_grad_(True)
        fn(x.reshape(-1, 32), bnd).sum().backward()
        g0 = x.grad.clone()
        x.grad = None
        ref(x).sum().backward()
        assert torch.allclose(g0, x.grad, atol=atol), fn.__name__


def test_rayops_error_messages(kal):
    C = kal._C.render.spc
    with pytest.raises(RuntimeError, match=r"Expected 2-dimensional tensor, but got 1-dimensional tensor for "
                                           r"argument #1 'feats' \(while checking arguments for cumsum_cuda\)"):
        C.cumsum_cuda(torch.zeros(4, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV), False, False)
    with pytest.raises(RuntimeError, match=r"argument #2 'pack_indices' to be Long"):
        C.diff_cuda(torch.zeros(4, 2, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV))
    with pytest.raises(RuntimeError, match=r"argument #1 'feats' to be one of Half, Float, Double"):
        C.cumprod_cuda(torch.zeros(4, 2, dtype=torch.int32, device=DEV), torch.zeros(1, dtype=torch.int32,
                                                                                      device=DEV), False, False)



@pytest.mark.devlib
@pytest.mark.parametrize('case', ['bench', 'adversarial', 'random_boxes', 'narrow_w'])
@pytest.mark.parametrize('K', [30, 8, 1, 64, 255])
def test_soft_mask_C_tile_path_equals_row_kernel(kal, case, K):
    """r06: the _C contract's f32 forward (dibr_soft_mask_forward_cuda) on the tile path -- the caller's
    bboxes binned, heavy rows split over waves, the (B,H,W,K) slot tensors padded with 16-byte stores
    and each hit stored at its slot -- against the per-row-wave kernel (dev param 30 = 1): mask, prob,
    idx and type bit-equal, on the bench mesh, adversarial faces (NaN / inf / ties / huge faces),
    caller bboxes unrelated to the faces (empty, inverted, a single NaN bound: also against the
    oracle) and a width that is not a multiple of 64; knum 1 .. 255.  Also against the r06e binning / order
    preamble (dev param 31 = 1; default r06: word binning and the chip order kernel on the soft bitmap)."""
    import bench
    from dibr_util import require_dev
    require_dev()
    m, sig = 1000., 7000.
    if case == 'adversarial':
        z, v, f = _adversarial_faces(torch.float32)
        fvz, fvi, feat = T(z), T(v), T(f)
        H, W = 97, 130
        _, sel = kal.render.mesh.rasterize(H, W, fvz, fvi, feat)
    else:
        H, W = (96, 128) if case != 'narrow_w' else (40, 70)
        inp = bench.dibr_inputs([0.3, 2.0], DEV, H=H, W=W)
        fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
        _, sel = kal.render.mesh.rasterize(H, W, fvz, fvi, feat, fnz >= 0)
    fm = (fvi * m).contiguous()
    bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
    if case == 'random_boxes':
        g = torch.Generator().manual_seed(5)
        rb = (torch.rand(bb.shape, generator=g) * 2400 - 1200).to(DEV)
        pick = (torch.rand(bb.shape[:2], generator=g) < 0.05).to(DEV)
        bb = torch.where(pick[..., None], rb, bb)
        bb[0, 7, 1] = float('nan')
        bb[1, 11, 2] = float('nan')
        bb = bb.contiguous()
    tile = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, sig, K, m)
    others = []
    try:
        _dev_param(30, 1)
        others.append(kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, sig, K, m))
        _dev_param(30, 0)
        # r06: the r06e preamble (atomic binning, bucket and one-workgroup order kernels: 31 = 1)
        for combo in ({31: 1},):
            for i, v in combo.items():
                _dev_param(i, v)
            others.append(kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, sig, K, m))
            for i in combo:
                _dev_param(i, 0)
    finally:
        for i in (30, 31):
            _dev_param(i, 0)
    for other in others:
        for n, x, y in zip(['mask', 'prob', 'idx', 'type'], tile, other):
            assert x.shape == y.shape and np.array_equal(A(x), A(y), equal_nan=True), n
    assert (A(tile[2]) >= 0).any()
    if case == 'random_boxes':  # single NaN bounds: the reference's per-comparison rule (the oracle)
        om, op, oi, ot = orc.dibr_soft_mask_forward(A(fm), A(bb), A(sel), sig, K, m)
        assert np.array_equal(A(tile[2]), oi) and np.array_equal(A(tile[3]), ot)
        np.testing.assert_allclose(A(tile[1]), op, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(A(tile[0]), om, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('K', [30, 4])
def test_soft_mask_C_bench_mesh_vs_oracle(kal, K):
    """The _C contract forward at the bench mesh's heavy pole tiles (the tile path, r06): slot tensors
    equal to the oracle's (probabilities and mask to expf ulps), and its backward on them."""
    import bench
    inp = bench.dibr_inputs([0.3, 2.0], DEV, H=96, W=128)
    fvz, fvi, feat, fnz = inp['fvz'], inp['fvi'], inp['feat'], inp['fnz']
    _, sel = kal.render.mesh.rasterize(96, 128, fvz, fvi, feat, fnz >= 0)
    fm = (fvi * 1000.).contiguous()
    bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
    mask, prob, cidx, ctype = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, sel, 7000., K, 1000.)
    om, op, oi, ot = orc.dibr_soft_mask_forward(A(fm), A(bb), A(sel), 7000., K, 1000.)
    assert np.array_equal(A(cidx), oi) and np.array_equal(A(ctype), ot)
    np.testing.assert_allclose(A(prob), op, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(A(mask), om, rtol=1e-6, atol=1e-7)
    assert (oi >= 0).sum() > (10000 if K == 30 else 2000)
    grad = torch.rand_like(mask)
    gi = kal._C.render.mesh.dibr_soft_mask_backward_cuda(grad, mask, sel, prob, cidx, ctype, fm, 7000., 1000.)
    ogi = orc.dibr_soft_mask_backward(A(grad), A(mask), A(sel), A(prob), oi, ot, A(fm), 7000., 1000.)
    assert_grads_equal(A(gi), ogi)
