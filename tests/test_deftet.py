"""deftet_sparse_render (reference render/mesh/deftet.py:269-417, test_deftet.py).

CPU tests pin the numpy oracle (oracle/oracle.py, deftet_*) against the reference's own
known answers (the simple case of test_deftet.py:36-230, transcribed in tests/golden/deftet.npz)
and against the reference's `_naive_deftet_sparse_render` run on the model.obj case of
test_deftet.py:335-551 (fixtures made by tests/golden/make_golden.py).  The naive oracle
orders by depth before truncating to knum and uses a strict lower range bound, the kernel
truncates in mesh order with `lo <= d`; the fixtures hold fewer than knum hits per pixel and
no depth on a bound, so both agree there.

GPU tests run the HIP path through kaolin.render.mesh.deftet_sparse_render and
kaolin._C.render.mesh.deftet_sparse_render_{forward,backward}_cuda and compare with the
oracle: face indices, depths, weights, features and gradients bit-exact (same operation order,
no contraction; the backward sums each face's items in item order, as the oracle does).  The
atomic fallback of the ABI (no workspace) is checked to 1e-5.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc


# ---------------------------------------------------------------------------- oracle pinning
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
@pytest.mark.parametrize('case', ['full', 'restricted'])
def test_oracle_simple_kat(golden, dtype, case):
    g = golden('deftet.npz')
    fvi, fvz = g['simple_fvi'].astype(dtype), g['simple_fvz'].astype(dtype)
    feat = np.concatenate([g['simple_feat_face'], g['simple_feat_vert']], -1).astype(dtype)
    pix = g['simple_pix'].astype(dtype)
    lo = -4. if case == 'full' else -2.1
    ranges = np.tile(np.array([lo, 0.], dtype), (2, 7, 1))
    interp, sidx, _ = orc.deftet_sparse_render(pix, ranges, fvz, fvi, feat, 5)
    gt_idx = g[f'simple_{case}_idx']
    np.testing.assert_array_equal(sidx, gt_idx)
    gt0 = (gt_idx + np.arange(2).reshape(2, 1, 1) * 3).astype(dtype)
    gt0[gt_idx == -1] = 0
    np.testing.assert_allclose(interp[..., 0], gt0, atol=1e-6)
    np.testing.assert_allclose(interp[..., 1], g[f'simple_{case}_feat_vert'], atol=3e-3, rtol=1e-5)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('up', [0, 1])
def test_oracle_vs_reference_naive(golden, dname, up):
    g = golden('deftet.npz')
    fvz, fvi, fuv, pix = (g[f'{dname}_{k}'] for k in ('fvz', 'fvi', 'fuv', 'pix'))
    q = f'{dname}_up{up}_'
    K = g[q + 'face_idx'].shape[-1]
    interp, sidx, weights = orc.deftet_sparse_render(pix, g[q + 'ranges'], fvz, fvi, fuv, K)
    np.testing.assert_array_equal(sidx, g[q + 'face_idx'])
    assert (sidx >= 0).any()
    # the naive renderer re-derives the weights in the k1/k3 form with a double eps, the kernel in
    # the cross-product form with a float eps: ~1e-5 relative apart on small faces; the reference
    # test's own tolerance (test_deftet.py:430-432) is 1e-4
    np.testing.assert_allclose(interp, g[q + 'features'], rtol=1e-4, atol=1e-4)
    g_img, g_feat = orc.deftet_sparse_render_backward(g[q + 'grad_out'], sidx, weights, fvi, fuv)
    # the reference test's own tolerances (test_deftet.py:493-496)
    np.testing.assert_allclose(g_img, g[q + 'grad_fvi'], rtol=5e-3, atol=5e-3)
    np.testing.assert_allclose(g_feat, g[q + 'grad_fuv'], rtol=1e-3, atol=1e-3)


def test_oracle_knum_truncates_in_mesh_order():
    """Kernel semantics (deftet_cuda.cu fwd): with more hits than knum, the FIRST knum faces in
    mesh order are kept (then sorted by depth), not the closest knum."""
    fvi = np.tile(np.array([[[-1., -1.], [1., -1.], [-1., 1.]]]), (1, 4, 1, 1))
    fvz = np.array([[[-4.] * 3, [-1.] * 3, [-3.] * 3, [-2.] * 3]])
    pix = np.array([[[-0.5, -0.5]]])
    ranges = np.array([[[-10., 0.]]])
    feat = np.arange(4.).reshape(1, 4, 1, 1).repeat(3, 2)
    _, sidx, _ = orc.deftet_sparse_render(pix, ranges, fvz, fvi, feat, 2)
    np.testing.assert_array_equal(sidx, [[[0, 1][::-1]]])


# ------------------------------------------------------------------------------- GPU parity
DEV = 'cuda'


def _T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _A(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope='module')
def kal():
    import kaolin
    return kaolin


def _grid_case(dtype, B=2, F=3000, H=48, W=40, seed=0, knum=12):
    """Random overlapping triangles (DefTet's volumetric use: many layers per pixel) rendered
    on an image grid, some pixels with more hits than knum."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (B, F, 1, 2))
    fvi = (c + rng.normal(0, 0.15, (B, F, 3, 2))).astype(dtype)
    fvz = rng.uniform(-3, -1, (B, F, 3)).astype(dtype)
    x = (2 * np.arange(W) + 1 - W) / W
    y = (H - 2 * np.arange(H) - 1.) / H
    pix = np.stack(np.meshgrid(x, y), -1).reshape(1, -1, 2).repeat(B, 0).astype(dtype)
    ranges = np.tile(np.array([-2.6, -1.2], dtype), (B, H * W, 1))
    feat = rng.uniform(-1, 1, (B, F, 3, 4)).astype(dtype)
    return pix, ranges, fvz, fvi, feat, knum


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_gpu_forward_cuda_raw_vs_oracle(kal, dtype):
    """_C.render.mesh.deftet_sparse_render_forward_cuda: unsorted mesh-order slots, bit-exact."""
    pix, ranges, fvz, fvi, feat, K = _grid_case(dtype, F=2000, H=24, W=20)
    bboxes = np.concatenate([fvi.min(2), fvi.max(2)], -1)
    out = kal._C.render.mesh.deftet_sparse_render_forward_cuda(_T(fvz), _T(fvi), _T(bboxes), _T(pix), _T(ranges),
                                                               K, 1e-8)
    torch.cuda.synchronize()
    ref = orc.deftet_sparse_render_forward(fvz, fvi, bboxes, pix, ranges, K, 1e-8)
    assert isinstance(out, list) and len(out) == 4
    np.testing.assert_array_equal(_A(out[0]), ref[0])
    assert (ref[0][..., -1] >= 0).any(), 'case must saturate knum somewhere'
    for a, b in zip(out[1:], ref[1:]):
        np.testing.assert_array_equal(_A(a), b)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_gpu_render_fwd_bwd_vs_oracle(kal, dtype):
    pix, ranges, fvz, fvi, feat, K = _grid_case(dtype)
    fvi_t = _T(fvi).requires_grad_(True)
    feat_t = _T(feat).requires_grad_(True)
    interp, idx = kal.render.mesh.deftet_sparse_render(_T(pix), _T(ranges), _T(fvz), fvi_t, feat_t, K)
    r_interp, r_idx, r_w = orc.deftet_sparse_render(pix, ranges, fvz, fvi, feat, K)
    np.testing.assert_array_equal(_A(idx), r_idx)
    np.testing.assert_array_equal(_A(interp), r_interp)
    grad = np.random.default_rng(5).uniform(0, 1, interp.shape).astype(dtype)
    interp.backward(_T(grad))
    g_img, g_feat = orc.deftet_sparse_render_backward(grad, r_idx, r_w, fvi, feat)
    # the gather backward sums each face's items in item order, as the oracle: bit-exact
    np.testing.assert_array_equal(_A(fvi_t.grad), g_img)
    np.testing.assert_array_equal(_A(feat_t.grad), g_feat)


@pytest.mark.gpu
def test_gpu_backward_atomic_fallback(kal):
    """Without a workspace the ABI falls back to the reference's float atomics (rounding-level)."""
    import ctypes
    from kaolin import _native as N
    pix, ranges, fvz, fvi, feat, K = _grid_case(np.float32, F=1500, H=20, W=24)
    r_interp, r_idx, r_w = orc.deftet_sparse_render(pix, ranges, fvz, fvi, feat, K)
    grad = np.random.default_rng(6).uniform(0, 1, r_interp.shape).astype(np.float32)
    B, P, _, D = grad.shape
    F = fvi.shape[1]
    g_img = torch.empty(fvi.shape, device=DEV)
    g_feat = torch.empty(feat.shape, device=DEV)
    gt, it, wt, ft, fet = _T(grad), _T(r_idx), _T(r_w), _T(fvi), _T(feat)
    N.check(N.lib().kl_deftet_sparse_render_backward(
        N.KL_F32, B, F, P, K, D, N.ptr(gt), N.ptr(it), N.ptr(wt), N.ptr(ft), N.ptr(fet), 1e-8, N.ptr(g_img),
        N.ptr(g_feat), None, 0, N.stream_of(torch.device(DEV))), 'deftet bwd')
    torch.cuda.synchronize()
    e_img, e_feat = orc.deftet_sparse_render_backward(grad, r_idx, r_w, fvi, feat)
    np.testing.assert_allclose(_A(g_img), e_img, rtol=1e-5, atol=1e-5 * max(np.abs(e_img).max(), 1.0))
    np.testing.assert_allclose(_A(g_feat), e_feat, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('up', [0, 1])
@pytest.mark.parametrize('as_list', [False, True])
def test_gpu_model_obj_vs_reference(kal, golden, dname, up, as_list):
    """test_deftet.py:420-551 on the committed fixtures (reference naive renderer)."""
    g = golden('deftet.npz')
    fvz, fvi, fuv, pix = (g[f'{dname}_{k}'] for k in ('fvz', 'fvi', 'fuv', 'pix'))
    q = f'{dname}_up{up}_'
    K = g[q + 'face_idx'].shape[-1]
    fvi_t = _T(fvi).requires_grad_(True)
    fuv_t = _T(fuv).requires_grad_(True)
    mask_t = torch.ones_like(fuv_t[..., :1], requires_grad=True)
    feats = [fuv_t, mask_t] if as_list else fuv_t
    interp, idx = kal.render.mesh.deftet_sparse_render(_T(pix), _T(g[q + 'ranges']), _T(fvz), fvi_t, feats, K)
    np.testing.assert_array_equal(_A(idx), g[q + 'face_idx'])
    uv = interp[0] if as_list else interp
    np.testing.assert_allclose(_A(uv), g[q + 'features'], rtol=1e-4, atol=1e-4)
    grad = _T(g[q + 'grad_out'])
    if as_list:
        torch.autograd.backward([interp[0], interp[1]], [grad, torch.zeros_like(interp[1])])
    else:
        interp.backward(grad)
    np.testing.assert_allclose(_A(fvi_t.grad), g[q + 'grad_fvi'], rtol=5e-3, atol=5e-3)
    np.testing.assert_allclose(_A(fuv_t.grad), g[q + 'grad_fuv'], rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_gpu_simple_kat(kal, golden, dtype):
    g = golden('deftet.npz')
    fvi, fvz = _T(g['simple_fvi']).to(dtype), _T(g['simple_fvz']).to(dtype)
    ff, fv = _T(g['simple_feat_face']).to(dtype), _T(g['simple_feat_vert']).to(dtype)
    pix = _T(g['simple_pix']).to(dtype)
    for case, lo in (('full', -4.), ('restricted', -2.1)):
        ranges = torch.tensor([[[lo, 0.]]], dtype=dtype, device=DEV).repeat(2, 7, 1)
        (f0, f1), idx = kal.render.mesh.deftet_sparse_render(pix, ranges, fvz, fvi, [ff, fv], 5)
        gt_idx = g[f'simple_{case}_idx']
        np.testing.assert_array_equal(_A(idx), gt_idx)
        gt0 = (gt_idx + np.arange(2).reshape(2, 1, 1) * 3).astype(np.float64)
        gt0[gt_idx == -1] = 0
        np.testing.assert_allclose(_A(f0)[..., 0], gt0, atol=1e-6)
        np.testing.assert_allclose(_A(f1)[..., 0], g[f'simple_{case}_feat_vert'], atol=3e-3, rtol=1e-5)


@pytest.mark.gpu
def test_gpu_edge_cases(kal):
    dt = torch.float32
    # no pixels, no faces, knum larger than any hit count
    fvz = torch.zeros((1, 0, 3), dtype=dt, device=DEV)
    fvi = torch.zeros((1, 0, 3, 2), dtype=dt, device=DEV)
    feat = torch.zeros((1, 0, 3, 2), dtype=dt, device=DEV)
    pix = torch.zeros((1, 5, 2), dtype=dt, device=DEV)
    rr = torch.tensor([[[-1., 0.]]], dtype=dt, device=DEV).repeat(1, 5, 1)
    f, i = kal.render.mesh.deftet_sparse_render(pix, rr, fvz, fvi, feat, 3)
    assert f.shape == (1, 5, 3, 2) and bool((i == -1).all()) and bool((f == 0).all())
    pix0 = torch.zeros((1, 0, 2), dtype=dt, device=DEV)
    f, i = kal.render.mesh.deftet_sparse_render(pix0, rr[:, :0], fvz, fvi, feat, 3)
    assert f.shape == (1, 0, 3, 2) and i.shape == (1, 0, 3)
    # the raw entry point reports the reference's argument names on a bad size
    with pytest.raises(RuntimeError, match='face_bboxes'):
        kal._C.render.mesh.deftet_sparse_render_forward_cuda(
            fvz, fvi, torch.zeros((1, 1, 4), dtype=dt, device=DEV), pix, rr, 3, 1e-8)
    with pytest.raises(RuntimeError, match='CPU fallback|GPU tensors'):
        kal.render.mesh.deftet_sparse_render(pix.cpu(), rr.cpu(), fvz.cpu(), fvi.cpu(), feat.cpu(), 3)


@pytest.mark.gpu
@pytest.mark.parametrize('knum', [1, 7, 300])
def test_gpu_knum_paths(kal, knum):
    """knum <= 256 takes the slot-parallel resolve, the default 300 the per-pixel one; both vs oracle."""
    pix, ranges, fvz, fvi, feat, _ = _grid_case(np.float32, B=1, F=600, H=12, W=10, seed=4)
    interp, idx = kal.render.mesh.deftet_sparse_render(_T(pix), _T(ranges), _T(fvz), _T(fvi), _T(feat), knum)
    r_interp, r_idx, _ = orc.deftet_sparse_render(pix, ranges, fvz, fvi, feat, knum)
    np.testing.assert_array_equal(_A(idx), r_idx)
    np.testing.assert_array_equal(_A(interp), r_interp)


@pytest.mark.gpu
@pytest.mark.parametrize('binned', [False, True])
def test_gpu_walk_quotient_underflow_edge(kal, binned):
    """Barycentric quotients at the underflow edge: face 0's first quotient at pixel 0 underflows to
    -0, a hit under the reference's `w >= 0`; face 1's is a tiny negative normal (a miss); faces 2-3
    are plain.  Both forwards, f64, vs the oracle (r06: guards any shortcut taken before the
    divisions, like the sign pre-test measured in DESIGN.md §3.6)."""
    dt = np.float64
    fvi = np.zeros((1, 4, 3, 2), dt)
    fvi[0, 0] = [[1e180, -1e180], [1e-150, 0.], [0., -1e-150]]
    fvi[0, 1] = [[1e20, -1e20], [1e-150, 0.], [0., -1e-150]]
    fvi[0, 2] = [[0.5, 0.5], [0.9, 0.5], [0.5, 0.9]]
    fvi[0, 3] = [[-0.5, -0.5], [0.5, -0.5], [0., 0.5]]
    fvz = np.full((1, 4, 3), -1.5, dt)
    fvz[0, 0] = [-1.4, -1.5, -1.6]
    pix = np.array([[[0., -1e-160], [0., -0.1], [0.6, 0.6]]], dt)
    ranges = np.tile(np.array([-2.6, -1.2], dt), (1, 3, 1))
    args = [_T(fvz), _T(fvi), None, _T(pix), _T(ranges), 4, 1e-8]
    out = kal._C.deftet_forward('deftet', *args, binned=binned)
    ref = orc.deftet_sparse_render_forward(fvz, fvi, None, pix, ranges, 4, 1e-8)
    assert ref[0][0, 0, 0] == 0 and np.signbit(ref[2][0, 0, 0])
    for x, r in zip(out, ref):
        np.testing.assert_array_equal(_A(x), r)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_gpu_binned_and_tile_forward_agree(kal, dtype):
    """The screen-grid forward (with an allocator) and the tile-walk forward (without) give the
    same slots, both equal to the oracle; includes NaN / inf faces and pixels off the mesh."""
    pix, ranges, fvz, fvi, feat, K = _grid_case(dtype, B=2, F=2500, H=30, W=26, seed=9)
    fvi = fvi.copy()
    fvi[0, 5, 1, 0] = np.nan
    fvi[1, 7, 2, 1] = np.inf
    pix = pix * dtype(1.3)  # some pixels outside every face's bbox
    args = [_T(fvz), _T(fvi), None, _T(pix), _T(ranges), K, 1e-8]
    a = kal._C.deftet_forward('deftet', *args, binned=True)
    b = kal._C.deftet_forward('deftet', *args, binned=False)
    ref = orc.deftet_sparse_render_forward(fvz, fvi, None, pix, ranges, K, 1e-8)
    for x, y, r in zip(a, b, ref):
        np.testing.assert_array_equal(_A(x), _A(y))
        np.testing.assert_array_equal(_A(x), r)


@pytest.mark.devlib
@pytest.mark.gpu
def test_gpu_binned_list_cap_falls_back_to_tile_walk(kal):
    """The screen-grid lists' total is counted in 64 bits; past the int32 scan's range the forward
    takes the tile walk (forced here with a 2^10 test cap, dev flag 1 << 24): same slots."""
    from dibr_util import require_dev
    lib = require_dev()
    pix, ranges, fvz, fvi, feat, K = _grid_case(np.float32, B=2, F=2500, H=30, W=26, seed=9)
    args = [_T(fvz), _T(fvi), None, _T(pix), _T(ranges), K, 1e-8]
    lib.kl_dev_set_flags(1 << 24)
    try:
        a = kal._C.deftet_forward('deftet', *args, binned=True)
    finally:
        lib.kl_dev_set_flags(0)
    ref = orc.deftet_sparse_render_forward(fvz, fvi, None, pix, ranges, K, 1e-8)
    for x, r in zip(a, ref):
        np.testing.assert_array_equal(_A(x), r)


@pytest.mark.devlib
@pytest.mark.gpu
@pytest.mark.parametrize('order', ['grid', 'shuffled'])
def test_gpu_tile_walk_pixel_order(kal, order):
    """With dev param 24 = 1 the tile walk visits the pixels in a spatial (Morton) order when there
    are enough of them (r05; off by default, it did not pay): the same slots either way, equal to the oracle,
    with pixels in image order or shuffled, non-finite pixels and a second view."""
    from dibr_util import require_dev
    lib = require_dev()
    pix, ranges, fvz, fvi, feat, K = _grid_case(np.float32, B=2, F=1500, H=40, W=36, seed=11)
    pix = pix.copy()
    if order == 'shuffled':
        perm = np.random.default_rng(3).permutation(pix.shape[1])
        pix, ranges = pix[:, perm], ranges[:, perm]
    pix[0, 17] = np.nan
    pix[1, 100, 0] = np.inf
    args = [_T(fvz), _T(fvi), None, _T(pix), _T(ranges), K, 1e-8]
    a = kal._C.deftet_forward('deftet', *args, binned=False)
    lib.kl_dev_set_param(24, 1)
    try:
        b = kal._C.deftet_forward('deftet', *args, binned=False)
    finally:
        lib.kl_dev_set_param(24, 0)
    ref = orc.deftet_sparse_render_forward(fvz, fvi, None, pix, ranges, K, 1e-8)
    for x, y, r in zip(a, b, ref):
        np.testing.assert_array_equal(_A(x), _A(y))
        np.testing.assert_array_equal(_A(x), r)
