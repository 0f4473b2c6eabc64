"""_C.render.spc.generate_primary_rays_cuda / generate_shadow_rays_cuda (raytrace.cpp:111-166,
234-283; raytrace_cuda.cu:764-909; deprecated upstream, bindings.cpp:86,88).

The reference has no test and no Python caller for either, so the oracle is a numpy restatement
of raytrace.cpp / raytrace_cuda.cu written here: the host matrix set-up in float32 in the
reference's operation order, the device rows in float64.  The GPU rows must be within a few
float32 ulps of it (the CUDA build's fma contraction and rsqrtf are not reproducible here:
parity unpinned beyond that tolerance); the shadow-ray count, order and ray map are exact.
"""
import numpy as np
import pytest
import torch

f32 = np.float32


def _norm32(v):
    v = v.astype(f32)
    d = f32(v[0] * v[0]) + f32(v[1] * v[1])
    d = f32(d + f32(v[2] * v[2]))
    inv = f32(f32(1) / np.sqrt(d, dtype=f32))
    return (v * inv).astype(f32)


def _crs3(a, b):
    return np.array([a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]], f32)


def _mm(a, b):
    c = np.zeros((4, 4), f32)
    for i in range(4):
        for j in range(4):
            s = f32(a[i, 0] * b[0, j])
            for k in range(1, 4):
                s = f32(s + f32(a[i, k] * b[k, j]))
            c[i, j] = s
    return c


def primary_rays_ref(height, width, eye, at, up, fov, world):
    """raytrace.cpp:128-162 + raytrace_cuda.cu:764-785."""
    W, H = f32(width), f32(height)
    ar = f32(W / H)
    th = f32(np.tan(f32(f32(0.5) * f32(fov)), dtype=f32))
    pvp = np.array([[f32(f32(f32(2) * ar) * th) / W, 0, 0, 0], [0, f32(f32(2) * th) / H, 0, 0], [0, 0, 0, 1],
                    [f32(f32(ar * th) * f32(f32(1) - W)) / W, f32(th * f32(f32(1) - H)) / H, -1, 0]], f32)
    z = _norm32(at - eye)
    x = _norm32(_crs3(z, up))
    y = _crs3(x, z)
    view = np.array([[*x, 0], [*y, 0], [*(-z), 0], [*eye, 1]], f32)
    tf = _mm(_mm(pvp, view), world.T.copy()).astype(np.float64)
    t = np.arange(height * width)
    px, py = (t % width).astype(np.float64), (t // height).astype(np.float64)
    org = np.broadcast_to(tf[2, :3], (len(t), 3))
    d = px[:, None] * tf[0, :3] + py[:, None] * tf[1, :3] + tf[3, :3]
    return org, d, tf


def shadow_rays_ref(ro, rd, light, plane):
    """raytrace.cpp:251-283 + raytrace_cuda.cu:790-909 in float64."""
    lt = 0.5 * (light.astype(np.float64) + 1.0)
    pl = np.array([2 * plane[0], 2 * plane[1], 2 * plane[2], plane[3] - plane[0] - plane[1] - plane[2]], np.float64)
    ro, rd = ro.astype(np.float64), rd.astype(np.float64)
    a = ro @ pl[:3] + pl[3]
    b = rd @ pl[:3]
    with np.errstate(divide='ignore', invalid='ignore'):
        t = -a / b
    info = (np.abs(b) > 1e-3) & (t > 0)
    cnt = int(info[:-1].sum()) if len(info) else 0  # the exclusive scan's entry at num - 1
    idx = np.nonzero(info)[0][:cnt]
    hit = ro[idx] + t[idx, None] * rd[idx]
    v = hit - lt
    return np.broadcast_to(lt, (cnt, 3)), v / np.linalg.norm(v, axis=-1, keepdims=True), idx, info


@pytest.fixture(scope='module')
def kal():
    import kaolin
    return kaolin


def test_primary_rays_argument_errors(kal):
    e, a, u, w = torch.zeros(3), torch.ones(3), torch.tensor([0., 1., 0.]), torch.eye(4)
    gen = kal._C.render.spc.generate_primary_rays_cuda
    with pytest.raises(RuntimeError, match='Eye must be a triplet'):
        gen(4, 4, torch.zeros(4), a, u, 1.0, w)
    with pytest.raises(RuntimeError, match='At must be byte'):
        gen(4, 4, e, a.double(), u, 1.0, w)
    with pytest.raises(RuntimeError, match=r'World must of size \{4, 4\}'):
        gen(4, 4, e, a, u, 1.0, torch.eye(3))
    with pytest.raises(RuntimeError, match='Up must be contiguous'):
        gen(4, 4, e, a, torch.zeros(3, 2)[:, 0], 1.0, w)


def test_shadow_rays_cpu_tensors_raise(kal):
    with pytest.raises(RuntimeError, match='GPU tensors'):
        kal._C.render.spc.generate_shadow_rays_cuda(torch.zeros(4, 3), torch.ones(4, 3), torch.zeros(3),
                                                    torch.ones(4))


def test_restatement_self_consistency():
    """The primary rays' restatement: the centre pixel's direction lies along the view axis
    (square image, identity world): the restated matrix is the pinhole camera it claims."""
    eye, at, up = np.array([0., 0., 3.], f32), np.zeros(3, f32), np.array([0., 1., 0.], f32)
    org, d, tf = primary_rays_ref(65, 65, eye, at, up, 0.7, np.eye(4, dtype=f32))
    c = d[32 * 65 + 32]
    assert abs(c[0]) < 1e-6 and abs(c[1]) < 1e-6 and c[2] < 0


@pytest.mark.gpu
@pytest.mark.parametrize('hw', [(48, 48), (32, 40), (1, 7)])
def test_primary_rays_vs_restatement(kal, hw):
    H, W = hw
    rng = np.random.default_rng(H * 100 + W)
    eye = rng.uniform(-3, 3, 3).astype(f32)
    at = rng.uniform(-0.5, 0.5, 3).astype(f32)
    up = np.array([0.1, 1.0, 0.2], f32)
    world = np.eye(4, dtype=f32)
    world[:3, :3] += rng.uniform(-0.1, 0.1, (3, 3)).astype(f32)
    world[3, :3] = rng.uniform(-0.2, 0.2, 3).astype(f32)
    org, dirs = kal._C.render.spc.generate_primary_rays_cuda(H, W, torch.from_numpy(eye), torch.from_numpy(at),
                                                             torch.from_numpy(up), 0.8, torch.from_numpy(world))
    ro, rd, tf = primary_rays_ref(H, W, eye, at, up, 0.8, world)
    assert org.shape == (H * W, 3) and org.dtype == torch.float32 and org.is_cuda
    scale = np.abs(tf).max() * max(H, W)
    np.testing.assert_allclose(org.cpu().numpy(), ro, rtol=0, atol=4e-7 * np.abs(tf).max())
    np.testing.assert_allclose(dirs.cpu().numpy(), rd, rtol=0, atol=4e-7 * scale)


@pytest.mark.gpu
def test_shadow_rays_vs_restatement(kal):
    rng = np.random.default_rng(5)
    n = 5000
    ro = rng.uniform(-1, 1, (n, 3)).astype(f32)
    rd = rng.normal(size=(n, 3)).astype(f32)
    rd[:50] = 0  # parallel to every plane: no hit
    rd[n - 1] = [0, -1, 0]  # the last ray hits; the reference's count leaves it out
    ro[n - 1] = [0, 0.5, 0]
    light = np.array([0.3, 0.9, -0.2], f32)
    plane = np.array([0.0, 1.0, 0.0, 0.4], f32)
    src, dst, mp = kal._C.render.spc.generate_shadow_rays_cuda(torch.from_numpy(ro).cuda(), torch.from_numpy(rd).cuda(),
                                                               torch.from_numpy(light), torch.from_numpy(plane))
    rsrc, rdst, ridx, info = shadow_rays_ref(ro, rd, light, plane)
    assert info[n - 1] and 100 < len(ridx) < n
    assert np.array_equal(mp.cpu().numpy(), ridx)
    np.testing.assert_array_equal(src.cpu().numpy(), rsrc.astype(f32))
    np.testing.assert_allclose(dst.cpu().numpy(), rdst, rtol=0, atol=3e-6)
    e = kal._C.render.spc.generate_shadow_rays_cuda(torch.zeros((0, 3), device='cuda'),
                                                    torch.zeros((0, 3), device='cuda'), torch.from_numpy(light),
                                                    torch.from_numpy(plane))
    assert all(t.shape[0] == 0 for t in e)
