"""check_sign (reference ops/mesh/check_sign.py:25-154, test_check_sign.py).

CPU: the numpy oracle (oracle/oracle.py, mesh_intersection_counts / check_sign) against the
reference's known answers (test_check_sign.py:26-186: points overlapping vertices and edges in
projection, in front of / behind the mesh, zero-area faces), transcribed in
tests/golden/check_sign.npz.  Argument errors of the front-end (no device needed).

GPU: kaolin.ops.mesh.check_sign (one batched launch) and
kaolin._C.ops.mesh.unbatched_mesh_intersection_cuda against the oracle, bit-exact (integer
crossing counts), and inside/outside of a closed sphere at a size the oracle does not reach.
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as orc


@pytest.mark.parametrize('dtype', [np.float32, np.float64])
@pytest.mark.parametrize('zero_area', [False, True])
def test_oracle_kat(golden, dtype, zero_area):
    g = golden('check_sign.npz')
    faces = np.concatenate([g['faces'], g['zero_area_faces']]) if zero_area else g['faces']
    out = orc.check_sign(g['verts'].astype(dtype), faces, g['points'].astype(dtype))
    np.testing.assert_array_equal(out, g['expected'])


@pytest.fixture(scope='module')
def kal():
    import kaolin
    return kaolin


@pytest.mark.parametrize('mutate,exc,msg', [
    (lambda v, f, p: (v, f.int(), p), TypeError, r'Expected faces entries to be torch.int64 but got torch.int32.'),
    (lambda v, f, p: (v.unsqueeze(-1), f, p), ValueError, r'Expected verts to have 3 dimensions but got 4 dimensions.'),
    (lambda v, f, p: (v, f.unsqueeze(-1), p), ValueError, r'Expected faces to have 2 dimensions but got 3 dimensions.'),
    (lambda v, f, p: (v, f, p.unsqueeze(-1)), ValueError,
     r'Expected points to have 3 dimensions but got 4 dimensions.'),
    (lambda v, f, p: (v[..., :2], f, p), ValueError, r'Expected verts to have 3 coordinates but got 2 coordinates.'),
    (lambda v, f, p: (v, f[:, :2], p), ValueError, r'Expected faces to have 3 vertices but got 2 vertices.'),
    (lambda v, f, p: (v, f, p[..., :2]), ValueError, r'Expected points to have 3 coordinates but got 2 coordinates.'),
])
def test_argument_errors(kal, golden, mutate, exc, msg):
    g = golden('check_sign.npz')
    v, f, p = torch.from_numpy(g['verts']), torch.from_numpy(g['faces']), torch.from_numpy(g['points'])
    with pytest.raises(exc, match=msg):
        kal.ops.mesh.check_sign(*mutate(v, f, p))
    with pytest.raises(TypeError, match=r"Expected hash_resolution to be int but got <class 'float'>."):
        kal.ops.mesh.check_sign(v, f, p, 512.0)


def test_cpu_tensors_raise(kal, golden):
    g = golden('check_sign.npz')
    with pytest.raises(RuntimeError, match='CPU fallback|GPU tensors'):
        kal.ops.mesh.check_sign(torch.from_numpy(g['verts']), torch.from_numpy(g['faces']),
                                torch.from_numpy(g['points']))


# ------------------------------------------------------------------------------- GPU parity
DEV = 'cuda'


def _T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _uv_sphere(n_lat, n_lon, radius=1.0):
    lat = np.linspace(0, math.pi, n_lat + 1)[1:-1]
    lon = np.arange(n_lon) * (2 * math.pi / n_lon)
    ring = np.stack([np.sin(lat)[:, None] * np.cos(lon)[None], np.cos(lat)[:, None] * np.ones_like(lon)[None],
                     np.sin(lat)[:, None] * np.sin(lon)[None]], -1).reshape(-1, 3)
    verts = np.concatenate([[[0, 1, 0]], ring, [[0, -1, 0]]]) * radius
    faces = []
    R = len(lat)
    for j in range(n_lon):
        j1 = (j + 1) % n_lon
        faces.append([0, 1 + j1, 1 + j])
        faces.append([1 + (R - 1) * n_lon + j, 1 + (R - 1) * n_lon + j1, len(verts) - 1])
        for i in range(R - 1):
            a, b = 1 + i * n_lon + j, 1 + i * n_lon + j1
            c, d = a + n_lon, b + n_lon
            faces += [[a, b, d], [a, d, c]]
    return verts, np.array(faces, np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('zero_area', [False, True])
def test_gpu_kat(kal, golden, dtype, zero_area):
    g = golden('check_sign.npz')
    faces = np.concatenate([g['faces'], g['zero_area_faces']]) if zero_area else g['faces']
    out = kal.ops.mesh.check_sign(_T(g['verts']).to(dtype), _T(faces), _T(g['points']).to(dtype))
    assert out.dtype == torch.bool
    np.testing.assert_array_equal(out.cpu().numpy(), g['expected'])
    out1 = kal.ops.mesh.check_sign(_T(g['verts'][:1]).to(dtype), _T(faces), _T(g['points'][:1]).to(dtype))
    np.testing.assert_array_equal(out1.cpu().numpy(), g['expected'][:1])


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_gpu_vs_oracle(kal, dtype):
    """Grid points on the sphere's own vertex coordinates (vertex / edge overlaps in projection)
    plus random points; raw _C counts and the batched front-end, both bit-exact."""
    verts, faces = _uv_sphere(12, 18, 0.8)
    verts = verts.astype(dtype)
    rng = np.random.default_rng(3)
    grid = np.stack(np.meshgrid(np.linspace(-1, 1, 9), verts[:40:3, 1], verts[:40:5, 2]), -1).reshape(-1, 3)
    pts = np.concatenate([grid, rng.uniform(-1, 1, (700, 3))]).astype(dtype)
    v1, v2, v3 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    cnt = kal._C.ops.mesh.unbatched_mesh_intersection_cuda(_T(pts), _T(v1), _T(v2), _T(v3))
    assert cnt.dtype == torch.from_numpy(pts).dtype and cnt.shape == (len(pts),)
    ref = orc.mesh_intersection_counts(pts, v1, v2, v3)
    np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.int64), ref)
    B = 2
    vb = np.stack([verts, verts * dtype(1.5) + dtype(0.1)])
    pb = np.stack([pts, pts * dtype(1.2)])
    out = kal.ops.mesh.check_sign(_T(vb), _T(faces), _T(pb))
    np.testing.assert_array_equal(out.cpu().numpy(), orc.check_sign(vb, faces, pb))
    assert out.shape == (B, len(pts))


@pytest.mark.gpu
def test_gpu_sphere_inside_property(kal):
    """20k-face sphere, 200k points: inside <=> |p| < r away from the surface."""
    verts, faces = _uv_sphere(101, 100, 1.0)
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1.3, 1.3, (1, 200000, 3)).astype(np.float32)
    out = kal.ops.mesh.check_sign(_T(verts[None].astype(np.float32)), _T(faces), _T(pts)).cpu().numpy()[0]
    r = np.linalg.norm(pts[0], axis=-1)
    far = np.abs(r - 1.0) > 0.01  # the tessellation is within 1e-3 of the sphere
    np.testing.assert_array_equal(out[far], (r < 1.0)[far])
    assert out[far].sum() > 10000


def _dev_flags(kal, flags):
    from dibr_util import dev_flags
    dev_flags(flags)


@pytest.mark.devlib
@pytest.mark.gpu
def test_gpu_list_total_coarsens_grid(kal):
    """The (y, z) cell lists' total is counted in 64 bits; past the int32 scan's range the grid
    is coarsened (here forced with a 2^10 test cap, dev flag 1 << 24).  Large faces spanning the
    whole box plus the sphere: counts still bit-exact."""
    verts, faces = _uv_sphere(12, 18, 0.8)
    big = np.array([[-2., -1., -1.], [2., 1.1, -0.9], [0.5, -0.9, 1.2], [0.1, 1., 1.]])
    verts = np.concatenate([verts, big]).astype(np.float32)
    n = len(verts) - 4
    faces = np.concatenate([faces, np.array([[n, n + 1, n + 2], [n + 1, n + 2, n + 3]] * 20)])
    pts = np.random.default_rng(5).uniform(-1, 1, (3000, 3)).astype(np.float32)
    v1, v2, v3 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    ref = orc.mesh_intersection_counts(pts, v1, v2, v3)
    _dev_flags(kal, 1 << 24)
    try:
        cnt = kal._C.ops.mesh.unbatched_mesh_intersection_cuda(_T(pts), _T(v1), _T(v2), _T(v3))
        out = kal.ops.mesh.check_sign(_T(verts[None]), _T(faces), _T(pts[None]))
    finally:
        _dev_flags(kal, 0)
    np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.int64), ref)
    np.testing.assert_array_equal(out.cpu().numpy(), orc.check_sign(verts[None], faces, pts[None]))


@pytest.mark.gpu
@pytest.mark.parametrize('bad', [-1, 10 ** 6])
def test_gpu_face_index_out_of_range_raises(kal, bad):
    """The reference's index_select raises on an index outside the vertices; so does the batched
    kernel (a device flag read back with the list total), instead of reading out of bounds."""
    verts, faces = _uv_sphere(6, 8, 0.8)
    faces = faces.copy()
    faces[3, 1] = bad
    pts = np.zeros((1, 10, 3), np.float32)
    with pytest.raises(RuntimeError, match='index out of range'):
        kal.ops.mesh.check_sign(_T(verts[None].astype(np.float32)), _T(faces), _T(pts))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_gpu_batch_nan_and_outside_points(kal, dtype):
    """maxlen taken on the device (check_sign.py:140-146, NaN propagated as torch's max / min):
    a NaN vertex that no face uses still makes its mesh's maxlen NaN (every point outside);
    NaN points, points outside the face box, duplicated points (one cell gets many) and a point
    count that is not a multiple of the workgroup -- every answer as the oracle's."""
    verts, faces = _uv_sphere(10, 14, 0.7)
    verts = np.concatenate([verts, np.zeros((1, 3))]).astype(dtype)
    rng = np.random.default_rng(11)
    P = 1237
    pts = rng.uniform(-1.5, 1.5, (3, P, 3)).astype(dtype)
    pts[0, :50] = np.nan
    pts[1, 100:400] = pts[1, 99]
    pts[2, :30, 1] = np.inf
    vb = np.stack([verts, verts * dtype(0.5), verts + dtype(0.2)])
    vb[1, -1, 2] = np.nan
    out = kal.ops.mesh.check_sign(_T(vb), _T(faces), _T(pts)).cpu().numpy()
    ref = orc.check_sign(vb, faces, pts)
    np.testing.assert_array_equal(out, ref)
    assert not out[1].any() and out[0].any() and out[2].any()


def _captured(fn):
    """fn() captured into a HIP graph (warmed up eagerly first) and replayed once."""
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    g.replay()
    torch.cuda.synchronize()
    return g, out


@pytest.mark.devlib
@pytest.mark.gpu
@pytest.mark.parametrize('overflow', [False, True])
def test_gpu_graph_capture(kal, overflow):
    """Under graph capture the entries take their capturable form (no allocator, nothing read
    back: the lists live in the workspace's fixed room).  Past that room (forced here with dev
    flag 1 << 26) cs_brute_kernel answers every point against every face on the device.  Both
    bit-exact to the oracle, and a replay after the inputs change answers the new inputs."""
    verts, faces = _uv_sphere(12, 18, 0.8)
    verts = verts.astype(np.float32)
    rng = np.random.default_rng(7)
    pts = rng.uniform(-1, 1, (2, 1500, 3)).astype(np.float32)
    vb = np.stack([verts, verts * np.float32(1.3)])
    tv, tf, tp = _T(vb), _T(faces), _T(pts)
    v1, v2, v3 = (_T(verts[faces[:, k]]) for k in range(3))
    _dev_flags(kal, (1 << 26) if overflow else 0)
    try:
        g, (out, cnt) = _captured(lambda: (kal.ops.mesh.check_sign(tv, tf, tp),
                                           kal._C.ops.mesh.unbatched_mesh_intersection_cuda(tp[0], v1, v2, v3)))
        np.testing.assert_array_equal(out.cpu().numpy(), orc.check_sign(vb, faces, pts))
        np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.int64),
                                      orc.mesh_intersection_counts(pts[0], verts[faces[:, 0]], verts[faces[:, 1]],
                                                                   verts[faces[:, 2]]))
        pts2 = rng.uniform(-1, 1, pts.shape).astype(np.float32)
        tp.copy_(_T(pts2))
        g.replay()
        torch.cuda.synchronize()
    finally:
        _dev_flags(kal, 0)
    np.testing.assert_array_equal(out.cpu().numpy(), orc.check_sign(vb, faces, pts2))
