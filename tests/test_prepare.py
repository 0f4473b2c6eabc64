"""prepare_vertices (render/mesh/utils.py:128-175) -- the fused DIB-R input preparation
(csrc/prepare.hip).

A floating-point path: the forward is compared with the oracle's float64 restatement
(oracle.prepare_vertices) and the gradients with torch autograd through the reference's
chain of ops in float64 on the CPU.  Tolerances: f64 1e-12 (forward) / 1e-11 (gradients)
relative to the output's scale; f32: the error against the float64 reference at most twice
that of the reference's own f32 chain run with torch on the GPU (or 1e-6 of the scale) -- the
f32 normals of small faces lose digits to cancellation in either implementation.
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as orc

DEV = 'cuda'


def _ref_chain(vertices, faces, proj, rot=None, trans=None, xf=None):
    """The reference's ops (utils.py:160-175, legacy.py:35-37,136-138, mesh.py:44-46,
    trianglemesh.py:328-334) in torch, for autograd in float64."""
    if xf is None:
        vc = torch.matmul(vertices - trans.view(-1, 1, 3), rot.permute(0, 2, 1))
    else:
        vc = torch.nn.functional.pad(vertices, (0, 1), mode='constant', value=1.) @ xf
    pp = vc * proj.view(-1, 1, 3)
    vi = pp[:, :, :2] / pp[:, :, 2:3]

    def gather(x):
        inp = x.unsqueeze(2).expand(-1, -1, faces.shape[-1], -1)
        idx = faces[None, ..., None].expand(x.shape[0], -1, -1, x.shape[-1])
        return torch.gather(inp, 1, idx)
    fvc, fvi = gather(vc), gather(vi)
    n = torch.cross(fvc[:, :, 1] - fvc[:, :, 0], fvc[:, :, 2] - fvc[:, :, 0], dim=2)
    fn = n / (n.norm(dim=2, keepdim=True) + 1e-10)
    return fvc, fvi, fn


def _scene(B, Bv, seed=0, n_lat=24, n_lon=40):
    g = torch.Generator().manual_seed(seed)
    lat = torch.linspace(0, math.pi, n_lat + 1, dtype=torch.float64)[1:-1]
    lon = torch.arange(n_lon, dtype=torch.float64) * (2 * math.pi / n_lon)
    ring = torch.stack([torch.sin(lat)[:, None] * torch.cos(lon)[None], torch.cos(lat)[:, None].expand(-1, n_lon),
                        torch.sin(lat)[:, None] * torch.sin(lon)[None]], -1).reshape(-1, 3)
    verts = torch.cat([torch.tensor([[0., 1., 0.]], dtype=torch.float64), ring,
                       torch.tensor([[0., -1., 0.]], dtype=torch.float64)])
    faces = []
    for j in range(n_lon):
        faces.append([0, 1 + (j + 1) % n_lon, 1 + j])
    for i in range(n_lat - 2):
        for j in range(n_lon):
            a, b = 1 + i * n_lon + j, 1 + i * n_lon + (j + 1) % n_lon
            faces += [[a, b, b + n_lon], [a, b + n_lon, a + n_lon]]
    last = verts.shape[0] - 1
    for j in range(n_lon):
        faces.append([1 + (n_lat - 2) * n_lon + j, 1 + (n_lat - 2) * n_lon + (j + 1) % n_lon, last])
    faces = torch.tensor(faces, dtype=torch.long)
    verts = verts[None] * 0.8 + 0.05 * torch.rand((Bv,) + verts.shape, generator=g, dtype=torch.float64)
    ang = torch.rand(B, generator=g, dtype=torch.float64) * 2 * math.pi
    pos = torch.stack([3 * torch.sin(ang), 0.5 + torch.rand(B, generator=g, dtype=torch.float64),
                       3 * torch.cos(ang)], 1)
    fwd = -pos / pos.norm(dim=1, keepdim=True)
    up = torch.tensor([[0., 1., 0.]], dtype=torch.float64).expand(B, 3)
    right = torch.cross(fwd, up, dim=1)
    right = right / right.norm(dim=1, keepdim=True)
    tup = torch.cross(right, fwd, dim=1)
    rot = torch.stack([right, tup, -fwd], 1)
    proj = torch.tensor([[1.0 / math.tan(0.4)], [1.0 / math.tan(0.4)], [-1.0]], dtype=torch.float64)
    return verts, faces, proj, rot, pos


def _close(a, b, rel):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item()
    assert err <= rel * scale, f'max abs err {err} > {rel} x {scale}'


def _close_as_torch(ours, torch32, ref64, floor=1e-6):
    """f32: the error against the float64 reference is at most twice the reference's own f32
    chain's (torch ops on the GPU), or `floor` of the output's scale."""
    ref64 = ref64.detach().cpu().double()
    scale = max(ref64.abs().max().item(), 1e-30)
    e_ours = (ours.detach().cpu().double() - ref64).abs().max().item()
    e_torch = (torch32.detach().cpu().double() - ref64).abs().max().item()
    assert e_ours <= max(2 * e_torch, floor * scale), (e_ours, e_torch, scale)


def test_cpu_path_matches_oracle():
    """CPU tensors take the reference's torch chain (as the reference does on every device)."""
    import kaolin as kal
    verts, faces, proj, rot, trans = _scene(3, 3, seed=1, n_lat=6, n_lon=8)
    out = kal.render.mesh.prepare_vertices(verts, faces, proj, rot, trans)
    ref = orc.prepare_vertices(verts.numpy(), faces.numpy(), proj.numpy(), rot.numpy(), trans.numpy())
    for o, r in zip(out, ref):
        np.testing.assert_allclose(o.numpy(), r, rtol=1e-12, atol=1e-12)
    xf = torch.cat([rot.transpose(1, 2), -(trans[:, None] @ rot.transpose(1, 2))], 1)
    out2 = kal.render.mesh.prepare_vertices(verts, faces, proj, camera_transform=xf)
    ref2 = orc.prepare_vertices(verts.numpy(), faces.numpy(), proj.numpy(), camera_transform=xf.numpy())
    for o, r in zip(out2, ref2):
        np.testing.assert_allclose(o.numpy(), r, rtol=1e-12, atol=1e-12)


def test_oracle_known_answer():
    """Identity camera at the origin looking down -z: hand-computed values."""
    v = np.array([[[0., 0., -2.], [1., 0., -2.], [0., 1., -4.]]])
    f = np.array([[0, 1, 2]])
    fvc, fvi, fn = orc.prepare_vertices(v, f, np.array([[2.], [2.], [-1.]]), np.eye(3)[None], np.zeros((1, 3)))
    np.testing.assert_array_equal(fvc[0, 0], v[0])
    np.testing.assert_allclose(fvi[0, 0], [[0., 0.], [1., 0.], [0., 0.5]])
    n = np.cross([1., 0., 0.], [0., 1., -2.])
    np.testing.assert_allclose(fn[0, 0], n / (np.linalg.norm(n) + 1e-10))


CASES = [  # (B, Bv, camera mode, proj batch)
    (4, 4, 'rt', 1),
    (4, 1, 'rt', 1),
    (3, 3, 'xf', 1),
    (5, 1, 'xf', 5),
]


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('B,Bv,mode,Bp', CASES)
def test_forward_backward_vs_reference(B, Bv, mode, Bp, dtype):
    import kaolin as kal
    verts, faces, proj, rot, trans = _scene(B, Bv, seed=B + Bv)
    xf = torch.cat([rot.transpose(1, 2), -(trans[:, None] @ rot.transpose(1, 2))], 1) if mode == 'xf' else None
    if Bp > 1:
        proj = proj.reshape(1, 3).repeat(Bp, 1) * (1 + 0.1 * torch.arange(Bp, dtype=torch.float64))[:, None]
    leaves = {'v': verts, 'p': proj}
    if mode == 'rt':
        leaves.update(r=rot, t=trans)
    else:
        leaves.update(x=xf)
    # reference: float64 autograd on the CPU, from the values rounded to `dtype`
    ref_in = {k: v.to(dtype).double().clone().requires_grad_(True) for k, v in leaves.items()}
    ref = _ref_chain(ref_in['v'], faces, ref_in['p'], ref_in.get('r'), ref_in.get('t'), ref_in.get('x'))
    g = torch.Generator().manual_seed(7)
    grads = [torch.rand(r.shape, generator=g, dtype=torch.float64) - 0.5 for r in ref]
    torch.autograd.backward(ref, grads)
    orc_out = orc.prepare_vertices(ref_in['v'].detach().numpy(), faces.numpy(), ref_in['p'].detach().numpy(),
                                   None if 'r' not in ref_in else ref_in['r'].detach().numpy(),
                                   None if 't' not in ref_in else ref_in['t'].detach().numpy(),
                                   None if 'x' not in ref_in else ref_in['x'].detach().numpy())
    gpu_in = {k: v.detach().to(dtype).to(DEV).clone().requires_grad_(True) for k, v in leaves.items()}
    out = kal.render.mesh.prepare_vertices(gpu_in['v'], faces.to(DEV), gpu_in['p'], gpu_in.get('r'), gpu_in.get('t'),
                                           gpu_in.get('x'))
    # the HIP node: the Python one or the compiled one (csrc/torch_ops.cpp), never the torch chain
    assert out[0].grad_fn is not None and ('PrepareVerticesHip' in type(out[0].grad_fn).__name__
                                           or 'PrepareVertices>' in out[0].grad_fn.name())
    torch.autograd.backward(out, [x.to(dtype).to(DEV) for x in grads])
    if dtype == torch.float32:
        # the reference's own f32 chain on the GPU (torch ops) -- the f32 bar is its error
        t32 = {k: v.detach().to(dtype).to(DEV).clone().requires_grad_(True) for k, v in leaves.items()}
        tout = _ref_chain(t32['v'], faces.to(DEV), t32['p'], t32.get('r'), t32.get('t'), t32.get('x'))
        torch.autograd.backward(tout, [x.to(dtype).to(DEV) for x in grads])
    for i, (o, r, ro) in enumerate(zip(out, ref, orc_out)):
        assert o.dtype == dtype and o.shape == r.shape
        if dtype == torch.float64:
            _close(o, r, 1e-12)
            _close(o, torch.from_numpy(ro), 1e-12)
        else:
            _close_as_torch(o, tout[i], r)
            _close_as_torch(o, tout[i], torch.from_numpy(ro))
    for k in leaves:
        assert gpu_in[k].grad is not None and gpu_in[k].grad.shape == gpu_in[k].shape, k
        if dtype == torch.float64:
            _close(gpu_in[k].grad, ref_in[k].grad, 1e-11)
        else:
            _close_as_torch(gpu_in[k].grad, t32[k].grad, ref_in[k].grad)


@pytest.mark.gpu
def test_partial_grads_and_missing_outputs():
    """Only the vertices require grad; only the normals feed the loss; then only the image."""
    import kaolin as kal
    verts, faces, proj, rot, trans = _scene(2, 2, seed=3)
    for which in (2, 1, 0):
        vd = verts.to(DEV).requires_grad_(True)
        out = kal.render.mesh.prepare_vertices(vd, faces.to(DEV), proj.to(DEV), rot.to(DEV), trans.to(DEV))
        out[which].sum().backward()
        vr = verts.clone().requires_grad_(True)
        ref = _ref_chain(vr, faces, proj, rot, trans)
        ref[which].sum().backward()
        _close(vd.grad, vr.grad, 1e-11)


@pytest.mark.gpu
def test_out_of_range_face_index():
    """The front-end raises torch.gather's error (index_vertices_by_faces) once per faces
    tensor; the kernel itself, called past that check, gives NaN rows, never a fault."""
    import kaolin as kal
    from kaolin.render.mesh.utils import PrepareVerticesHip
    verts, faces, proj, rot, trans = _scene(2, 2, seed=4, n_lat=6, n_lon=8)
    bad = faces.clone()
    bad[3, 1] = verts.shape[1] + 100
    bad[5, 0] = -1
    args = [t.float().to(DEV) for t in (verts, proj, rot, trans)]
    with pytest.raises(RuntimeError, match='out of bounds for dimension 1'):
        kal.render.mesh.prepare_vertices(args[0], bad.to(DEV), *args[1:])
    hi = faces.clone()
    hi[0, 0] = verts.shape[1]
    with pytest.raises(RuntimeError, match=f'index {verts.shape[1]} is out of bounds'):
        kal.render.mesh.prepare_vertices(args[0], hi.to(DEV), *args[1:])
    fvc, fvi, fn = PrepareVerticesHip.apply(args[0], bad.to(DEV), args[1], args[2], args[3], None, (2, 2, 2, 1))
    assert torch.isnan(fvc[:, 3]).all() and torch.isnan(fvc[:, 5]).all()
    good = torch.ones(faces.shape[0], dtype=torch.bool)
    good[[3, 5]] = False
    assert torch.isfinite(fvc[:, good]).all() and torch.isfinite(fn[:, good]).all()
    # a valid faces tensor passes, and is not re-read on the next call
    f_ok = faces.to(DEV)
    kal.render.mesh.prepare_vertices(args[0], f_ok, *args[1:])
    kal.render.mesh.prepare_vertices(args[0], f_ok, *args[1:])


@pytest.mark.gpu
def test_batch_one_vertices_and_camera_with_batched_projection():
    """Bv == Bc == 1 < Bp: torch gives face_vertices_camera and face_normals a batch of 1 and
    face_vertices_image a batch of Bp; the front-end returns the same shapes and gradients."""
    import kaolin as kal
    verts, faces, proj, rot, trans = _scene(1, 1, seed=9)
    proj = proj.reshape(1, 3).repeat(4, 1) * (1 + 0.1 * torch.arange(4, dtype=torch.float64))[:, None]
    leaves = [t.to(DEV).requires_grad_(True) for t in (verts, proj, rot, trans)]
    out = kal.render.mesh.prepare_vertices(leaves[0], faces.to(DEV), *leaves[1:])
    ref_in = [t.clone().requires_grad_(True) for t in (verts, proj, rot, trans)]
    ref = _ref_chain(ref_in[0], faces, *ref_in[1:])
    assert [tuple(o.shape) for o in out] == [tuple(r.shape) for r in ref]
    assert out[0].shape[0] == 1 and out[1].shape[0] == 4 and out[2].shape[0] == 1
    g = torch.Generator().manual_seed(3)
    grads = [torch.rand(r.shape, generator=g, dtype=torch.float64) for r in ref]
    torch.autograd.backward(out, [x.to(DEV) for x in grads])
    torch.autograd.backward(ref, grads)
    for a, b in zip(leaves, ref_in):
        _close(a.grad, b.grad, 1e-11)


@pytest.mark.gpu
def test_feeds_dibr_rasterization():
    """prepare_vertices -> dibr_rasterization end to end equals the same chain with the torch
    preparation (forward bit-equal inputs are not required: the rasterizer input is compared)."""
    import kaolin as kal
    verts, faces, proj, rot, trans = _scene(2, 2, seed=5)
    args = [t.float().to(DEV) for t in (verts, proj, rot, trans)]
    fvc, fvi, fn = kal.render.mesh.prepare_vertices(args[0], faces.to(DEV), *args[1:])
    rfvc, rfvi, rfn = _ref_chain(args[0], faces.to(DEV), *args[1:])
    _close(fvi, rfvi, 2e-6)
    feats, mask, idx = kal.render.mesh.dibr_rasterization(64, 64, fvc[..., -1], fvi, torch.rand_like(fvc),
                                                          fn[..., -1])
    assert feats.shape == (2, 64, 64, 3) and (idx >= 0).any()
