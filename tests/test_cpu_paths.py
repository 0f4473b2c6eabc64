"""The reference's CPU behaviour on the drop-in front-ends (no GPU, no oracle):

* point_to_mesh_distance on CPU tensors runs the brute-force torch path
  (reference kaolin/metrics/trianglemesh.py:83-85 -> :143-268);
* trianglemeshes_to_voxelgrids is device-agnostic torch in the reference
  (ops/conversions/trianglemesh.py:29-110; its test parametrizes CPU,
  kaolin/utils/testing.py:37-38).

Both are checked bit for bit against the committed fixtures that the reference itself
produced (tests/golden/make_golden.py).
"""
import numpy as np
import pytest
import torch

import kaolin
from kaolin.metrics import trianglemesh as tm


def test_p2m_cpu_kat(golden):
    """test_trianglemesh.py:26-80 KAT (expected values typed to 4 decimals)."""
    g = golden('p2m.npz')
    d, i, t = tm._unbatched_naive_point_to_mesh_distance(torch.from_numpy(g['kat_points']),
                                                          torch.from_numpy(g['kat_face_vertices']))
    np.testing.assert_allclose(d.numpy(), g['kat_dist'], rtol=1e-12, atol=1e-12)
    assert np.array_equal(i.numpy(), g['kat_face_idx'])
    assert np.array_equal(t.numpy(), g['kat_dist_type'])


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_p2m_cpu_matches_reference_run(golden, dname):
    """1025 points x 1025 faces run through the reference's naive path with autograd:
    distances, indices, types and both gradients bit-equal."""
    g = golden('p2m.npz')
    p = torch.from_numpy(g[f'rand_{dname}_points']).requires_grad_(True)
    fv = torch.from_numpy(g[f'rand_{dname}_face_vertices']).requires_grad_(True)
    d, i, t = kaolin.metrics.trianglemesh.point_to_mesh_distance(p[None], fv[None])
    d.backward(torch.from_numpy(g[f'rand_{dname}_grad_out'])[None])
    assert np.array_equal(d[0].detach().numpy(), g[f'rand_{dname}_dist'])
    assert np.array_equal(i[0].numpy(), g[f'rand_{dname}_face_idx'])
    assert np.array_equal(t[0].numpy(), g[f'rand_{dname}_dist_type'])
    assert np.array_equal(p.grad.numpy(), g[f'rand_{dname}_grad_points'])
    assert np.array_equal(fv.grad.numpy(), g[f'rand_{dname}_grad_face_vertices'])


def test_p2m_cpu_chunking_is_invisible():
    """Point chunks of the selection pass do not change the result."""
    g = torch.Generator().manual_seed(5)
    p, fv = torch.randn((300, 3), generator=g), torch.randn((40, 3, 3), generator=g)
    i_a, t_a = tm._naive_select(p, fv)
    i_b, t_b = tm._naive_select(p, fv, chunk_elems=40 * 7)
    assert torch.equal(i_a, i_b) and torch.equal(t_a, t_b)


VOXEL_CASES = ['batched', 'origins', 'scale', 'res7', 'default_os', 'sphere32', 'random24']


@pytest.mark.parametrize('name', VOXEL_CASES)
@pytest.mark.parametrize('return_sparse', [False, True])
def test_voxelgrid_cpu_matches_reference(golden, name, return_sparse):
    """ops/conversions/test_trianglemesh.py KATs and reference-run meshes: the occupied set."""
    g = golden('voxelgrid.npz')
    v, f = torch.from_numpy(g[f'{name}_vertices']), torch.from_numpy(g[f'{name}_faces'])
    o = torch.from_numpy(g[f'{name}_origin']) if f'{name}_origin' in g.files else None
    s = torch.from_numpy(g[f'{name}_scale']) if f'{name}_scale' in g.files else None
    grid = kaolin.ops.conversions.trianglemeshes_to_voxelgrids(v, f, int(g[f'{name}_resolution']), o, s,
                                                               return_sparse=return_sparse)
    if return_sparse:
        assert grid.is_sparse
        grid = grid.to_dense()
    assert grid.dtype == v.dtype and grid.shape == (v.shape[0],) + (int(g[f'{name}_resolution']),) * 3
    occ = torch.nonzero(grid).numpy().astype(np.int32)
    assert np.array_equal(occ, g[f'{name}_occupied'])
    assert torch.all(grid[grid != 0] == 1)


def test_voxelgrid_cpu_f64():
    v = torch.tensor([[[0., 0., 0.], [1., 0., 0.], [0., 0., 1.]]], dtype=torch.float64)
    grid = kaolin.ops.conversions.trianglemeshes_to_voxelgrids(v, torch.tensor([[0, 1, 2]]), 3,
                                                               torch.zeros((1, 3), dtype=torch.float64),
                                                               torch.ones(1, dtype=torch.float64))
    assert grid.dtype == torch.float64
    # trianglemesh.py:69-81 docstring example
    expected = torch.tensor([[[1., 1., 1.], [0., 0., 0.], [0., 0., 0.]], [[1., 1., 0.], [0., 0., 0.], [0., 0., 0.]],
                             [[1., 0., 0.], [0., 0., 0.], [0., 0., 0.]]], dtype=torch.float64)
    assert torch.equal(grid[0], expected)


def _distinct_faces(g, nv, nf):
    """faces with three distinct vertices each (no zero-area face: its unit normal's second
    derivative is NaN in the reference too)"""
    return torch.stack([torch.randperm(nv, generator=g)[:3] for _ in range(nf)])


def test_compiled_reference_chains_match_python():
    """The compiled nodes' double-backward chains (csrc/torch_ops.cpp *_chain, ATen) are the
    reference's torch chains (the Python front-ends' fallbacks) op for op: outputs, first and
    second derivatives bit-equal on CPU tensors.  grid_sample's backward has no derivative in
    torch, so texture_mapping's second derivative raises in both."""
    from kaolin import _ext
    e = _ext.get()
    if e is None:
        pytest.skip('compiled extension not built')
    from kaolin.metrics.render import _mask_iou_torch
    from kaolin.render.mesh.utils import _prepare_vertices_torch, _texture_mapping_torch
    g = torch.Generator().manual_seed(0)

    def derivs(f, inputs, second=True):
        xs = [x.clone().requires_grad_(True) for x in inputs]
        ys = f(*xs)
        ys = list(ys) if isinstance(ys, (list, tuple)) else [ys]
        loss = sum((y * (k + 1.5)).sum() for k, y in enumerate(ys))
        d1 = torch.autograd.grad(loss, xs, create_graph=True, allow_unused=True)
        out = [y.detach() for y in ys] + [d.detach() for d in d1 if d is not None]
        if second:
            out += [d for d in torch.autograd.grad(sum((d * d).sum() for d in d1 if d is not None), xs,
                                                   allow_unused=True) if d is not None]
        return out

    def check(f1, f2, inputs, second=True):
        a, b = derivs(f1, inputs, second), derivs(f2, inputs, second)
        assert len(a) == len(b)
        for x, y in zip(a, b):
            assert torch.equal(x, y)

    a, b = torch.rand((2, 8, 8), generator=g), torch.rand((2, 8, 8), generator=g)
    check(e._mask_iou_chain, _mask_iou_torch, [a, b])
    v = torch.rand((2, 30, 3), generator=g)
    f = _distinct_faces(g, 30, 40)
    proj = torch.tensor([[1.8], [1.8], [-1.]])
    rot = torch.linalg.qr(torch.randn((2, 3, 3), generator=g))[0]
    trans = torch.tensor([[0., 0., 3.], [0.1, 0., 3.2]])
    xf = torch.randn((2, 4, 3), generator=g)
    check(lambda *x: e._prepare_chain(x[0], f, x[1], x[2], x[3], None),
          lambda *x: _prepare_vertices_torch(x[0], f, x[1], x[2], x[3], None), [v, proj, rot, trans])
    check(lambda *x: e._prepare_chain(x[0], f, x[1], None, None, x[2]),
          lambda *x: _prepare_vertices_torch(x[0], f, x[1], None, None, x[2]), [v, proj, xf])
    uv, tex = torch.rand((2, 5, 7, 2), generator=g), torch.rand((2, 3, 16, 16), generator=g)
    for mode, code in (('bilinear', 1), ('nearest', 0)):
        f1 = lambda c, t: e._texture_chain(c, t, code)  # noqa: E731
        f2 = lambda c, t: _texture_mapping_torch(c, t, mode).reshape(2, -1, 3)  # noqa: E731
        check(f1, f2, [uv, tex], second=False)
        for fn in (f1, f2):
            with pytest.raises(RuntimeError, match='grid_sampler_2d_backward is not implemented'):
                derivs(fn, [uv, tex])
