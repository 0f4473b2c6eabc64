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
