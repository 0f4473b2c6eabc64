"""The §8e sharded paths' per-rank halves on the GPU, emulated in one process (the gloo tests in
test_distributed_cpu.py cover the collectives on CPU tensors, where the GPU kernels do not run).

Each test splits the work the way kaolin.distributed does on N ranks, runs every shard's GPU half,
combines the shards as the collective would (concatenation for all-gathers, a float64 sum for the
all-reduce of double sums, OR for the bit grids) and compares with the unsharded GPU op.
"""
import numpy as np
import pytest
import torch

from dibr_util import assert_grads_equal

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module')
def kal():
    import kaolin
    return kaolin


@pytest.mark.parametrize('world', [2, 3])
def test_p2m_sharded_backward_sums_equal_unsharded(kal, world):
    """sharded_point_to_mesh_distance's backward: every rank's double face sums
    (distributed._p2m_face_sums, kl_unbatched_triangle_distance_backward_sums), added in float64 and
    rounded once, give the unsharded GPU face gradient; each shard's point gradient is the
    unsharded rows (the exact path had never run with more than one shard)."""
    from kaolin.distributed import _p2m_face_sums, shard_bounds
    g = torch.Generator().manual_seed(0)
    pts = torch.randn((20000, 3), generator=g).to(DEV)
    fv = torch.randn((2000, 3, 3), generator=g).to(DEV)
    gd = torch.rand((20000,), generator=g).to(DEV)
    p = pts.clone().requires_grad_(True)
    f = fv.clone().requires_grad_(True)
    d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(p.unsqueeze(0), f.unsqueeze(0))
    d.backward(gd.unsqueeze(0))
    total = torch.zeros((2000, 3, 3), dtype=torch.float64, device=DEV)
    for r in range(world):
        lo, hi = shard_bounds(20000, r, world)
        gp, sums = _p2m_face_sums(gd[lo:hi], pts[lo:hi].contiguous(), fv, i[0, lo:hi], t[0, lo:hi])
        assert torch.equal(gp, p.grad[lo:hi]), r
        total += sums
    assert_grads_equal(total.float().cpu().numpy(), f.grad.cpu().numpy())


@pytest.mark.parametrize('world', [2, 3])
def test_sided_sharded_backward_sums_equal_unsharded(kal, world):
    """sharded_sided_distance's backward: the ranks' grad_p2 double sums
    (kl_sided_distance_backward_sums), added and rounded once, equal the unsharded GPU backward
    (which rounds its own double sum: deterministic from run to run)."""
    from kaolin import _C
    from kaolin.distributed import shard_bounds
    g = torch.Generator().manual_seed(1)
    p1 = torch.rand((2, 5000, 3), generator=g).to(DEV)
    p2 = torch.rand((2, 700, 3), generator=g).to(DEV)
    gd = torch.rand((2, 5000), generator=g).to(DEV)
    grads = []
    for _ in range(2):
        a, b = p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)
        d, idx = kal.metrics.pointcloud.sided_distance(a, b)
        d.backward(gd)
        grads.append((a.grad, b.grad))
    assert torch.equal(grads[0][1], grads[1][1])  # deterministic grad_p2
    total = torch.zeros((2, 700, 3), dtype=torch.float64, device=DEV)
    for r in range(world):
        lo, hi = shard_bounds(5000, r, world)
        g1, sums = _C.sided_distance_backward_sums(gd[:, lo:hi].contiguous(), p1[:, lo:hi].contiguous(), p2,
                                                   idx[:, lo:hi].contiguous())
        assert torch.equal(g1, grads[0][0][:, lo:hi]), r
        total += sums
    assert_grads_equal(total.float().cpu().numpy(), grads[0][1].cpu().numpy())


def test_sided_backward_vs_oracle_f64_sums(kal):
    """The double-sum grad_p2 against the oracle's (float64 inputs, 1e-12)."""
    from oracle import oracle as orc
    g = torch.Generator().manual_seed(2)
    p1 = torch.rand((1, 3000, 3), generator=g, dtype=torch.float64)
    p2 = torch.rand((1, 400, 3), generator=g, dtype=torch.float64)
    gd = torch.rand((1, 3000), generator=g, dtype=torch.float64)
    a, b = p1.to(DEV).requires_grad_(True), p2.to(DEV).requires_grad_(True)
    d, idx = kal.metrics.pointcloud.sided_distance(a, b)
    d.backward(gd.to(DEV))
    og1, og2 = orc.sided_distance_backward(gd.numpy(), p1.numpy(), p2.numpy(), idx.cpu().numpy())
    assert np.array_equal(a.grad.cpu().numpy(), og1)
    np.testing.assert_allclose(b.grad.cpu().numpy(), og2, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('world', [2, 3])
def test_voxelgrid_face_split_bit_grids(kal, world):
    """sharded_trianglemeshes_to_voxelgrids' face split: the OR of the shards' bit grids
    (R^3 / 8 bytes) unpacks to the unsharded dense grid (GPU, R = 64 and a non-multiple-of-8 R)."""
    from kaolin.distributed import _pack_bits, _unpack_bits, shard_bounds
    from kaolin.ops.conversions import trianglemeshes_to_voxelgrids
    g = torch.Generator().manual_seed(3)
    verts = torch.rand((1, 300, 3), generator=g).to(DEV)
    faces = torch.randint(0, 300, (500, 3), generator=g).to(DEV)
    origin = torch.min(verts, dim=1)[0]
    scale = torch.max(torch.max(verts, dim=1)[0] - origin, dim=1)[0]
    for R in (64, 37):
        full = trianglemeshes_to_voxelgrids(verts, faces, R, origin, scale)
        bits = None
        for r in range(world):
            lo, hi = shard_bounds(500, r, world)
            b = _pack_bits(trianglemeshes_to_voxelgrids(verts, faces[lo:hi], R, origin, scale))
            bits = b if bits is None else bits | b
        assert bits.numel() == -(-R ** 3 // 8)
        assert torch.equal(_unpack_bits(bits, full), full)
