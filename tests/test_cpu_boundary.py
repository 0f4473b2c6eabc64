"""CPU-only checks of the drop-in boundary: the C-ABI library loads and exports every
symbol include/kaolin_hip.h declares, the _C registry has the reference's layout, the
argument checks reproduce the reference's messages, and CPU tensors fail loudly."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, 'include', 'kaolin_hip.h')).read()
    return sorted(set(re.findall(r'^\s*(?:const\s+char\s*\*\s*|int\s+|size_t\s+)(kl_\w+)\s*\(', hdr, re.M)))


def test_library_exports_every_declared_symbol():
    from kaolin import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f'{s} declared in include/kaolin_hip.h but not exported'
    assert set(syms) == set(_native.exported_symbols())


def test_abi_version_and_error_channel():
    from kaolin import _native
    lib = _native.lib()
    assert lib.kl_abi_version() == 4
    # a dtype the rasterizer does not implement reports through kl_last_error (no GPU work)
    rc = lib.kl_packed_rasterize_forward(7, 4, 4, 1, 0, 1, 1, None, None, None, None, None, 1.0, 1e-8,
                                         None, None, None, None, 0, None)
    assert rc == -1
    assert b'not implemented' in lib.kl_last_error()


def test_workspace_sizes():
    from kaolin import _native
    lib = _native.lib()
    # rasterizer visibility buffer: 8 B key + 4 B index + 1 B flag per pixel, + big-face queue
    P = 4 * 512 * 512
    assert lib.kl_rasterize_workspace_bytes(4, 512, 512, 50000) == 13 * P + (4 * 50000 + 1) * 4
    # soft-mask bins: 8x64 tiles of 64x8 px, ceil(ceil(50000/64)/32) = 25 words, + f64 bboxes
    # + the tile-order sort buffers + f64 bboxes
    assert lib.kl_soft_mask_workspace_bytes(4, 512, 512, 50000) >= 4 * 8 * 64 * 25 * 4 + 4 * 50000 * 4 * 8


def test_C_registry_layout():
    import kaolin
    C = kaolin._C
    for path in ['render.mesh.packed_rasterize_forward_cuda', 'render.mesh.rasterize_backward_cuda',
                 'render.mesh.dibr_soft_mask_forward_cuda', 'render.mesh.dibr_soft_mask_backward_cuda',
                 'metrics.sided_distance_forward_cuda', 'metrics.sided_distance_backward_cuda',
                 'metrics.unbatched_triangle_distance_forward_cuda',
                 'metrics.unbatched_triangle_distance_backward_cuda', 'ops.conversions.mesh_to_spc_cuda',
                 'ops.spc.morton_to_octree', 'ops.spc.scan_octrees_cuda', 'ops.spc.generate_points_cuda',
                 'render.spc.raytrace_cuda', 'render.spc.mark_pack_boundaries_cuda', 'render.spc.diff_cuda',
                 'render.spc.inclusive_sum_cuda', 'render.spc.sum_reduce_cuda', 'render.spc.cumsum_cuda',
                 'render.spc.cumprod_cuda', 'render.spc.generate_primary_rays_cuda',
                 'render.spc.generate_shadow_rays_cuda', 'render.spc.raytrace_fixed_cuda',
                 'ops.conversions.mesh_to_spc_fixed_cuda']:
        obj = C
        for part in path.split('.'):
            obj = getattr(obj, part)
        assert callable(obj)


def test_check_messages():
    from kaolin._checks import Arg, check_size, check_same_type
    with pytest.raises(RuntimeError, match=r"Expected tensor of size \[3, 3, 3\], but got tensor of size "
                                           r"\[2, 3, 3\] for argument #2 'p2' \(while checking arguments for "
                                           r"sided_distance_forward_cuda\)"):
        check_size('sided_distance_forward_cuda', Arg(torch.zeros(2, 3, 3), 'p2', 2), (3, 3, 3))
    with pytest.raises(RuntimeError, match=r"Expected 3-dimensional tensor, but got 4-dimensional tensor for "
                                           r"argument #1 'p1' \(while checking arguments for "
                                           r"sided_distance_forward_cuda\)"):
        check_size('sided_distance_forward_cuda', Arg(torch.zeros(3, 2, 3, 4), 'p1', 1), (3, 2, 3))
    with pytest.raises(RuntimeError, match='to have the same type'):
        check_same_type('f', Arg(torch.zeros(1), 'a', 1), Arg(torch.zeros(1, dtype=torch.double), 'b', 2))


def test_cpu_tensors_fail_loudly():
    import kaolin
    with pytest.raises(RuntimeError, match='on CPU'):
        kaolin.metrics.pointcloud.sided_distance(torch.rand(1, 4, 3), torch.rand(1, 5, 3))
    with pytest.raises(RuntimeError):
        kaolin.render.mesh.rasterize(8, 8, torch.rand(1, 2, 3), torch.rand(1, 2, 3, 2), torch.rand(1, 2, 3, 1))
    with pytest.raises(RuntimeError, match='on CPU'):
        kaolin.ops.spc.points_to_morton(torch.zeros(4, 3, dtype=torch.int16))
    with pytest.raises(RuntimeError, match='on CPU'):
        kaolin.ops.spc.morton_to_points(torch.zeros(4, dtype=torch.long))
    bnd = torch.tensor([True, False, True])
    for fn in (kaolin.render.spc.cumsum, kaolin.render.spc.cumprod, kaolin.render.spc.sum_reduce,
               kaolin.render.spc.diff):
        with pytest.raises(RuntimeError, match='on CPU'):
            fn(torch.rand(3, 2), bnd)


def test_voxelgrid_resolution_type():
    import kaolin
    with pytest.raises(TypeError, match=r"Expected resolution to be int but got .*"):
        kaolin.ops.conversions.trianglemeshes_to_voxelgrids(torch.rand(1, 3, 3), torch.tensor([[0, 1, 2]]), 2.3)
