"""Generate the committed golden fixtures under tests/golden/*.npz.

Runs ONLY in the build container, where the reference (NVIDIA Kaolin 0.14.0,
/root/reference) is importable as plain Python.  Its native module ``kaolin._C``
is not built there, so the three native modules are stubbed and
only the reference's *pure-PyTorch* code runs:

* the reference test oracles (``_naive_deftet_sparse_render``,
  ``_unbatched_naive_point_to_mesh_distance``, ``_sided_distance``,
  ``trianglemeshes_to_voxelgrids``),
* its input-preparation helpers (``io.obj.import_mesh``, legacy camera fns,
  ``index_vertices_by_faces``, ``face_normals``),
* its golden data files (``tests/samples/dibr/**.pt``, loaded with
  ``torch.load(weights_only=True)``).

Known-answer tests that live only inside the reference's test sources
(mesh_to_spc level 3, raytrace nuggets/depths, scan_octrees/generate_points,
p2m / sided KATs) are transcribed below as DATA (inputs + expected outputs).

Nothing from the reference travels to the GPU box except the .npz written here.
Usage:  python tests/golden/make_golden.py
"""
import math
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    for name in ['kaolin._C', 'kaolin.ops.conversions.mise',
                 'kaolin.ops.mesh.triangle_hash']:
        sys.modules[name] = types.ModuleType(name)
    import torch
    torch.cuda.synchronize = lambda *a, **k: None
    import warnings
    warnings.filterwarnings('ignore')
    import kaolin
    return torch, kaolin


torch, kal = _import_reference()
from kaolin.render.mesh.deftet import _naive_deftet_sparse_render  # noqa: E402
from kaolin.metrics import trianglemesh as ref_tm  # noqa: E402
from kaolin.metrics import pointcloud as ref_pc  # noqa: E402
from kaolin.ops.conversions import trianglemeshes_to_voxelgrids  # noqa: E402

SAMPLES = os.path.join(REF, 'tests', 'samples')


def _load_pt(path):
    return torch.load(path, weights_only=True, map_location='cpu')


def save(name, **arrays):
    out = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
           for k, v in arrays.items()}
    np.savez_compressed(os.path.join(HERE, name), **out)
    sz = os.path.getsize(os.path.join(HERE, name))
    print(f'wrote {name}: {len(out)} arrays, {sz/1024:.1f} KiB')


# --------------------------------------------------------------------------
# DIB-R "simple" case (tests/python/kaolin/render/mesh/test_dibr.py:36-191)
# --------------------------------------------------------------------------
def dibr_simple():
    H, W = 35, 31
    fvi = torch.tensor(
        [[[[-0.7, 0.], [0., -0.7], [0., 0.7]],
          [[-0.7, 0.], [0., 0.7], [0., -0.7]],
          [[0., -0.7], [0., 0.7], [0.7, 0.]]],
         [[[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]],
          [[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]],
          [[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]]]], dtype=torch.double)
    fvz = torch.tensor(
        [[[-2., -1., -1.], [-2.5, -3., -3.], [-2., -2., -2.]],
         [[-2., -1., -3.], [-2., -2., -2.], [-2., -3., -1.]]], dtype=torch.double)
    arrays = dict(face_vertices_image=fvi, face_vertices_z=fvz)
    # rasterize oracle (knum=1) gives selected_face_idx, as the test fixture does
    pix, ranges = _pixel_coords_ranges(fvz, H, W, vertices_z=None)
    feat = torch.zeros(fvz.shape + (1,), dtype=torch.double)
    _, idx = _naive_deftet_sparse_render(pix, ranges, fvz, fvi, feat, 1)
    arrays['selected_face_idx'] = idx.reshape(2, H, W)
    gtdir = os.path.join(SAMPLES, 'dibr', 'simple')
    arrays['new_face_idx'] = _load_pt(os.path.join(gtdir, 'new_face_idx_35_31.pt'))
    for sig in (7000, 70):
        for box in (0.02, 0.2):
            tag = f'{H}_{W}_{sig}_{box}'
            arrays[f'soft_mask_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'soft_mask_{tag}.pt')).double()
            arrays[f'close_face_idx_{sig}_{box}'] = (_load_pt(os.path.join(gtdir, f'close_face_idx_{tag}.pt')).long() - 1).short()
            arrays[f'close_face_prob_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'close_face_dist_{tag}.pt')).double()
            arrays[f'close_face_dist_type_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'close_face_dist_type_{tag}.pt')).to(torch.uint8)
            arrays[f'grad_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'grad_face_vertices_image_{tag}.pt')).double()
    save('dibr_simple.npz', **arrays)


def _pixel_coords_ranges(face_vertices_z, H, W, vertices_z=None):
    """Same pixel centres / render ranges as test_rasterization.py:115-131."""
    B = face_vertices_z.shape[0]
    dtype = face_vertices_z.dtype
    x = (2 * torch.arange(W, dtype=dtype) + 1 - W) / W
    y = (H - 2 * torch.arange(H, dtype=dtype) - 1.) / H
    pix = torch.stack([x.reshape(1, 1, -1).repeat(B, H, 1),
                       y.reshape(1, -1, 1).repeat(B, 1, W)], dim=-1).reshape(B, -1, 2)
    zsrc = face_vertices_z.reshape(B, -1) if vertices_z is None else vertices_z
    min_z = zsrc.min(dim=1)[0]
    max_z = zsrc.max(dim=1)[0]
    rr = torch.stack([min_z - 1e-2, max_z + 1e-2], dim=-1)
    return pix, rr.unsqueeze(1).repeat(1, H * W, 1)


# --------------------------------------------------------------------------
# DIB-R / rasterize "sphere" case (model.obj, 3 cameras) test_dibr.py:193-394,
# test_rasterization.py:33-232
# --------------------------------------------------------------------------
def _sphere_inputs(dtype, flip):
    mesh = kal.io.obj.import_mesh(os.path.join(SAMPLES, 'model.obj'), with_materials=True)
    faces = mesh.faces
    if flip:
        faces = torch.flip(faces, dims=(-1,))
    B = 3
    cam_pos = torch.tensor([[0.5, 0.5, 3.], [2., 2., -2.], [3., 0.5, 0.5]], dtype=dtype)
    look_at = torch.full((B, 3), 0.5, dtype=dtype)
    up = torch.tensor([[0., 1., 0.]], dtype=dtype).repeat(B, 1)
    proj = kal.render.camera.generate_perspective_projection(fovyangle=math.pi / 4., dtype=dtype)
    v = mesh.vertices.to(dtype).unsqueeze(0)
    vmin = v.min(dim=1, keepdims=True)[0]
    vmax = v.max(dim=1, keepdims=True)[0]
    v = (v - vmin) / (vmax - vmin)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(cam_pos, look_at, up)
    vcam = kal.render.camera.rotate_translate_points(v, rot, trans)
    vimg = kal.render.camera.perspective_camera(vcam, proj)
    fvcam = kal.ops.mesh.index_vertices_by_faces(vcam, faces)
    fvz = fvcam[..., -1].contiguous()
    fvi = kal.ops.mesh.index_vertices_by_faces(vimg, faces)
    fnz = kal.ops.mesh.face_normals(fvcam, unit=True)[..., -1]
    fuv_idx = mesh.face_uvs_idx
    if flip:
        fuv_idx = torch.flip(fuv_idx, dims=(-1,))
    fuv = kal.ops.mesh.index_vertices_by_faces(mesh.uvs.unsqueeze(0).to(dtype), fuv_idx).repeat(B, 1, 1, 1)
    # valid faces of test_rasterization.py:94-99
    min_z = fvz.reshape(B, -1).min(dim=1, keepdims=True)[0]
    max_z = fvz.reshape(B, -1).max(dim=1, keepdims=True)[0]
    mid = (min_z + max_z) / 2.
    valid = torch.all(fvz < mid.unsqueeze(-1), dim=-1)
    return dict(face_vertices_z=fvz, face_vertices_image=fvi, face_normals_z=fnz,
                face_uvs=fuv, valid_faces=valid, vertices_camera_z=vcam[..., -1])


def dibr_sphere():
    H, W = 35, 31
    gtdir = os.path.join(SAMPLES, 'dibr', 'sphere')
    arrays = {}
    for dname, dtype in (('f32', torch.float), ('f64', torch.double)):
        for flip in (0, 1):
            inp = _sphere_inputs(dtype, bool(flip))
            p = f'{dname}_flip{flip}_'
            for k in ('face_vertices_z', 'face_vertices_image', 'face_normals_z', 'face_uvs', 'valid_faces'):
                arrays[p + k] = inp[k]
            B = 3
            pix, rr = _pixel_coords_ranges(inp['face_vertices_z'], H, W, vertices_z=inp['vertices_camera_z'])
            for use_valid in (0, 1):
                kw = {'valid_faces': inp['valid_faces']} if use_valid else {}
                fvi = inp['face_vertices_image'].clone().requires_grad_(True)
                fuv = inp['face_uvs'].clone().requires_grad_(True)
                feats, idx = _naive_deftet_sparse_render(pix, rr, inp['face_vertices_z'], fvi, fuv, 1, **kw)
                feats = feats.reshape(B, H, W, -1)
                g = torch.Generator().manual_seed(1234 + use_valid)
                grad_out = torch.rand(feats.shape, generator=g, dtype=dtype)
                feats.backward(grad_out)
                q = p + f'valid{use_valid}_'
                arrays[q + 'features'] = feats.detach()
                arrays[q + 'face_idx'] = idx.reshape(B, H, W)
                arrays[q + 'grad_out'] = grad_out
                arrays[q + 'grad_face_vertices_image'] = fvi.grad
                arrays[q + 'grad_face_uvs'] = fuv.grad
    for sig in (7000, 70):
        for box in (0.02, 0.01):
            tag = f'{H}_{W}_{sig}_{box}'
            arrays[f'soft_mask_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'soft_mask_{tag}.pt')).double()
            arrays[f'close_face_idx_{sig}_{box}'] = (_load_pt(os.path.join(gtdir, f'close_face_idx_{tag}.pt')).long() - 1).short()
            arrays[f'close_face_prob_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'close_face_dist_{tag}.pt')).double()
            arrays[f'close_face_dist_type_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'close_face_dist_type_{tag}.pt')).to(torch.uint8)
            arrays[f'grad_{sig}_{box}'] = _load_pt(os.path.join(gtdir, f'grad_face_vertices_image_{tag}.pt')).double()
    save('dibr_sphere.npz', **arrays)


def dibr_sphere_scaled_eps():
    """The sphere case through the reference's naive renderer in float64, set up to compute
    what the CUDA kernel computes, so these vectors pin the restatement's arithmetic and not
    just the reference tests' tolerance band.  Two differences of the naive oracle are undone:
    * pixel centres: the kernel forms them in float, ``multiplier / W * (2i + 1 - W)``
      (rasterization_cuda.cu:85-86), also for f64 inputs; here they are those float values
      divided by the multiplier (in float64);
    * eps: the naive oracle normalises by k3 + eps in UNSCALED coordinates; the kernel's
      forward by k3 + copysign(eps) in coordinates x multiplier, where k3 is multiplier^2
      larger (rasterization_cuda.cu:96-99): the forward fixtures use eps = 1e-8 / 1000^2.  The
      kernel's backward works in unscaled coordinates with eps itself
      (rasterization_cuda.cu:262-275): the gradient fixtures use eps = 1e-8."""
    H, W = 35, 31
    m = 1000.
    arrays = {}
    for dname, dtype in (('f32', torch.float), ('f64', torch.double)):
        for flip in (0, 1):
            inp = _sphere_inputs(dtype, bool(flip))
            p = f'{dname}_flip{flip}_'
            B = 3
            fvz64 = inp['face_vertices_z'].double()
            _, rr = _pixel_coords_ranges(fvz64, H, W, vertices_z=inp['vertices_camera_z'].double())
            mf = torch.tensor(m, dtype=torch.float32)
            x = ((mf / W) * (2 * torch.arange(W) + 1 - W).float()).double() / m
            y = ((mf / H) * (H - 2 * torch.arange(H) - 1).float()).double() / m
            pix = torch.stack([x.reshape(1, 1, -1).repeat(B, H, 1), y.reshape(1, -1, 1).repeat(B, 1, W)],
                              dim=-1).reshape(B, -1, 2)
            for use_valid in (0, 1):
                kw = {'valid_faces': inp['valid_faces']} if use_valid else {}
                q = p + f'valid{use_valid}_'
                fvi = inp['face_vertices_image'].double()
                fuv = inp['face_uvs'].double()
                g = torch.Generator().manual_seed(1234 + use_valid)
                grad_out = torch.rand((B, H, W, fuv.shape[-1]), generator=g, dtype=dtype).double()
                # forward eps: features, and the feature gradient (sum of grad x forward weights)
                fuv_r = fuv.clone().requires_grad_(True)
                feats, idx = _naive_deftet_sparse_render(pix, rr, fvz64, fvi, fuv_r, 1, eps=1e-8 / m ** 2, **kw)
                feats = feats.reshape(B, H, W, -1)
                feats.backward(grad_out)
                arrays[q + 'features'] = feats.detach()
                arrays[q + 'face_idx'] = idx.reshape(B, H, W)
                arrays[q + 'grad_face_uvs'] = fuv_r.grad
                # backward eps: the vertex gradient
                fvi_r = fvi.clone().requires_grad_(True)
                feats, _ = _naive_deftet_sparse_render(pix, rr, fvz64, fvi_r, fuv, 1, eps=1e-8, **kw)
                feats.reshape(B, H, W, -1).backward(grad_out)
                arrays[q + 'grad_face_vertices_image'] = fvi_r.grad
    save('dibr_sphere_scaled_eps.npz', **arrays)


# --------------------------------------------------------------------------
# point_to_mesh_distance (tests/python/kaolin/metrics/test_trianglemesh.py)
# --------------------------------------------------------------------------
def p2m():
    arrays = {}
    # KAT :24-79
    pts = torch.tensor([[0., -1., -1.], [1., -1., -1.], [-1., -1., -1.], [0., -1., 2.],
                        [1., -1., 2.], [-1, -1., 2.], [0., 2., 0.5], [1., 2., 0.5],
                        [-1., 2., 0.5], [0., -1., 0.5], [1., -1., 0.5], [-1., -1., 0.5],
                        [0., 1., 1.], [1., 1., 1.], [-1., 1., 1.], [0., 1., 0.], [1., 1., 0.],
                        [-1., 1., 0.], [1., 0.5, 0.5], [-1., 0.5, 0.5]], dtype=torch.double)
    verts = torch.tensor([[0., 0., 0.], [0., 0., 1.], [0., 1., 0.5], [0.5, 0., 0.],
                          [0.5, 0., 1.], [0.5, 1., 0.5]], dtype=torch.double)
    faces = torch.tensor([[0, 1, 2], [3, 4, 5]])
    arrays['kat_points'] = pts
    arrays['kat_face_vertices'] = verts[faces]
    arrays['kat_dist'] = torch.tensor([2.0000, 2.2500, 3.0000, 2.0000, 2.2500, 3.0000, 1.0000, 1.2500, 2.0000,
                                       1.0000, 1.2500, 2.0000, 0.2000, 0.4500, 1.2000, 0.2000, 0.4500, 1.2000,
                                       0.2500, 1.0000], dtype=torch.double)
    arrays['kat_face_idx'] = torch.tensor([0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 1, 0])
    arrays['kat_dist_type'] = torch.tensor([1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 0, 0], dtype=torch.int32)
    d, i, t = ref_tm._unbatched_naive_point_to_mesh_distance(pts, verts[faces])
    assert torch.equal(i, arrays['kat_face_idx']) and torch.equal(t, arrays['kat_dist_type'])
    # random 1025 x 1025 (:81-152), seeded here; oracle outputs + autograd grads
    for dname, dtype in (('f32', torch.float), ('f64', torch.double)):
        g = torch.Generator().manual_seed(7 if dname == 'f32' else 8)
        P = torch.randn((1025, 3), generator=g, dtype=dtype)
        FV = torch.randn((1025, 3, 3), generator=g, dtype=dtype)
        P1 = P.clone().requires_grad_(True)
        FV1 = FV.clone().requires_grad_(True)
        d, i, t = ref_tm._unbatched_naive_point_to_mesh_distance(P1, FV1)
        gout = torch.rand(d.shape, generator=g, dtype=dtype)
        d.backward(gout)
        arrays[f'rand_{dname}_points'] = P
        arrays[f'rand_{dname}_face_vertices'] = FV
        arrays[f'rand_{dname}_dist'] = d.detach()
        arrays[f'rand_{dname}_face_idx'] = i
        arrays[f'rand_{dname}_dist_type'] = t
        arrays[f'rand_{dname}_grad_out'] = gout
        arrays[f'rand_{dname}_grad_points'] = P1.grad
        arrays[f'rand_{dname}_grad_face_vertices'] = FV1.grad
    save('p2m.npz', **arrays)


# --------------------------------------------------------------------------
# sided_distance (tests/python/kaolin/metrics/test_pointcloud.py)
# --------------------------------------------------------------------------
def sided():
    arrays = {}
    arrays['kat_p1'] = torch.tensor([[[8.8977, 4.1709, 1.2839], [8.5640, 7.7767, 9.4214]],
                                     [[0.5431, 6.4495, 11.4914], [3.2126, 8.0865, 3.1018]]], dtype=torch.double)
    arrays['kat_p2'] = torch.tensor([[[6.9340, 6.1152, 3.4435], [0.1032, 9.8181, 11.3350]],
                                     [[11.4006, 2.2154, 7.9589], [4.2586, 1.4133, 7.2606]]], dtype=torch.double)
    arrays['kat_dist'] = torch.tensor([[12.3003, 41.1528], [57.0679, 62.9213]], dtype=torch.double)
    arrays['kat_idx'] = torch.tensor([[0, 0], [1, 1]])
    # integer-valued "large" input (:58-67): many exact ties -> lowest index wins
    g = torch.Generator().manual_seed(0)
    p1 = torch.randint(0, 100, (3, 100, 3), generator=g).double()
    p2 = torch.randint(0, 100, (3, 50, 3), generator=g).double()
    arrays['large_p1'] = p1
    arrays['large_p2'] = p2
    arrays['large_dist'] = ref_pc._sided_distance(p1, p2)
    # random float clouds (cfg1 distribution: U[0,1]^3, seed 0)
    g = torch.Generator().manual_seed(0)
    q1 = torch.rand((2, 700, 3), generator=g, dtype=torch.float)
    q2 = torch.rand((2, 900, 3), generator=g, dtype=torch.float)
    arrays['rand_p1'] = q1
    arrays['rand_p2'] = q2
    arrays['rand_dist'] = ref_pc._sided_distance(q1, q2)
    save('sided.npz', **arrays)


# --------------------------------------------------------------------------
# trianglemeshes_to_voxelgrids (pure PyTorch reference run directly)
# --------------------------------------------------------------------------
def _uv_sphere(n_lat, n_lon, radius=1.0, dtype=torch.float):
    lat = torch.linspace(0, math.pi, n_lat + 1, dtype=torch.double)[1:-1]
    lon = torch.arange(n_lon, dtype=torch.double) * (2 * math.pi / n_lon)
    ring = torch.stack([torch.sin(lat)[:, None] * torch.cos(lon)[None],
                        torch.cos(lat)[:, None].expand(-1, n_lon),
                        torch.sin(lat)[:, None] * torch.sin(lon)[None]], -1).reshape(-1, 3)
    verts = torch.cat([torch.tensor([[0., 1., 0.]], dtype=torch.double), ring,
                       torch.tensor([[0., -1., 0.]], dtype=torch.double)]) * radius
    faces = []
    nr = n_lat - 1
    for j in range(n_lon):
        faces.append([0, 1 + (j + 1) % n_lon, 1 + j])
    for i in range(nr - 1):
        for j in range(n_lon):
            a = 1 + i * n_lon + j
            b = 1 + i * n_lon + (j + 1) % n_lon
            c = 1 + (i + 1) * n_lon + j
            d = 1 + (i + 1) * n_lon + (j + 1) % n_lon
            faces.append([a, b, d])
            faces.append([a, d, c])
    last = 1 + nr * n_lon
    for j in range(n_lon):
        a = 1 + (nr - 1) * n_lon + j
        b = 1 + (nr - 1) * n_lon + (j + 1) % n_lon
        faces.append([a, b, last])
    return verts.to(dtype), torch.tensor(faces, dtype=torch.long)


def voxelgrid():
    arrays = {}
    cases = []
    # KAT inputs of ops/conversions/test_trianglemesh.py:45-242
    cases.append(('batched', torch.tensor([[[0, 0, 0], [1, 0, 0], [0, 0, 1]],
                                           [[0, 0, 0], [0, 1, 0], [1, 0, 1]]], dtype=torch.float),
                  torch.tensor([[0, 1, 2]]), 3, torch.zeros((2, 3)), torch.ones(2)))
    cases.append(('origins', torch.tensor([[[0, 0, 0], [1, 0, 0], [0, 0, 1]]], dtype=torch.float),
                  torch.tensor([[0, 1, 2]]), 3, torch.ones((1, 3)) * 0.5, torch.ones(1)))
    cases.append(('scale', torch.tensor([[[0, 0, 0], [1, 0, 0], [0, 0, 1]]], dtype=torch.float),
                  torch.tensor([[0, 1, 2]]), 3, torch.zeros((1, 3)), torch.ones(1) * 2))
    cases.append(('res7', torch.tensor([[[0, 0, 0], [1, 0, 0], [0, 0, 1]]], dtype=torch.float),
                  torch.tensor([[0, 1, 2]]), 7, torch.zeros((1, 3)), torch.ones(1)))
    cases.append(('default_os', torch.tensor([[[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0]]], dtype=torch.float),
                  torch.tensor([[0, 1, 2], [1, 2, 3]]), 5, None, None))
    sv, sf = _uv_sphere(24, 40, 0.9)
    cases.append(('sphere32', sv.unsqueeze(0), sf, 32, None, None))
    g = torch.Generator().manual_seed(3)
    rv = torch.rand((2, 60, 3), generator=g)
    rf = torch.randint(0, 60, (80, 3), generator=g)
    cases.append(('random24', rv, rf, 24, None, None))
    for name, v, f, R, o, s in cases:
        vg = trianglemeshes_to_voxelgrids(v, f, R, o, s)
        arrays[f'{name}_vertices'] = v
        arrays[f'{name}_faces'] = f
        arrays[f'{name}_resolution'] = np.int64(R)
        if o is not None:
            arrays[f'{name}_origin'] = o
            arrays[f'{name}_scale'] = s
        arrays[f'{name}_occupied'] = torch.nonzero(vg).to(torch.int32)  # (N,4) b,x,y,z sorted
        print(name, 'occupied', int(vg.sum()))
    save('voxelgrid.npz', **arrays)


# --------------------------------------------------------------------------
# SPC KATs: mesh_to_spc (ops/conversions/test_trianglemesh.py:244-369),
# raytrace (render/spc/test_raytrace.py:22-345), scan/generate (ops/spc/test_spc.py:33-80)
# --------------------------------------------------------------------------
def spc():
    arrays = {}
    faces = np.array([[0, 1, 2], [2, 1, 3], [4, 5, 6], [7, 8, 9]])
    verts = np.array([[-0.4272, 0.0795, 0.3548], [-0.9217, 0.3106, 0.1516], [-0.2636, 0.3794, -0.7979],
                      [0.1259, 0.9089, 0.7439], [0.0710, -0.6947, -0.0480], [0.6215, 0.2809, -0.0480],
                      [0.4972, 0.3347, 0.4422], [-0.4374, 0.4967, -0.6047], [0.0397, 0.1230, -0.7417],
                      [-0.3534, 0.9970, -0.4558]], dtype=np.float32)
    arrays['m2s_face_vertices'] = verts[faces]
    arrays['m2s_level'] = np.int64(3)
    arrays['m2s_octree'] = np.array([252, 242, 213, 10, 5, 35, 29, 232, 172, 79, 170, 55, 245, 48,
                                     7, 179, 81, 8, 162, 4, 209, 2, 32, 10, 176, 11, 4, 15], dtype=np.uint8)
    arrays['m2s_face_idx'] = np.array([0, 0, 0, 0, 0, 0, 3, 1, 0, 0, 0, 0, 1, 3, 3, 3, 3, 1, 1, 3, 1, 1,
                                       0, 0, 0, 0, 0, 1, 1, 1, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2,
                                       2, 2, 2, 2, 2, 2, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 2, 2, 2, 2], dtype=np.int64)
    arrays['m2s_bary'] = np.array([
        [4.5012e-08, 7.7766e-01], [2.8764e-01, 4.0506e-01], [3.5860e-08, 4.7760e-01], [1.0753e-01, 5.5666e-01],
        [2.5024e-08, 3.0500e-04], [5.3537e-03, 1.7265e-01], [2.4690e-01, 7.5310e-01], [8.8672e-01, 4.2031e-09],
        [4.0263e-01, 1.9203e-05], [6.0202e-01, 3.6483e-08], [2.2252e-01, 1.5161e-01], [4.3968e-01, 1.3058e-01],
        [7.3768e-01, 2.0286e-02], [6.2631e-01, 8.5154e-02], [2.8269e-01, 2.0198e-02], [7.7711e-08, 4.6322e-01],
        [9.7272e-08, 2.4475e-01], [6.3429e-01, 1.7624e-01], [4.4455e-01, 2.6633e-01], [1.8181e-01, 2.8813e-08],
        [7.0239e-01, 3.2221e-08], [5.5041e-01, 2.5328e-02], [1.7266e-01, 8.1010e-01], [1.7232e-08, 9.5489e-01],
        [5.0481e-01, 3.8403e-01], [6.9277e-01, 3.0723e-01], [3.2469e-01, 5.3563e-01], [2.7070e-08, 7.3333e-01],
        [1.4894e-01, 5.9743e-01], [5.6993e-09, 6.5052e-01], [8.0139e-01, 4.1631e-08], [1.0000e+00, 0.0000e+00],
        [2.5233e-01, 4.4148e-01], [2.5480e-01, 3.5643e-01], [6.5063e-02, 4.4652e-01], [3.6067e-01, 1.1542e-01],
        [1.7093e-01, 2.0551e-01], [1.7340e-01, 1.2046e-01], [4.2470e-08, 4.2354e-01], [2.3278e-08, 2.7855e-01],
        [4.6319e-08, 1.9574e-01], [9.2212e-01, 7.7879e-02], [7.2775e-01, 2.7225e-01], [6.1808e-01, 3.8192e-01],
        [4.2371e-01, 5.7629e-01], [8.7880e-01, 2.5213e-08], [7.0510e-01, 8.7381e-09], [6.1462e-01, 1.1334e-01],
        [4.1944e-01, 2.4449e-01], [3.7678e-01, 3.8143e-08], [3.8031e-08, 9.9842e-01], [2.2935e-01, 7.7065e-01],
        [1.1967e-01, 8.8033e-01], [0.0000e+00, 1.0000e+00], [2.2426e-01, 3.7564e-01], [2.0308e-01, 1.5850e-08],
        [2.3061e-02, 3.8613e-02], [3.9331e-01, 1.1329e-08], [2.5610e-01, 1.6592e-08], [2.0898e-01, 1.9427e-08],
        [7.1771e-02, 1.6657e-08], [1.1603e-01, 5.9735e-01], [1.1001e-01, 1.2918e-01], [2.4004e-08, 6.5422e-01],
        [2.3279e-08, 1.8040e-01]], dtype=np.float32)

    # scan_octrees / generate_points KAT (test_spc.py:33-80)
    bits = [[0, 0, 0, 1, 0, 0, 0, 1],
            [0, 0, 0, 0, 0, 1, 1, 0], [0, 0, 1, 0, 0, 0, 0, 0],
            [1, 0, 0, 0, 0, 0, 0, 0], [1, 0, 0, 0, 0, 0, 0, 0], [0, 0, 0, 0, 1, 0, 0, 0],
            [1, 0, 0, 0, 0, 0, 0, 0],
            [0, 1, 1, 1, 0, 0, 0, 0],
            [0, 0, 1, 0, 0, 0, 0, 0], [1, 1, 1, 1, 1, 1, 1, 1], [0, 1, 0, 1, 0, 1, 0, 1]]
    # test_spc.py builds bytes as bits_to_uint8(torch.flip(bits_t)): column j -> bit (7 - j)
    arrays['scan_octrees'] = np.array([sum(int(b[j]) << (7 - j) for j in range(8)) for b in bits], dtype=np.uint8)
    arrays['scan_lengths'] = np.array([6, 5], dtype=np.int32)
    arrays['scan_max_level'] = np.int64(3)
    arrays['scan_pyramids'] = np.array([[[1, 2, 3, 3, 0], [0, 1, 3, 6, 9]],
                                        [[1, 1, 3, 13, 0], [0, 1, 2, 5, 18]]], dtype=np.int32)
    arrays['scan_exsum'] = np.array([0, 2, 4, 5, 6, 7, 8, 0, 1, 4, 5, 13, 17], dtype=np.int32)
    arrays['scan_points'] = np.array([
        [0, 0, 0], [0, 0, 0], [1, 0, 0], [0, 0, 1], [0, 1, 0], [3, 0, 1], [1, 1, 3], [1, 3, 1], [6, 1, 3],
        [0, 0, 0], [1, 1, 1], [3, 2, 2], [3, 2, 3], [3, 3, 2], [7, 4, 5], [6, 4, 6], [6, 4, 7], [6, 5, 6],
        [6, 5, 7], [7, 4, 6], [7, 4, 7], [7, 5, 6], [7, 5, 7], [6, 6, 4], [6, 7, 4], [7, 6, 4], [7, 7, 4]],
        dtype=np.int16)

    # raytrace KAT octree (test_raytrace.py:24-31)
    rbits = [[0, 0, 0, 1, 0, 1, 1, 1],
             [1, 1, 1, 1, 1, 1, 1, 1], [0, 0, 0, 0, 0, 0, 1, 1],
             [0, 0, 0, 0, 0, 0, 0, 1], [0, 0, 0, 0, 0, 0, 0, 0]]
    arrays['rt_octree'] = np.array([sum(int(b[j]) << (7 - j) for j in range(8)) for b in rbits], dtype=np.uint8)

    def rays_origin(h, w, dist):
        ii, jj = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing='ij')
        ii = (ii * np.float32(2.) / np.float32(h)) - np.float32((h - 1.) / h)
        jj = (jj * np.float32(2.) / np.float32(w)) - np.float32((w - 1.) / w)
        return np.stack([ii, jj, np.full_like(ii, dist)], -1).reshape(-1, 3).astype(np.float32)

    cases = {
        'positive': (-3, [0., 0., 1.], 2, False, False,
                     [[0, 5], [0, 6], [0, 13], [0, 14], [1, 7], [1, 8], [2, 15], [4, 9], [4, 10], [5, 11], [5, 12]], None),
        'negative': (3, [0., 0., -1.], 2, False, False,
                     [[0, 14], [0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]], None),
        'none': (3, [0., 0., 1.], 2, True, True, np.zeros((0, 2)), np.zeros((0, 2))),
        'coarser': (-3, [0., 0., 1.], 1, False, False,
                    [[0, 1], [0, 2], [1, 1], [1, 2], [2, 3], [3, 3], [4, 1], [4, 2], [5, 1], [5, 2], [6, 3], [7, 3],
                     [8, 4], [9, 4], [12, 4], [13, 4]], None),
        'depth': (3, [0., 0., -1.], 2, True, False,
                  [[0, 14], [0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]],
                  [[2.0], [2.5], [3.0], [3.5], [3.0], [3.5], [3.5], [3.0], [3.5], [3.0], [3.5]]),
        'depth_exit': (3, [0., 0., -1.], 2, True, True,
                       [[0, 14], [0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]],
                       [[2.0, 2.5], [2.5, 3.0], [3.0, 3.5], [3.5, 4.0], [3.0, 3.5], [3.5, 4.0], [3.5, 4.0],
                        [3.0, 3.5], [3.5, 4.0], [3.0, 3.5], [3.5, 4.0]]),
        'inside_nodepth': (0.9, [0., 0., -1.], 2, False, False,
                           [[0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]], None),
        'inside_depth': (0.9, [0., 0., -1.], 2, True, False,
                         [[0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]],
                         [[0.4], [0.9], [1.4], [0.9], [1.4], [1.4], [0.9], [1.4], [0.9], [1.4]]),
        'inside_exit': (0.9, [0., 0., -1.], 2, True, True,
                        [[0, 13], [0, 6], [0, 5], [1, 8], [1, 7], [2, 15], [4, 10], [4, 9], [5, 12], [5, 11]],
                        [[0.4, 0.9], [0.9, 1.4], [1.4, 1.9], [0.9, 1.4], [1.4, 1.9], [1.4, 1.9], [0.9, 1.4],
                         [1.4, 1.9], [0.9, 1.4], [1.4, 1.9]]),
    }
    for name, (dist, d, level, rd, we, nug, dep) in cases.items():
        arrays[f'rt_{name}_origin'] = rays_origin(4, 4, dist)
        arrays[f'rt_{name}_direction'] = np.tile(np.array(d, dtype=np.float32), (16, 1))
        arrays[f'rt_{name}_cfg'] = np.array([level, int(rd), int(we)], dtype=np.int64)
        arrays[f'rt_{name}_nuggets'] = np.array(nug, dtype=np.int32).reshape(-1, 2)
        if dep is not None:
            arrays[f'rt_{name}_depth'] = np.array(dep, dtype=np.float32).reshape(len(nug), 2 if we else 1)
    # ambiguous raytrace (test_raytrace.py:270-300)
    arrays['rt_ambiguous_octree'] = np.array([255], dtype=np.uint8)
    arrays['rt_ambiguous_origin'] = np.array([[0., 0., 3.], [3., 3., 3.]], dtype=np.float32)
    arrays['rt_ambiguous_direction'] = np.array([[0., 0., -1.], [-1. / 3., -1. / 3., -1. / 3.]], dtype=np.float32)
    arrays['rt_ambiguous_nuggets'] = np.array([[0, 2], [0, 1], [0, 4], [0, 6], [0, 3], [0, 5], [0, 8], [0, 7],
                                               [1, 8], [1, 1]], dtype=np.int32)
    # mark_pack_boundaries KAT on the 'positive' case ridx (test_raytrace.py:302-315)
    arrays['rt_positive_first_hits'] = np.array([1, 0, 0, 0, 1, 0, 1, 1, 0, 1, 0], dtype=np.bool_)
    save('spc.npz', **arrays)


def rayops():
    """Packed ray-op KATs transcribed from render/spc/test_rayops.py:20-208 (data only):
    feats (6,2), tau (6,1), boundaries [1,0,1,0,0,1], and every expected output there."""
    f = np.array([[1, 1], [1, 1], [1, 1], [2, 2], [3, 3], [5, 5]], dtype=np.float32)
    arrays = {
        'feats': f,
        'tau': np.array([[0], [0], [0], [1], [0], [1]], dtype=np.float32),
        'boundaries': np.array([1, 0, 1, 0, 0, 1], dtype=np.bool_),
        'ridx': np.array([1, 1, 1, 1, 2, 2, 3, 3, 3], dtype=np.int32),
        'ridx_boundaries': np.array([1, 0, 0, 0, 1, 0, 1, 0, 0], dtype=np.bool_),
        'diff': np.array([[0, 0], [0, 0], [1, 1], [1, 1], [0, 0], [0, 0]], dtype=np.float32),
        'sum_reduce': np.array([[2, 2], [6, 6], [5, 5]], dtype=np.float32),
        'cumsum': np.array([[1, 1], [2, 2], [1, 1], [3, 3], [6, 6], [5, 5]], dtype=np.float32),
        'cumsum_reverse': np.array([[2, 2], [1, 1], [6, 6], [5, 5], [3, 3], [5, 5]], dtype=np.float32),
        'cumsum_exclusive': np.array([[0, 0], [1, 1], [0, 0], [1, 1], [3, 3], [0, 0]], dtype=np.float32),
        'cumsum_exclusive_reverse': np.array([[1, 1], [0, 0], [5, 5], [3, 3], [0, 0], [0, 0]], dtype=np.float32),
        'cumprod': np.array([[1, 1], [1, 1], [1, 1], [2, 2], [6, 6], [5, 5]], dtype=np.float32),
        'cumprod_reverse': np.array([[1, 1], [1, 1], [6, 6], [6, 6], [3, 3], [5, 5]], dtype=np.float32),
        'cumprod_exclusive': np.array([[1, 1], [1, 1], [1, 1], [1, 1], [2, 2], [1, 1]], dtype=np.float32),
        'cumprod_exclusive_reverse': np.array([[1, 1], [1, 1], [6, 6], [3, 3], [1, 1], [1, 1]], dtype=np.float32),
        # exponential_integration(exclusive=False), atol 1e-4 in the reference test
        'expint_feats': np.array([[0, 0], [0.4651, 0.4651], [1.1627, 1.1627]], dtype=np.float32),
        'expint_transmittance': np.array([[0.0], [0.0], [0.0], [0.2325], [0.0], [0.2325]], dtype=np.float32),
    }
    save('rayops.npz', **arrays)


# --------------------------------------------------------------------------
# DefTet sparse render (tests/python/kaolin/render/mesh/test_deftet.py)
# --------------------------------------------------------------------------
def deftet():
    """Simple-case KATs transcribed from test_deftet.py:36-230 (data only), and the model.obj
    case of test_deftet.py:335-551 run through the reference's _naive_deftet_sparse_render
    (forward + autograd backward) in f32 and f64."""
    arrays = {
        'simple_fvi': np.array(
            [[[[-1., 0.], [0., -1.], [0., 1.]], [[-1., 0.], [0., 1.], [0., -1.]], [[0., -1.], [0., 1.], [1., 0.]]],
             [[[-1., -1.], [1., -1.], [-1., 1.]], [[-1., -1.], [1., -1.], [-1., 1.]],
              [[-1., -1.], [1., -1.], [-1., 1.]]]]),
        'simple_fvz': np.array([[[-2., -1., -1.], [-2.5, -3., -3.], [-2., -2., -2.]],
                                [[-2., -1., -3.], [-2., -2., -2.], [-2., -3., -1.]]]),
        'simple_feat_face': np.array([[[[0.]] * 3, [[1.]] * 3, [[2.]] * 3], [[[3.]] * 3, [[4.]] * 3, [[5.]] * 3]]),
        'simple_feat_vert': np.arange(18, dtype=np.float64).reshape(2, 3, 3, 1),
        'simple_pix': np.array(
            [[[-0.999, 0.], [-0.001, -0.998], [0.001, 0.998], [0.999, 0.], [-0.45, 0.], [0.45, 0.], [-0.999, -0.999]],
             [[-0.998, -0.999], [0.998, -0.999], [-0.999, 0.998], [-0.001, -0.], [0., -0.999], [-0.999, 0.],
              [0.001, 0.001]]]),
        # test_full_render (range [-4, 0), knum=5)
        'simple_full_idx': np.array(
            [[[0, 1, -1, -1, -1], [0, 1, -1, -1, -1], [2, -1, -1, -1, -1], [2, -1, -1, -1, -1],
              [0, 1, -1, -1, -1], [2, -1, -1, -1, -1], [-1, -1, -1, -1, -1]],
             [[0, 1, 2, -1, -1], [0, 1, 2, -1, -1], [2, 1, 0, -1, -1], [2, 1, 0, -1, -1],
              [0, 1, 2, -1, -1], [2, 1, 0, -1, -1], [-1, -1, -1, -1, -1]]], dtype=np.int64),
        'simple_full_feat_vert': np.array(
            [[[0., 3., 0., 0., 0.], [1., 5., 0., 0., 0.], [7., 0., 0., 0., 0.], [8., 0., 0., 0., 0.],
              [0.825, 3.825, 0., 0., 0.], [7.175, 0., 0., 0., 0.], [0., 0., 0., 0., 0.]],
             [[9., 12., 15., 0., 0.], [10., 13., 16., 0., 0.], [17., 14., 11., 0., 0.], [16.5, 13.5, 10.5, 0., 0.],
              [9.5, 12.5, 15.5, 0., 0.], [16., 13., 10., 0., 0.], [0., 0., 0., 0., 0.]]]),
        # test_restricted_range (range [-2.1, 0), knum=5)
        'simple_restricted_idx': np.array(
            [[[0, -1, -1, -1, -1], [0, -1, -1, -1, -1], [2, -1, -1, -1, -1], [2, -1, -1, -1, -1],
              [0, -1, -1, -1, -1], [2, -1, -1, -1, -1], [-1, -1, -1, -1, -1]],
             [[0, 1, 2, -1, -1], [0, 1, -1, -1, -1], [2, 1, -1, -1, -1], [2, 1, 0, -1, -1],
              [0, 1, -1, -1, -1], [2, 1, -1, -1, -1], [-1, -1, -1, -1, -1]]], dtype=np.int64),
        'simple_restricted_feat_vert': np.array(
            [[[0., 0., 0., 0., 0.], [1., 0., 0., 0., 0.], [7., 0., 0., 0., 0.], [8., 0., 0., 0., 0.],
              [0.825, 0., 0., 0., 0.], [7.175, 0., 0., 0., 0.], [0., 0., 0., 0., 0.]],
             [[9., 12., 15., 0., 0.], [10., 13., 0., 0., 0.], [17., 14., 0., 0., 0.], [16.5, 13.5, 10.5, 0., 0.],
              [9.5, 12.5, 0., 0., 0.], [16., 13., 0., 0., 0.], [0., 0., 0., 0., 0.]]]),
    }
    P, K = 128, 20
    for dname, dtype in (('f32', torch.float), ('f64', torch.double)):
        inp = _sphere_inputs(dtype, False)
        fvz, fvi, fuv = inp['face_vertices_z'], inp['face_vertices_image'], inp['face_uvs']
        vz = inp['vertices_camera_z']
        B = fvz.shape[0]
        g = torch.Generator().manual_seed(77)
        pix = torch.rand((B, P, 2), generator=g, dtype=dtype) * 2. - 1.
        arrays[f'{dname}_fvz'] = fvz
        arrays[f'{dname}_fvi'] = fvi
        arrays[f'{dname}_fuv'] = fuv
        arrays[f'{dname}_pix'] = pix
        for up in (0, 1):
            min_z, max_z = vz.min(dim=1)[0], vz.max(dim=1)[0]
            lo = (min_z + max_z) / 2. if up else min_z
            rr = torch.nn.functional.pad(lo.unsqueeze(-1), (0, 1), value=0.).unsqueeze(1).repeat(1, P, 1)
            fvi_r = fvi.clone().requires_grad_(True)
            fuv_r = fuv.clone().requires_grad_(True)
            feats, idx = _naive_deftet_sparse_render(pix, rr, fvz, fvi_r, fuv_r, K)
            grad_out = torch.rand(feats.shape, generator=g, dtype=dtype)
            feats.backward(grad_out)
            q = f'{dname}_up{up}_'
            arrays[q + 'ranges'] = rr
            arrays[q + 'features'] = feats.detach()
            arrays[q + 'face_idx'] = idx
            arrays[q + 'grad_out'] = grad_out
            arrays[q + 'grad_fvi'] = fvi_r.grad
            arrays[q + 'grad_fuv'] = fuv_r.grad
    save('deftet.npz', **arrays)


# --------------------------------------------------------------------------
# check_sign (tests/python/kaolin/ops/mesh/test_check_sign.py:26-186): transcribed data
# --------------------------------------------------------------------------
def check_sign():
    v = np.array([[1., 0., 0.], [1., 0., 1.], [1., -1., -1.], [1., 1., -1.],
                  [-1., 0., 0.], [-1., 0., -4.], [-1., -4., 4.], [-1., 4., 4.]])
    faces = np.array([[0, 1, 2], [0, 2, 3], [0, 3, 1], [1, 2, 6], [2, 3, 5], [3, 1, 7],
                      [5, 6, 2], [6, 7, 1], [7, 5, 3], [4, 6, 5], [4, 7, 6], [4, 5, 7]], np.int64)
    p = np.array([[0.9, 0., 0.], [0.9, 0., -1.], [0.9, 0., -0.9], [0.9, 0.1, -1.0], [0.9, 0., 1.],
                  [0.9, -1., -1.], [0.9, 1., -1.], [-0.99, 0., -3.9], [-0.99, -3.9, 3.9], [-0.99, 3.9, 3.9],
                  [0.9, 0., -4.], [0.9, -4., 4.], [0.9, 4., 4.], [0.9, 0., 4.], [-0.9, 0., -3.9],
                  [-0.9, -3.9, 3.9], [-0.9, 3.9, 3.9], [0.5, 0., 5.], [0.5, -5., 4.], [1.1, 0., 0.],
                  [1.1, 0., -1.], [1.1, 0., -0.9], [1.1, 0.1, -1.0], [1.1, 0., 1.], [1.1, -1., -1.],
                  [1.1, 1., -1.], [-1.1, 0., 0.], [-1.1, 0., -1.], [-1.1, 0., -0.9], [-1.1, 0.1, -1.0],
                  [-1.1, 0., 1.], [-1.1, -1., -1.], [-1.1, 1., -1.]])
    e = np.array([True] * 10 + [False] * 23)
    save('check_sign.npz', verts=np.stack([v, -v]), faces=faces,
         zero_area_faces=np.array([[1, 1, 1], [0, 0, 0], [2, 2, 2], [3, 3, 3]], np.int64),
         points=np.stack([p, -p[::-1]]), expected=np.stack([e, e[::-1]]))


if __name__ == '__main__':
    torch.set_num_threads(8)
    if len(sys.argv) > 1:  # regenerate only the named fixtures
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    dibr_simple()
    dibr_sphere()
    dibr_sphere_scaled_eps()
    p2m()
    sided()
    voxelgrid()
    spc()
    rayops()
