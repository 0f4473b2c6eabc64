"""Compact soft-mask backward on the simple golden mesh with dev flags (development aid).
usage: python scripts/dev/diag_bwd.py DTYPE(f32|f64) FLAGS"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
import kaolin as kal  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402

dt = torch.float32 if sys.argv[1] == 'f32' else torch.float64
lib = N.lib()
lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'dibr_simple.npz'))
fvi = torch.from_numpy(g['face_vertices_image']).to('cuda', dt)
fvz = torch.from_numpy(g['face_vertices_z']).to('cuda', dt)
_, sel = kal.render.mesh.rasterize(35, 31, fvz, fvi, torch.zeros(fvz.shape + (1,), dtype=dt, device='cuda'))
mask, st = _fused.soft_mask_forward_compact(fvi, sel, 7000., 0.02, 30, 1000.)
torch.cuda.synchronize()
print('forward ok', flush=True)
lib.kl_dev_set_flags(int(sys.argv[2]))
gi = _fused.soft_mask_backward_compact(torch.ones_like(mask), mask, st, fvi, 7000., 1000.)
torch.cuda.synchronize()
lib.kl_dev_set_flags(0)
print('backward ok', float(gi.abs().sum()), flush=True)
