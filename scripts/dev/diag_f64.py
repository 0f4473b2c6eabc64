"""Compact soft-mask forward state on the simple golden mesh, f32 vs f64 (development aid)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
import kaolin as kal  # noqa: E402
from kaolin import _fused  # noqa: E402

g = np.load(os.path.join(ROOT, 'tests', 'golden', 'dibr_simple.npz'))
for dt in (torch.float32, torch.float64):
    fvi = torch.from_numpy(g['face_vertices_image']).to('cuda', dt)
    fvz = torch.from_numpy(g['face_vertices_z']).to('cuda', dt)
    _, sel = kal.render.mesh.rasterize(35, 31, fvz, fvi, torch.zeros(fvz.shape + (1,), dtype=dt, device='cuda'))
    mask, st = _fused.soft_mask_forward_compact(fvi, sel, 7000., 0.02, 30, 1000.)
    torch.cuda.synchronize()
    hits = st.hits.cpu().numpy().astype(np.int64)
    seg = st.seg_tot.cpu().numpy()
    print(dt, 'hits', hits.sum(), 'seg_tot', seg.sum(), seg.min(), seg.max(), 'per-row hits',
          hits.sum(-1).ravel()[:10], 'seg', seg[:10], flush=True)
