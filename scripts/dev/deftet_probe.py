"""Dev probe: deftet forward / resolve / backward and check_sign timings under workload variants."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
import bench  # noqa: E402
import kaolin as kal  # noqa: E402
from kaolin import _C  # noqa: E402


def ms(fn, n=5):
    return bench._event_ms(fn, n)


dev = torch.device('cuda', 0)
inp = bench.dibr_inputs([0.0, 1.57, 3.14, 4.71], dev)
fvz, fvi, feat, H, W = inp['fvz'], inp['fvi'], inp['feat'], inp['H'], inp['W']
B = fvz.shape[0]
x = (2 * torch.arange(W, device=dev, dtype=torch.float32) + 1 - W) / W
y = (H - 2 * torch.arange(H, device=dev, dtype=torch.float32) - 1.) / H
pix = torch.stack([x.view(1, -1).expand(H, W), y.view(-1, 1).expand(H, W)], -1).reshape(1, -1, 2).expand(B, -1, -1).contiguous()
zmin, zmax = fvz.reshape(B, -1).min(1)[0], fvz.reshape(B, -1).max(1)[0]
rr = torch.stack([zmin - 1e-2, zmax + 1e-2], -1).unsqueeze(1).expand(-1, H * W, -1).contiguous()
for K in (8, 2):
    f = lambda: _C.deftet_forward('f', fvz, fvi, None, pix, rr, K, 1e-8)  # noqa: E731
    idx, d, w0, w1 = f()
    print(f'K={K} fwd {ms(f):.3f} ms  hits {int((idx >= 0).sum())}', flush=True)
    r = lambda: _C.deftet_resolve(idx, d, w0, w1, feat)  # noqa: E731
    print(f'K={K} resolve {ms(r):.3f} ms', flush=True)
    sidx, wts, interp = r()
    g = torch.rand_like(interp)
    bw = lambda: kal._C.render.mesh.deftet_sparse_render_backward_cuda(g, sidx, wts, fvi, feat, 1e-8)  # noqa: E731
    print(f'K={K} bwd {ms(bw):.3f} ms', flush=True)
# empty range: no hits, same walk
rr0 = rr.clone()
rr0[..., 1] = rr0[..., 0]
f = lambda: _C.deftet_forward('f', fvz, fvi, None, pix, rr0, 8, 1e-8)  # noqa: E731
print(f'empty-range fwd {ms(f):.3f} ms', flush=True)
# a quarter of the pixels
f = lambda: _C.deftet_forward('f', fvz, fvi, None, pix[:, ::4].contiguous(), rr[:, ::4].contiguous(), 8, 1e-8)  # noqa
print(f'quarter-pixels fwd {ms(f):.3f} ms', flush=True)
verts, faces = bench.uv_sphere(126, 200, dev)
for n in (1000000, 100000):
    pts = (torch.rand((1, n, 3), generator=torch.Generator().manual_seed(3)) * 2 - 1).to(dev)
    v = verts.unsqueeze(0).contiguous()
    print(f'check_sign n={n} {ms(lambda: kal.ops.mesh.check_sign(v, faces, pts)):.3f} ms', flush=True)
