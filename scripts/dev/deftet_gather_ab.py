"""A/B of the deftet backward's gather kernel on the bench workload (4 views x 512^2, 50k faces, knum 8):
f32 at 5 waves per EU (96 VGPRs, default) against no bound (110 VGPRs, 4 waves; dev param 33 = 1);
equality of the gradients (development aid, run with KAOLIN_HIP_LIB pointing at the dev library)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kaolin as kal  # noqa: E402
from kaolin import _C, _native as N  # noqa: E402


def main():
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    dev = torch.device('cuda', 0)
    inp = bench.dibr_inputs([0.0, 1.57, 3.14, 4.71], dev)
    fvz, fvi, feat, H, W = inp['fvz'], inp['fvi'], inp['feat'], inp['H'], inp['W']
    B = fvz.shape[0]
    x = (2 * torch.arange(W, device=dev, dtype=torch.float32) + 1 - W) / W
    y = (H - 2 * torch.arange(H, device=dev, dtype=torch.float32) - 1.) / H
    pix = torch.stack([x.view(1, -1).expand(H, W), y.view(-1, 1).expand(H, W)], -1).reshape(1, -1, 2)
    pix = pix.expand(B, -1, -1).contiguous()
    zmin, zmax = fvz.reshape(B, -1).min(1)[0], fvz.reshape(B, -1).max(1)[0]
    rr = torch.stack([zmin - 1e-2, zmax + 1e-2], -1).unsqueeze(1).expand(-1, H * W, -1).contiguous()
    idx, d, w0, w1 = _C.deftet_forward('f', fvz, fvi, None, pix, rr, 8, 1e-8)
    sidx, wts, interp = _C.deftet_resolve(idx, d, w0, w1, feat)
    g = torch.rand_like(interp)
    bw = lambda: kal._C.render.mesh.deftet_sparse_render_backward_cuda(g, sidx, wts, fvi, feat, 1e-8)  # noqa: E731
    outs = {}
    for v in (0, 1, 0, 1, 0, 1):
        lib.kl_dev_set_param(33, v)
        outs[v] = bw()
        print(f'param 33={v}: deftet backward {bench._event_ms(bw, 10):.3f} ms', flush=True)
    lib.kl_dev_set_param(33, 0)
    print('equal:', all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])), flush=True)
    for v in (0, 1, 0, 1):
        lib.kl_dev_set_param(33, v)
        r = bench.deftet_bench(inp, 10)
        print(f"param 33={v}: deftet leg {r['ms']} ms (forward {r['fwd_ms']} ms), {r['value']} Mpx/s", flush=True)
    lib.kl_dev_set_param(33, 0)


if __name__ == '__main__':
    main()
