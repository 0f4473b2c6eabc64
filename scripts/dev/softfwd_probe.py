"""Time attribution for dibr_soft_mask forward on the bench workload (development aid).

Variants: the bench inputs; knum=1 (same selection, ~1/30 of the slot writes); every
pixel covered (no selection, every slot padding: the store pattern alone); no pixel
covered (heavier selection).  Plus torch fills of the same outputs as a store-rate
reference.  usage: python scripts/dev/softfwd_probe.py [variant-prefix]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    valid = inp['fnz'] >= 0
    feats, idx, w = _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)
    fvi = inp['fvi']
    allcov = torch.zeros_like(idx)
    nocov = torch.full_like(idx, -1)
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for name, sel, K in (('bench K=30', idx, 30), ('bench K=1', idx, 1), ('all covered K=30', allcov, 30),
                         ('none covered K=30', nocov, 30)):
        if only and not name.startswith(only):
            continue
        t = timeit(lambda: _fused.soft_mask_forward(fvi, sel, 7000., 0.02, K, 1000., with_hits=True))
        tc = timeit(lambda: _fused.soft_mask_forward_compact(fvi, sel, 7000., 0.02, K, 1000.))
        print('%-22s slots %8.1f us   compact %8.1f us' % (name, t, tc), flush=True)
    if only:
        return
    B = idx.shape[0]
    p = torch.empty((B, H, W, 30), device='cuda')
    i = torch.empty((B, H, W, 30), device='cuda', dtype=torch.int64)
    ty = torch.empty((B, H, W, 30), device='cuda', dtype=torch.uint8)
    t = timeit(lambda: (p.fill_(0), i.fill_(-1), ty.fill_(0)))
    print('%-22s %8.1f us  (%.0f GB/s)' % ('torch fills', t, (p.numel() * 13) / t / 1e3), flush=True)


if __name__ == '__main__':
    main()
