"""Ablation timing of the DIB-R ops on the bench workload (development aid).

Runs each op of bench.py's cfg3 step alone, timed with HIP events, with the library's
dev flags (kl_dev_set_flags) switching parts of kernels off.  Results are wrong while a
flag is set; this only attributes time.  usage: python scripts/dev/ablate.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402


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
    lib = N.lib()
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    valid = inp['fnz'] >= 0
    feats, idx, w = _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)
    mask, state = _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, 30, 1000.)
    gm = inp['g_mask']
    ops = {
        'rasterize_forward': lambda: _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid,
                                                              1000., 1e-8),
        'soft_mask_forward': lambda: _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, 30, 1000.),
        'soft_mask_backward': lambda: _fused.soft_mask_backward_compact(gm, mask, state, inp['fvi'], 7000., 1000.),
        'rasterize_backward': lambda: _fused.rasterize_backward(inp['g_feat'], idx, w, inp['fvi'], inp['feat'],
                                                                valid, 1000., 1e-8),
    }
    flags = [int(f) for f in os.environ.get('ABLATE_FLAGS', '0,1,2,4,6,7').split(',')]
    for name, fn in ops.items():
        row = []
        for f in flags:
            lib.kl_dev_set_flags(f)
            row.append('flags=%d: %7.1f us' % (f, timeit(fn)))
        lib.kl_dev_set_flags(0)
        print('%-20s %s' % (name, '  '.join(row)), flush=True)


if __name__ == '__main__':
    main()
