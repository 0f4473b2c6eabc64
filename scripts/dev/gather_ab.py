"""A/B timing of the backward kernels on the cfg3 workload under dev flags (development aid).

usage: python scripts/dev/gather_ab.py SPEC [SPEC ...]
SPEC: comma-separated settings, each FLAGS (an int: dev flag bits) or pK=V (dev param K); "0" = product path
Times the standalone gather (rasterize_backward with the forward's face ranges) and the whole
dibr_backward with HIP events, and checks each flag's gradients against flag 0's.
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(3):
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
    specs = sys.argv[1:] or ['0']
    lib = N.lib()
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]

    def apply(spec):
        lib.kl_dev_set_flags(0)
        for k in range(16):
            lib.kl_dev_set_param(k, 0)
        for item in spec.split(','):
            if item.startswith('p'):
                k, v = item[1:].split('=')
                lib.kl_dev_set_param(int(k), int(v, 0))
            else:
                lib.kl_dev_set_flags(int(item, 0))
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    feats, idx, w, mask, state, ranges = _fused.dibr_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'],
                                                             7000., 0.02, 30, 1000., 1e-8)
    ref = None
    for fl in specs:
        apply(fl)
        g = lambda: _fused.rasterize_backward(inp['g_feat'], idx, w, inp['fvi'], inp['feat'], None, 1000., 1e-8,  # noqa
                                             face_normals_z=inp['fnz'], face_ranges=ranges)
        d = lambda: _fused.dibr_backward(inp['g_feat'], inp['g_mask'], idx, w, inp['fvi'], inp['feat'],  # noqa
                                         inp['fnz'], mask, state, 7000., 1000., 1e-8, ranges)
        tg, td = timeit(g), timeit(d)
        out = d()
        torch.cuda.synchronize()
        same = ''
        if ref is None:
            ref = out
        else:
            same = 'equal' if all(torch.equal(a, b) for a, b in zip(out, ref)) else 'DIFFERENT'
        print(f'{fl}: gather {tg:.1f} us, dibr_backward {td:.1f} us {same}', flush=True)
    apply('0')


if __name__ == '__main__':
    main()
