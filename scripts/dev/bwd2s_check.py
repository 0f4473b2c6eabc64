"""Bit-equality and timing of the fused backward under a dev parameter against the default
(development aid).  usage: python scripts/dev/bwd2s_check.py IDX=V[,IDX=V]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts', 'dev'))
import bench  # noqa: E402
from param_ab import timeit  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402


def main():
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    fw = lambda: _fused.dibr_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02, 30,  # noqa
                                     1000., 1e-8)
    feats, idx_, w, mask, state, ranges = fw()
    d = lambda: _fused.dibr_backward(inp['g_feat'], inp['g_mask'], idx_, w, inp['fvi'], inp['feat'],  # noqa
                                     inp['fnz'], mask, state, 7000., 1000., 1e-8, ranges)
    combo = [tuple(int(y) for y in kv.split('=')) for kv in sys.argv[1].split(',')]
    outs = {}
    for name, params in (('default', []), (sys.argv[1], combo), ('default2', [])):
        for i in range(16):
            lib.kl_dev_set_param(i, 0)
        for i, v in params:
            lib.kl_dev_set_param(i, v)
        r = [x.clone() for x in d() if x is not None]
        torch.cuda.synchronize()
        outs[name] = r
        print(f'{name}: dibr_backward {timeit(d):.1f} us', flush=True)
    for name in (sys.argv[1], 'default2'):
        same = all(torch.equal(a, b) for a, b in zip(outs['default'], outs[name]))
        print(f'{name} bit-equal to default: {same}', flush=True)
    for i in range(16):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
