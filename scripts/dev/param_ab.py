"""A/B timing of dibr_backward / dibr_forward on the cfg3 workload under dev params
(development aid).  usage: python scripts/dev/param_ab.py IDX V1 V2 ...   (0 = built-in value)
       python scripts/dev/param_ab.py combo I=V,I=V ...  (several parameters per run)"""
import ctypes
import os
import sys

ROOT0 = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the dev controls live in the dev library (make dev); the compiled node would load the product one
os.environ.setdefault('KAOLIN_HIP_LIB', os.path.join(ROOT0, 'kaolin-windows_amd', 'kaolin', '_lib', 'dev',
                                                     'libkaolin_hip.so'))
os.environ.setdefault('KAOLIN_NO_EXT', '1')
import torch  # noqa: E402

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
    if sys.argv[1] == 'combo':
        combos = [[tuple(int(y) for y in kv.split('=')) for kv in c.split(',')] for c in sys.argv[2:]]
    else:
        combos = [[(int(sys.argv[1]), int(x))] for x in sys.argv[2:]] or [[(int(sys.argv[1]), 0)]]
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    for combo in combos:
        for i in range(32):
            lib.kl_dev_set_param(i, 0)
        for i, v in combo:
            lib.kl_dev_set_param(i, v)
        idx, v = combo[0][0], ','.join(f'{i}={x}' for i, x in combo)
        fw = lambda: _fused.dibr_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02, 30,  # noqa
                                         1000., 1e-8)
        feats, idx_, w, mask, state, ranges = fw()
        d = lambda: _fused.dibr_backward(inp['g_feat'], inp['g_mask'], idx_, w, inp['fvi'], inp['feat'],  # noqa
                                         inp['fnz'], mask, state, 7000., 1000., 1e-8, ranges)
        print(f'params {v}: dibr_forward {timeit(fw):.1f} us, dibr_backward {timeit(d):.1f} us', flush=True)
    for i in range(32):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
