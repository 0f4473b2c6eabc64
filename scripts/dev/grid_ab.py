"""dibr_forward at cfg3 with the raster / soft grids cut (dev params 28 / 29 = G), outputs compared
with the default launch (development aid): python scripts/dev/grid_ab.py 28=3000 29=4000 ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('KAOLIN_HIP_LIB', os.path.join(ROOT, 'kaolin-windows_amd', 'kaolin', '_lib', 'dev',
                                                     'libkaolin_hip.so'))
os.environ.setdefault('KAOLIN_NO_EXT', '1')
import torch  # noqa: E402

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402
from param_ab import timeit  # noqa: E402


def main():
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    fw = lambda: _fused.dibr_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02, 30,  # noqa
                                     1000., 1e-8)
    ref = [t.clone() for t in fw()[:4]]
    for rep in range(2):
        for c in ['0=0'] + sys.argv[1:]:
            for i in range(32):
                lib.kl_dev_set_param(i, 0)
            for kv in c.split(','):
                i, v = (int(x) for x in kv.split('='))
                lib.kl_dev_set_param(i, v)
            out = fw()
            torch.cuda.synchronize()
            same = all(torch.equal(a, b) for a, b in zip(out[:4], ref))
            print(f'params {c}: dibr_forward {timeit(fw):.1f} us, equal: {same}', flush=True)
    for i in range(32):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
