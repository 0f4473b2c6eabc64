"""A/B timing of the _C contract soft-mask forward (bench.soft_mask_c_leg: binning + order + slot
kernel, cfg3 views, HIP events) under dev params, outputs checked equal across the variants
(development aid).  usage: python scripts/dev/csm_ab.py 16=0 16=1 ...   (IDX=V[,IDX=V]; 0 = built-in)"""
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
from kaolin import _native as N  # noqa: E402


def main():
    import kaolin as kal
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    inp = bench.dibr_inputs(bench.views_for_rank(0, 1, 4), torch.device('cuda'), 512, 512)
    inp['stats'] = bench.workload_stats(inp)
    with torch.no_grad():
        _, fidx = kal.render.mesh.rasterize(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'] >= 0)
        fm = inp['fvi'] * 1000.
        bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
    ref = None
    for rep in range(2):
        for c in sys.argv[1:] or ['16=0']:
            for i in range(32):
                lib.kl_dev_set_param(i, 0)
            for kv in c.split(','):
                i, v = (int(x) for x in kv.split('='))
                lib.kl_dev_set_param(i, v)
            out = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, fidx, 7000., 30, 1000.)
            torch.cuda.synchronize()
            same = ref is None or all(torch.equal(a, b) for a, b in zip(out, ref))
            if ref is None:
                ref = [t.clone() for t in out]
            del out
            r = bench.soft_mask_c_leg(inp, 10)
            print(f'params {c}: _C soft mask {r["ms"]} ms, frac {r["roofline"]["frac"]}, equal: {same}', flush=True)
    for i in range(32):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
