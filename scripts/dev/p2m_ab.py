"""A/B timing of point_to_mesh_distance's forward on the cfg2 workload (100k points x 20k faces)
under dev params, outputs checked equal across the variants (development aid).
usage: python scripts/dev/p2m_ab.py 11=0 11=1 ...   (IDX=V[,IDX=V]; 0 = built-in value)"""
import ctypes
import os
import sys

ROOT0 = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('KAOLIN_HIP_LIB', os.path.join(ROOT0, 'kaolin-windows_amd', 'kaolin', '_lib', 'dev',
                                                     'libkaolin_hip.so'))
os.environ.setdefault('KAOLIN_NO_EXT', '1')
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _native as N  # noqa: E402


def main():
    import kaolin as kal
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    pts, fv = (t[None].contiguous() for t in bench.p2m_inputs("cuda")[:2])
    fn = lambda: kal.metrics.trianglemesh.point_to_mesh_distance(pts, fv)  # noqa: E731
    ref = None
    for c in sys.argv[1:] or ['11=0']:
        for i in range(32):
            lib.kl_dev_set_param(i, 0)
        for kv in c.split(','):
            i, v = (int(x) for x in kv.split('='))
            lib.kl_dev_set_param(i, v)
        out = fn()
        torch.cuda.synchronize()
        same = ref is None or all(torch.equal(a, b) for a, b in zip(out, ref))
        ref = ref if ref is not None else out
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f'params {c}: point_to_mesh {s.elapsed_time(e) / 10:.3f} ms, equal to the first: {same}', flush=True)
    for i in range(32):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
