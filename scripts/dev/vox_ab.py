"""A/B timing of the cfg4 voxelgrid (trianglemeshes_to_voxelgrids, R=512) under dev params, grids
checked equal (development aid).  usage: python scripts/dev/vox_ab.py 21=0 21=1 ..."""
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
    verts, faces = bench.cfg4_inputs('cuda')
    fn = lambda: kal.ops.conversions.trianglemeshes_to_voxelgrids(verts[None], faces, 512)  # noqa: E731
    ref = None
    for rep in range(2):
        for c in sys.argv[1:] or ['21=0']:
            for i in range(32):
                lib.kl_dev_set_param(i, 0)
            for kv in c.split(','):
                i, v = (int(x) for x in kv.split('='))
                lib.kl_dev_set_param(i, v)
            g = fn()
            torch.cuda.synchronize()
            same = ref is None or torch.equal(g, ref)
            if ref is None:
                ref = g.clone()
            del g
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            print(f'params {c}: voxelgrid {s.elapsed_time(e) / 10:.4f} ms, equal: {same}', flush=True)
    for i in range(32):
        lib.kl_dev_set_param(i, 0)


if __name__ == '__main__':
    main()
