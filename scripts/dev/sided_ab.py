"""A/B of sided_distance's forward on cfg1 (2,048 x 2,048 f32): p2's tiles split over workgroups
(default) against one pass (dev param 23 = 1); kernel-only and front-end timings (development aid)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
import kaolin as kal  # noqa: E402
from kaolin import _native as N  # noqa: E402


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
    lib = N.lib()
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    g = torch.Generator().manual_seed(0)
    p1 = torch.rand((1, 2048, 3), generator=g).cuda()
    p2 = torch.rand((1, 2048, 3), generator=g).cuda()
    dist = torch.empty((1, 2048), device='cuda')
    idx = torch.empty((1, 2048), dtype=torch.long, device='cuda')
    st = N.stream_of(p1.device)
    raw = lambda: lib.kl_sided_distance_forward(N.dtype_code(p1.dtype), 1, 2048, 2048, N.ptr(p1), N.ptr(p2),  # noqa
                                                N.ptr(dist), ctypes.c_void_p(idx.data_ptr()), st)
    front = lambda: kal.metrics.pointcloud.sided_distance(p1, p2)  # noqa: E731
    for v in (0, 1, 0, 1):
        lib.kl_dev_set_param(23, v)
        print(f'param 23={v}: C call {timeit(raw):.1f} us, front-end {timeit(front):.1f} us', flush=True)
    lib.kl_dev_set_param(23, 0)


if __name__ == '__main__':
    main()
