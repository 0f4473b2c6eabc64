"""Wall-clock phase stamps of tile_countorder_chip_kernel (dev aid; a `make STAMPS=1` library
loaded through KAOLIN_HIP_LIB).  Prints the count workgroups' (count, publish) and each bitmap's
workgroup 0's (barrier passed, prefix, placement) phases in microseconds from the earliest start."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402

lib = N.lib()
lib.kl_dev_set_debug.argtypes = [ctypes.c_void_p]
inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
AT = 1 << 24  # kOrderStampsAt (csrc/common.h)
dbg = torch.zeros(AT + 128, dtype=torch.int64, device='cuda')
fw = lambda: _fused.dibr_forward(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02,  # noqa
                                 30, 1000., 1e-8)
for _ in range(3):
    fw()
lib.kl_dev_set_debug(ctypes.c_void_p(dbg.data_ptr()))
for rep in range(4):
    dbg.zero_()
    fw()
    torch.cuda.synchronize()
    d = dbg[AT:AT + 72].cpu().tolist()
    t0 = min(x for x in d if x)
    us = lambda x: (x - t0) / 100 if x else float('nan')  # noqa: E731
    cw = [(us(d[4 * b]), us(d[4 * b + 1]), us(d[4 * b + 2])) for b in range(16) if d[4 * b]]
    print(f'rep {rep}: count workgroups (start, counted, arrived) us: ' +
          ' '.join(f'({a:.1f},{b:.1f},{c:.1f})' for a, b, c in cw))
    for w in range(2):
        s = d[64 + 4 * w:64 + 4 * w + 4]
        print(f'  bitmap {w} workgroup 0: barrier passed {us(s[0]):.2f} histograms {us(s[3]):.2f} prefix {us(s[1]):.2f} placed {us(s[2]):.2f} us')
lib.kl_dev_set_debug(None)
