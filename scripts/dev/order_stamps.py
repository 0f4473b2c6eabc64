"""Wall-clock phase stamps of tile_countorder2_kernel (dev aid; a `make STAMPS=1` library loaded
through KAOLIN_HIP_LIB).  Prints per block: count, prefix, placement in microseconds."""
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
# every stamping kernel writes into this buffer (per-wave stamps from 0); the order kernel's 8
# at kOrderStampsAt = 2^24 (csrc/common.h)
AT = 1 << 24
dbg = torch.zeros(AT + 64, dtype=torch.int64, device='cuda')
fw = lambda: _fused.dibr_forward(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02,  # noqa
                                 30, 1000., 1e-8)
for _ in range(3):
    fw()
lib.kl_dev_set_debug(ctypes.c_void_p(dbg.data_ptr()))
for rep in range(5):
    fw()
    torch.cuda.synchronize()
    d = dbg[AT:AT + 8].cpu().tolist()
    for blk in range(2):
        t = d[blk * 4:blk * 4 + 4]
        print(f'rep {rep} block {blk}: count {(t[1] - t[0]) / 100:.2f} us, prefix {(t[2] - t[1]) / 100:.2f} us, '
              f'place {(t[3] - t[2]) / 100:.2f} us, total {(t[3] - t[0]) / 100:.2f} us')
lib.kl_dev_set_debug(None)
