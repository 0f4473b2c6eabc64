"""Per-wave timing stamps of the compact soft-mask forward (development aid).

Runs soft_mask_forward_compact on the bench workload with the library's dev stamp buffer
(kl_dev_set_debug; a `make STAMPS=1` build, loaded through KAOLIN_HIP_LIB) and prints where
the waves spend their cycles: walk (step 1) and evaluation + mask (steps 2-3), the slowest
rows and the wall-clock span.  10 stamps per wave (softtile.hip, soft_tile_fwd_kernel).
usage: python scripts/dev/stamps.py [knum]      (STAMPS_DUMP=path.npy saves the raw stamps)
"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused, _native as N  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    lib = N.lib()
    lib.kl_dev_set_debug.argtypes = [ctypes.c_void_p]
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    flags = int(os.environ.get('STAMPS_FLAGS', '0'), 0)
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    params = [int(x) for x in os.environ.get('STAMPS_PARAMS', '').split(',') if x]
    for k, v in enumerate(params):  # SoftSplit b4, b8, cap4, cap8 (tileorder.h)
        lib.kl_dev_set_param(k, v)
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    valid = inp['fnz'] >= 0
    _, idx, _ = _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)
    nwaves = 4 * (H // 8) * (W // 64) * 8 * 4  # grid bound (tiles x 8 parts x 4 waves)
    dbg = torch.zeros(max(nwaves * 10, (1 << 24) + 64), dtype=torch.int64, device="cuda")  # order stamps at 2^24
    for _ in range(3):
        _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, K, 1000.)
    lib.kl_dev_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    lib.kl_dev_set_flags(flags)
    _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, K, 1000.)
    torch.cuda.synchronize()
    lib.kl_dev_set_flags(0)
    lib.kl_dev_set_debug(None)
    d = dbg[:nwaves * 10].view(nwaves, 10).cpu().numpy().astype(np.uint64)
    d = d[d[:, 3] != 0]
    if os.environ.get('STAMPS_DUMP'):
        np.save(os.environ['STAMPS_DUMP'], d)
    t0, t1, t2, w0, w1 = (d[:, k].astype(np.float64) for k in range(5))
    hits = d[:, 5].astype(np.int64)
    nch = (d[:, 6] >> np.uint64(32)).astype(np.int64)
    qi = (d[:, 6] & np.uint64(0xff)).astype(np.int64)
    Q = ((d[:, 6] >> np.uint64(8)) & np.uint64(0xff)).astype(np.int64)
    row = (d[:, 7] >> np.uint64(32)).astype(np.int64)
    tile = (d[:, 7] & np.uint64(0xffffffff)).astype(np.int64)
    walk, ev = t1 - t0, t2 - t1
    fill = d[:, 8].astype(np.float64)
    start_us = (w0 - w0.min()) / 100.0
    end_us = (w1 - w0.min()) / 100.0
    span = end_us.max()
    print(f'knum={K} waves={len(d)} wall span {span:.1f} us; waves by Q: '
          f'{dict(collections.Counter(Q.tolist()))}')
    lead = qi == 0
    hot = lead & (hits > 0)
    print(f'rows with hits: {hot.sum()}  walk cycles mean {walk[hot].mean():.0f} max {walk[hot].max():.0f} | '
          f'eval+mask mean {ev[hot].mean():.0f} max {ev[hot].max():.0f} | fill (in walk) mean {fill[hot].mean():.0f} '
          f'max {fill[hot].max():.0f} | list entries mean {nch[hot].mean():.1f}')
    print(f'rows without hits: {(lead & (hits == 0)).sum()}  duration mean '
          f'{(end_us - start_us)[lead & (hits == 0)].mean():.2f} us')
    for q in (0.5, 0.9, 0.99, 1.0):
        print(f'  wave end quantile {q}: {np.quantile(end_us, q):.1f} us, start {np.quantile(start_us, q):.1f} us')
    order = np.argsort(-(end_us - start_us) * lead)[:12]
    print('slowest rows: tile row Q start_us end_us walk_cyc (fill_cyc) eval_cyc hits chunks')
    for k in order:
        print(f'  {tile[k]:6d} {row[k]:4d} {Q[k]} {start_us[k]:7.1f} {end_us[k]:7.1f} {walk[k]:8.0f} ({fill[k]:6.0f}) '
              f'{ev[k]:8.0f} {hits[k]:5d} {nch[k]:4d}')
    bins = np.linspace(0, span, 21)
    busy = [int(((start_us <= b) & (end_us > b)).sum()) for b in bins[:-1]]
    print('waves in flight every 5% of the span:', busy)


if __name__ == '__main__':
    main()
