"""Per-wave timing stamps of the compact soft-mask forward (development aid).

Runs soft_mask_forward_compact on the bench workload with the library's dev stamp buffer
(kl_dev_set_debug) and prints where the waves spend their cycles: selection (steps 1-2)
and evaluation (step 3), the slowest waves and the wall-clock span.
usage: python scripts/dev/stamps.py [knum] [rows per workgroup]
"""
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
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    lib = N.lib()
    lib.kl_dev_set_debug.argtypes = [ctypes.c_void_p]
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    lib.kl_dev_set_flags(rows << 8)
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    valid = inp['fnz'] >= 0
    _, idx, _ = _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)
    nwaves = 4 * H * (W // 64)
    dbg = torch.zeros(nwaves * 12, dtype=torch.int64, device='cuda')
    for _ in range(3):
        _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, K, 1000.)
    lib.kl_dev_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, K, 1000.)
    torch.cuda.synchronize()
    lib.kl_dev_set_debug(None)
    lib.kl_dev_set_flags(0)
    d = dbg.view(nwaves, 12).cpu().numpy().astype(np.uint64)
    if os.environ.get('STAMPS_DUMP'):
        np.save(os.environ['STAMPS_DUMP'], d)
    t0, t1, t2, w0, w1 = (d[:, k].astype(np.float64) for k in range(5))
    hits = d[:, 5].astype(np.int64)
    entries = (d[:, 6] >> np.uint64(32)).astype(np.int64)
    iters = (d[:, 6] & np.uint64(0xffffffff)).astype(np.int64)
    groups = (d[:, 7] >> np.uint64(32)).astype(np.int64)
    tile = (d[:, 7] & np.uint64(0xffffffff)).astype(np.int64)
    c_fill, c_walk, c_sync = (d[:, k].astype(np.float64) for k in (8, 9, 10))
    c_pf = (d[:, 11] >> np.uint64(42)).astype(np.float64)
    c_test = ((d[:, 11] >> np.uint64(21)) & np.uint64(0x1fffff)).astype(np.float64)
    c_s1 = (d[:, 11] & np.uint64(0x1fffff)).astype(np.float64)
    sel = t1 - t0
    ev = t2 - t1
    span_us = (w1.max() - w0.min()) / 100.0
    print(f'knum={K} rows/WG={rows or "default"} waves={nwaves} wall span {span_us:.1f} us')
    print(f'cycles/wave: selection mean {sel.mean():.0f} max {sel.max():.0f} | eval mean {ev.mean():.0f} '
          f'max {ev.max():.0f} | sum over waves {(sel.sum() + ev.sum()) / 1e6:.1f} Mcyc')
    print(f'totals: hits {hits.sum()} list entries {entries.sum()} face iterations {iters.sum()} '
          f'groups {groups.sum()}')
    start_us = (w0 - w0.min()) / 100.0
    end_us = (w1 - w0.min()) / 100.0
    for q in (0.5, 0.9, 0.99, 1.0):
        print(f'  wave end quantile {q}: {np.quantile(end_us, q):.1f} us, start {np.quantile(start_us, q):.1f} us')
    order = np.argsort(-(sel + ev))[:12]
    print(f'selection split (mean cycles): fill {c_fill.mean():.0f} walk {c_walk.mean():.0f} sync {c_sync.mean():.0f}')
    print(f'fill split (mean cycles): prefetch {c_pf.mean():.0f} test(+load wait) {c_test.mean():.0f} '
          f'sync1 {c_s1.mean():.0f}; heaviest wave: {c_pf[np.argmax(c_fill)]:.0f} {c_test[np.argmax(c_fill)]:.0f} '
          f'{c_s1[np.argmax(c_fill)]:.0f} of {c_fill.max():.0f}')
    print('slowest waves: tile  start_us end_us  sel_cyc (fill walk sync) eval_cyc  hits entries iters groups')
    for k in order:
        print(f'  {tile[k]:6d} {start_us[k]:7.1f} {end_us[k]:7.1f} {sel[k]:8.0f} ({c_fill[k]:7.0f} {c_walk[k]:7.0f} '
              f'{c_sync[k]:6.0f}) {ev[k]:8.0f} {hits[k]:5d} {entries[k]:6d} {iters[k]:5d} {groups[k]:4d}')
    # busy-wave histogram over time (concurrency)
    bins = np.linspace(0, span_us, 21)
    busy = [((start_us <= b) & (end_us > b)).sum() for b in bins[:-1]]
    print('waves in flight every 5% of the span:', busy)


if __name__ == '__main__':
    main()
