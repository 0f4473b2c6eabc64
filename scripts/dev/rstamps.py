"""Per-wave timing stamps of the tile rasterizer forward (development aid).

Runs the fused rasterize_forward on the bench workload with the library's dev stamp
buffer (kl_dev_set_debug) and prints fill / walk cycles, candidate visits and the tail.
usage: python scripts/dev/rstamps.py [split_from:split_log2 ...]   (default 5:2; 31:0 = no split,
       "grid" = grid order without split)
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
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    for a in (sys.argv[1:] or ['5:2']):
        if a == 'grid':
            run(inp, 1 << 12, 0, a)


        else:
            sf, sl = (int(x) for x in a.split(':'))
            run(inp, (sf << 16) | (sl << 21), sl, a)


def run(inp, flags, sl, label):
    lib = N.lib()
    lib.kl_dev_set_debug.argtypes = [ctypes.c_void_p]
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    lib.kl_dev_set_flags(flags)
    H, W = inp['H'], inp['W']
    B = inp['fvi'].shape[0]
    nt = B * (H // 8) * (W // 64)
    nw = (nt << sl) * 8
    dbg = torch.zeros(nw * 15, dtype=torch.int64, device='cuda')
    args = (H, W, inp['fvz'], inp['fvi'], inp['feat'], None, 1000., 1e-8)
    for _ in range(3):
        _fused.rasterize_forward(*args, face_normals_z=inp['fnz'])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        _fused.rasterize_forward(*args, face_normals_z=inp['fnz'])
    e1.record()
    torch.cuda.synchronize()
    print(f'=== {label}: rasterize_forward {e0.elapsed_time(e1) / 20 * 1000:.1f} us per call')
    lib.kl_dev_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    _fused.rasterize_forward(*args, face_normals_z=inp['fnz'])
    torch.cuda.synchronize()
    lib.kl_dev_set_debug(None)
    lib.kl_dev_set_flags(0)
    if not bool(dbg.any()):
        print('  (no stamps: build the library with `make -B -C kaolin-windows_amd/csrc STAMPS=1`)')
        return
    d = dbg[:nw * 8].view(nw, 8).cpu().numpy().astype(np.uint64)
    v = dbg[nw * 8:nw * 10].view(nw, 2).cpu().numpy().astype(np.int64)
    ph = dbg[nw * 10:].view(nw, 5).cpu().numpy().astype(np.float64)
    live = d[:, 3] != 0  # workgroups past the item count write no stamps
    d, v, ph = d[live], v[live], ph[live]
    nw = int(live.sum())
    t0, t1, w0, w1, cf, cw = (d[:, k].astype(np.float64) for k in range(6))
    entries = (d[:, 6] >> np.uint64(32)).astype(np.int64)
    iters = (d[:, 6] & np.uint64(0xffffffff)).astype(np.int64)
    steps = (d[:, 7] >> np.uint64(32)).astype(np.int64)
    tile = (d[:, 7] & np.uint64(0xffffffff)).astype(np.int64)
    visits, vmax = v[:, 0], v[:, 1]
    cyc = t1 - t0
    span = (w1.max() - w0.min()) / 100.0
    print(f'waves {nw} wall span {span:.1f} us; cycles/wave mean {cyc.mean():.0f} max {cyc.max():.0f}')
    print(f'fill mean {cf.mean():.0f} max {cf.max():.0f} | walk mean {cw.mean():.0f} max {cw.max():.0f}')
    print('fill phases mean (issue, test, sync1, write+sync2, wait for loads):', ph.mean(0).round(0), 'slowest wave:',
          ph[np.argmax(cyc)].round(0))
    print(f'totals: list entries {entries.sum()} (per tile {entries.sum() / nt:.0f}) steps/tile {steps.mean():.2f} '
          f'visits {visits.sum()} wave iterations {iters.sum()} (x64 = {iters.sum() * 64}) '
          f'lane efficiency {visits.sum() / max(1, iters.sum() * 64):.3f}')
    start = (w0 - w0.min()) / 100.0
    end = (w1 - w0.min()) / 100.0
    for q in (0.5, 0.9, 0.99, 1.0):
        print(f'  wave end quantile {q}: {np.quantile(end, q):.1f} us, start {np.quantile(start, q):.1f} us')
    order = np.argsort(-cyc)[:12]
    print('slowest waves: tile start_us end_us cycles (fill walk) entries iters visits maxlane steps')
    for k in order:
        print(f'  {tile[k]:6d} {start[k]:7.1f} {end[k]:7.1f} {cyc[k]:8.0f} ({cf[k]:7.0f} {cw[k]:7.0f}) '
              f'{entries[k]:6d} {iters[k]:6d} {visits[k]:7d} {vmax[k]:5d} {steps[k]:4d}')
    bins = np.linspace(0, span, 21)
    print('waves in flight every 5% of the span:', [int(((start <= b) & (end > b)).sum()) for b in bins[:-1]])


if __name__ == '__main__':
    main()
