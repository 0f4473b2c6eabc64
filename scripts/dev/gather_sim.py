"""Lane-utilisation model of rasterize_bwd_gather2_kernel on the bench workload (development aid):
from the forward's face_idx and face ranges, each face's bbox pixels in row-major order, lane s of
its 8 taking elements s, s+8, ..., GATHER_BATCH per lane per round; a wave (8 faces) runs
max-over-faces rounds and, per round, max-over-lanes won pixels iterations.  Prints the share of
lane-iterations that add a won pixel, and the same for a won-pixel-balanced assignment."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused  # noqa: E402

GB = int(os.environ.get('GB', '3'))


def main():
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W, F = inp['H'], inp['W'], inp['F']
    f, idx, w, m, st, rg = _fused.dibr_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02,
                                                30, 1000., 1e-8)
    idx = idx.cpu().numpy()
    B = idx.shape[0]
    rg = rg.cpu().numpy().reshape(B * F, 2).astype(np.uint32)
    ix0, ix1 = (rg[:, 0] & 0xffff).astype(np.int64), (rg[:, 0] >> 16).astype(np.int64)
    iy0, iy1 = (rg[:, 1] & 0xffff).astype(np.int64), (rg[:, 1] >> 16).astype(np.int64)
    valid = (ix0 <= ix1) & (iy0 <= iy1)
    wd = np.where(valid, ix1 - ix0 + 1, 0)
    ht = np.where(valid, iy1 - iy0 + 1, 0)
    area = wd * ht
    small = valid & (area <= 1024)
    won_tot = np.bincount((idx + (np.arange(B)[:, None, None] * F)).reshape(-1)[idx.reshape(-1) >= 0], minlength=B * F)
    print(f'faces {B * F}, with range {valid.sum()}, small {small.sum()}, bbox px (small) {area[small].sum()}, '
          f'won px {won_tot.sum()} (small faces {won_tot[small].sum()})')
    iters = 0
    iters_bal = 0
    iters_round = 0
    rounds_tot = 0
    won_sum = 0
    nw = (B * F + 7) // 8
    for wv in range(nw):
        faces = range(wv * 8, min(wv * 8 + 8, B * F))
        fl = [t for t in faces if small[t]]
        if not fl:
            continue
        per_face_lane = []
        R = 0
        for t in fl:
            b = t // F
            ff = t - b * F
            sub = idx[b, iy0[t]:iy1[t] + 1, ix0[t]:ix1[t] + 1].reshape(-1) == ff
            n = sub.size
            r = -(-n // (8 * GB))
            R = max(R, r)
            pad = np.zeros(r * 8 * GB, bool)
            pad[:n] = sub
            per_face_lane.append(pad)
            won_sum += sub.sum()
        # per round: each face's lanes s take elements round*8*GB + s + 8*u, u < GB
        for rr in range(R):
            mx = 0
            mxb = 0
            for pad in per_face_lane:
                seg = pad[rr * 8 * GB:(rr + 1) * 8 * GB]
                if seg.size == 0:
                    continue
                lanes = seg.reshape(GB, 8).sum(0)
                mx = max(mx, lanes.max())
                mxb = max(mxb, -(-int(seg.sum()) // 8))
            iters += mx
            iters_round += mxb
        rounds_tot += R
        # balanced: each face's won pixels spread over its 8 lanes, the wave runs max over faces
        iters_bal += max(-(-int(p.sum()) // 8) for p in per_face_lane)
    print(f'GATHER_BATCH {GB}: waves with work {nw}, rounds {rounds_tot}, add iterations {iters}, '
          f'lane utilisation {won_sum / max(1, iters * 64):.3f}; balanced per face: iterations {iters_bal}, '
          f'utilisation {won_sum / max(1, iters_bal * 64):.3f}; balanced per face and round: iterations '
          f'{iters_round}, utilisation {won_sum / max(1, iters_round * 64):.3f}')


if __name__ == '__main__':
    main()
