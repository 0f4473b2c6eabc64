"""Capture each DIB-R op alone in a HIP graph and replay it (sync + check after every
replay) -- isolates graph-replay problems to one op.  Development aid."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kaolin import _fused  # noqa: E402


def graph_of(fn):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def main():
    which = sys.argv[1:] or ['rf', 'sf', 'sb', 'rb']
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    H, W = inp['H'], inp['W']
    valid = inp['fnz'] >= 0
    feats, idx, w = _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)
    mask, prob, cidx, ctype, hits = _fused.soft_mask_forward(inp['fvi'], idx, 7000., 0.02, 30, 1000., with_hits=True)
    ops = {
        'rf': lambda: _fused.rasterize_forward(H, W, inp['fvz'], inp['fvi'], inp['feat'], valid, 1000., 1e-8)[1],
        'sf': lambda: _fused.soft_mask_forward(inp['fvi'], idx, 7000., 0.02, 30, 1000., with_hits=True)[2],
        'sb': lambda: _fused.soft_mask_backward(inp['g_mask'], mask, idx, prob, cidx, ctype, inp['fvi'], 7000.,
                                                1000., hits),
        'rb': lambda: _fused.rasterize_backward(inp['g_feat'], idx, w, inp['fvi'], inp['feat'], valid, 1000.,
                                                1e-8)[0],
    }
    for name in which:
        ref = ops[name]().clone()
        torch.cuda.synchronize()
        g, out = graph_of(ops[name])
        for r in range(30):
            g.replay()
            torch.cuda.synchronize()
            same = torch.equal(out, ref) if out.dtype != torch.float32 else torch.allclose(out, ref, 1e-4, 1e-5)
            if not same:
                print(name, 'replay', r, 'MISMATCH', flush=True)
                break
        print(name, 'ok', flush=True)


if __name__ == '__main__':
    main()
