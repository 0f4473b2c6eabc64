"""Host-side cost of the eager cfg3 step (development aid).

Times the eager step (no op timer), the host time per step with the GPU kept busy, and a
cProfile of the step's Python.  usage: python scripts/dev/host_profile.py [steps]
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    inp = bench.dibr_inputs([0.0, 1.5707963, 3.1415927, 4.712389], 'cuda')
    step = lambda: bench.dibr_step(inp, 1)  # noqa: E731
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'eager: {(t2 - t0) / n * 1e6:.1f} us/step (host loop {(t1 - t0) / n * 1e6:.1f} us/step)')
    # host-only cost of the pieces
    fvi = inp['fvi'].detach().requires_grad_(True)
    feat = inp['feat'].detach().requires_grad_(True)
    import kaolin as kal
    reps = 200
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = kal.render.mesh.dibr_rasterization(inp['H'], inp['W'], inp['fvz'], fvi, feat, inp['fnz'],
                                                 sigmainv=7000, boxlen=0.02, knum=30, multiplier=1000, eps=1e-8)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f'forward call: {(t1 - t0) / reps * 1e6:.1f} us host')
    t0 = time.perf_counter()
    for _ in range(reps):
        torch.autograd.backward([out[0], out[1]], [inp['g_feat'], inp['g_mask']], retain_graph=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f'backward call: {(t1 - t0) / reps * 1e6:.1f} us host')
    from kaolin import _fused, _native as N
    f = _fused.dibr_forward(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02, 30,
                            1000., 1e-8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f = _fused.dibr_forward(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'], 7000., 0.02,
                                30, 1000., 1e-8)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f'_fused.dibr_forward: {(t1 - t0) / reps * 1e6:.1f} us host')
    feats, idx, w, mask, state, ranges = f
    t0 = time.perf_counter()
    for _ in range(reps):
        _fused.dibr_backward(inp['g_feat'], inp['g_mask'], idx, w, inp['fvi'], inp['feat'], inp['fnz'], mask, state,
                             7000., 1000., 1e-8, ranges)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f'_fused.dibr_backward: {(t1 - t0) / reps * 1e6:.1f} us host')
    x = torch.empty(16, device='cuda')
    ws = torch.zeros(N.lib().kl_loss_dot2_workspace_bytes(), dtype=torch.uint8, device='cuda')
    out = torch.empty(1, device='cuda')
    args = (N.ptr(x), N.ptr(x), 16, N.ptr(x), N.ptr(x), 16, N.ptr(ws), N.ptr(out), N.stream_of(x.device))
    lib = N.lib()
    t0 = time.perf_counter()
    for _ in range(1000):
        lib.kl_loss_dot2(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f'kl_loss_dot2 (2 launches, prebuilt args): {(t1 - t0) / 1000 * 1e6:.1f} us host')
    t0 = time.perf_counter()
    for _ in range(1000):
        torch.empty((4, 512, 512, 3), device='cuda')
    t1 = time.perf_counter()
    print(f'torch.empty: {(t1 - t0) / 1000 * 1e6:.2f} us host')
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(30)


if __name__ == '__main__':
    main()
