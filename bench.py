"""bench.py -- DIB-R 512^2 forward+backward throughput (Mpixels/s) on MI355X, plus
point_to_mesh_distance (Mpairs/s), per BASELINE.json.

Workload (BASELINE.json configs[2]), per rank:
  UV sphere 126 lat x 200 lon = 50,000 faces, radius 0.9*(1+0.01*N(0,1)) per vertex
  (seed 0); 4 views (azimuth 90 deg apart, distance 3, look-at 0, up +y, fovy pi/4);
  features D=3 = [uv, 1]; dibr_rasterization(512, 512, ..., sigmainv=7000,
  boxlen=0.02, knum=30, multiplier=1000, eps=1e-8); loss = <feat, g_feat> +
  <soft_mask, g_mask> with g ~ U[0,1] (seed 1); backward to face_vertices_image and
  face_features.  One step = that forward + backward over the rank's 4 views.
Multi-GPU: one process per GPU (torchrun); each rank renders its own 4 views of the
replicated mesh (weak scaling, global batch 4N), per-shard losses are all-gathered
over RCCL each step; time = max over ranks.

Also reported: p2m (configs[1]: 100k points vs 20k faces, forward) Mpairs/s, the §8f
sub-benches (deftet_sparse_render fwd+bwd on the same views, check_sign 1M points), the
roofline of the dominant op (HIP events on its stream over the timed region) and a
CPU baseline (the C oracle, 1 thread, on a stated row sample of view 0).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
sys.path.insert(0, ROOT)

import kaolin as kal  # noqa: E402
from kaolin import _native  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector peak


def uv_sphere(n_lat, n_lon, device, dtype=torch.float32, seed=0):
    lat = torch.linspace(0, math.pi, n_lat + 1, dtype=torch.float64)[1:-1]
    lon = torch.arange(n_lon, dtype=torch.float64) * (2 * math.pi / n_lon)
    ring = torch.stack([torch.sin(lat)[:, None] * torch.cos(lon)[None], torch.cos(lat)[:, None].expand(-1, n_lon),
                        torch.sin(lat)[:, None] * torch.sin(lon)[None]], -1).reshape(-1, 3)
    verts = torch.cat([torch.tensor([[0., 1., 0.]], dtype=torch.float64), ring,
                       torch.tensor([[0., -1., 0.]], dtype=torch.float64)])
    g = torch.Generator().manual_seed(seed)
    verts = verts * (0.9 * (1 + 0.01 * torch.randn((verts.shape[0], 1), generator=g, dtype=torch.float64)))
    nr = n_lat - 1
    j = torch.arange(n_lon)
    jn = (j + 1) % n_lon
    top = torch.stack([torch.zeros_like(j), 1 + jn, 1 + j], -1)
    i = torch.arange(nr - 1)[:, None]
    a = 1 + i * n_lon + j
    b = 1 + i * n_lon + jn
    c = a + n_lon
    d = b + n_lon
    mid = torch.stack([torch.stack([a, b, d], -1), torch.stack([a, d, c], -1)], 2).reshape(-1, 3)
    last = 1 + nr * n_lon
    bot = torch.stack([1 + (nr - 1) * n_lon + j, 1 + (nr - 1) * n_lon + jn, torch.full_like(j, last)], -1)
    faces = torch.cat([top, mid, bot]).to(device)
    return verts.to(device=device, dtype=dtype), faces


def dibr_inputs(views, device, H=512, W=512):
    verts, faces = uv_sphere(126, 200, device)
    assert faces.shape[0] == 50000
    B = len(views)
    az = torch.tensor(views, dtype=torch.float32, device=device)
    cam = torch.stack([3 * torch.sin(az), torch.zeros_like(az), 3 * torch.cos(az)], -1)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(
        cam, torch.zeros_like(cam), torch.tensor([[0., 1., 0.]], device=device).repeat(B, 1))
    v = verts.unsqueeze(0).repeat(B, 1, 1)
    vc = kal.render.camera.rotate_translate_points(v, rot, trans)
    proj = kal.render.camera.generate_perspective_projection(math.pi / 4).to(device)
    vi = kal.render.camera.perspective_camera(vc, proj)
    fvc = kal.ops.mesh.index_vertices_by_faces(vc, faces)
    fvz = fvc[..., -1].contiguous()
    fvi = kal.ops.mesh.index_vertices_by_faces(vi, faces).contiguous()
    fnz = kal.ops.mesh.face_normals(fvc, unit=True)[..., -1].contiguous()
    # sphere parametrisation uv + constant 1 (the tutorial's [uv, mask] features)
    u = torch.atan2(verts[:, 2], verts[:, 0]) / (2 * math.pi) + 0.5
    vv = torch.acos(torch.clamp(verts[:, 1] / verts.norm(dim=1), -1, 1)) / math.pi
    vfeat = torch.stack([u, vv, torch.ones_like(u)], -1).unsqueeze(0).repeat(B, 1, 1)
    feat = kal.ops.mesh.index_vertices_by_faces(vfeat, faces).contiguous()
    g = torch.Generator(device='cpu').manual_seed(1)
    g_feat = torch.rand((B, H, W, 3), generator=g).to(device)
    g_mask = torch.rand((B, H, W), generator=g).to(device)
    return dict(fvz=fvz, fvi=fvi, feat=feat, fnz=fnz, g_feat=g_feat, g_mask=g_mask, H=H, W=W, F=faces.shape[0])


def views_for_rank(rank, world, per_rank):
    """Contiguous shard of the world's per_rank*world azimuths (weak scaling: fixed per rank)."""
    n = per_rank * world
    return [2 * math.pi * (rank * per_rank + k) / n for k in range(per_rank)]


def gather_losses(loss, world):
    """The step's only collective: all_gather of the per-shard scalar losses."""
    out = [torch.empty_like(loss) for _ in range(world)]
    dist.all_gather(out, loss.detach())
    return torch.stack(out)


def max_over_ranks(elapsed, device, world):
    if world == 1:
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def loss_dot2(a, ga, b, gb, inp):
    """L = <a, ga> + <b, gb> in one launch (kl_loss_dot2: fp64 accumulation, deterministic; two
    torch.dot calls plus their add were four launches, ~25 us per step)."""
    if os.environ.get('KL_BENCH_TORCH_LOSS'):  # dev A/B: the two-torch.dot loss
        with torch.no_grad():
            return torch.dot(a.reshape(-1), ga.reshape(-1)) + torch.dot(b.reshape(-1), gb.reshape(-1))
    if 'loss_ws' not in inp:
        inp['loss_ws'] = torch.zeros(_native.lib().kl_loss_dot2_workspace_bytes(), dtype=torch.uint8, device=a.device)
    out = torch.empty(1, dtype=torch.float32, device=a.device)
    _native.check(_native.lib().kl_loss_dot2(_native.ptr(a), _native.ptr(ga), a.numel(), _native.ptr(b),
                                             _native.ptr(gb), b.numel(), _native.ptr(inp['loss_ws']),
                                             _native.ptr(out), _native.stream_of(a.device)), 'kl_loss_dot2')
    return out[0]


def dibr_compute(inp):
    """dibr_rasterization forward + the loss L = <features, g_feat> + <soft_mask, g_mask> + backward
    (everything but the collective).  dL/dfeatures = g_feat and dL/dsoft_mask = g_mask exactly, so the
    backward is driven with them directly (torch.autograd.backward) -- the same gradients as
    L.backward() without the broadcast kernels of the sum's backward; L itself is two dot products
    (one fused launch, loss_dot2)."""
    fvi = inp['fvi'].detach().requires_grad_(True)
    feat = inp['feat'].detach().requires_grad_(True)
    feats, mask, idx = kal.render.mesh.dibr_rasterization(inp['H'], inp['W'], inp['fvz'], fvi, feat, inp['fnz'],
                                                          sigmainv=7000, boxlen=0.02, knum=30, multiplier=1000,
                                                          eps=1e-8)
    loss = loss_dot2(feats.detach(), inp['g_feat'], mask.detach(), inp['g_mask'], inp)
    torch.autograd.backward([feats, mask], [inp['g_feat'], inp['g_mask']])
    return loss, fvi.grad, feat.grad, mask, idx


def dibr_step(inp, world):
    loss, gfvi, gfeat, mask, idx = dibr_compute(inp)
    if world > 1:  # per-shard losses all-gathered over RCCL / xGMI
        gather_losses(loss, world)
    return gfvi, gfeat, mask, idx


def graphed_step(inp, world):
    """The same step with dibr_compute captured once in a HIP graph (its ~35 launches
    replayed as one); the loss all_gather stays an eager RCCL call.  Inputs are static
    buffers, as in a training loop that copies each batch into them."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            dibr_compute(inp)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_out = dibr_compute(inp)

    def step():
        graph.replay()
        if world > 1:
            gather_losses(static_out[0], world)
        return static_out
    return step, static_out


def op_bytes(name, inp, stats):
    """Algorithmic HBM bytes of one call of each op (SURVEY.md §8d decomposition, fp32)."""
    B, H, W = inp['fvz'].shape[0], inp['H'], inp['W']
    F = inp['F']
    D, K, s = 3, 30, 4
    px = B * H * W
    nv = stats['valid_faces']
    if name == 'dibr_soft_mask_forward_cuda':
        # the _C contract: read sel (8/px) + faces (fvi 24 + bbox 16); write mask + K x (prob 4 + idx 8 + type 1)
        return px * (8 + s + K * (s + 8 + 1)) + B * F * (6 * s + 4 * s)
    if name == 'dibr_soft_mask_forward':
        # compact state: read sel (8/px), faces (fvi 24 + bbox write/read 2 x 16); write mask + hits (4 + 1)
        # per px and one record (face 4 + prob 4) per hit
        return px * (8 + s + 1) + stats['hits'] * (4 + s) + B * F * (6 * s + 2 * 4 * s)
    if name == 'dibr_soft_mask_backward_cuda':
        # read grad, mask, sel per px + used slots (+ terminator) of uncovered px; write grad (B,F,3,2)
        return px * (s + s + 8) + stats['slot_reads'] * (8 + s + 1) + B * F * 6 * s * 2
    if name == 'dibr_soft_mask_backward':
        # compact state: read grad, mask, hits per px + one record per hit + faces; add into grad (B,F,3,2)
        return px * (s + s + 1) + stats['hits'] * (4 + s) + B * F * 6 * s * 2
    if name == 'packed_rasterize_forward_cuda':
        return px * (8 + 3 * s + D * s) + nv * (3 * s + 6 * s + 4 * s + 3 * D * s)
    if name == 'dibr_rasterize_forward':
        # write idx/weights/features; read (valid mask + z + image coords) of all faces + features of valid ones
        return px * (8 + 3 * s + D * s) + B * F * (1 + 3 * s + 6 * s) + nv * 3 * D * s
    if name == 'dibr_forward':
        # both of the above in one call: the faces are read once for both
        return (op_bytes('dibr_rasterize_forward', inp, stats) + op_bytes('dibr_soft_mask_forward', inp, stats)
                - B * F * 6 * s)
    if name in ('rasterize_backward_cuda', 'dibr_rasterize_backward'):
        return px * (8 + 3 * s + D * s) + B * F * (6 * s + 3 * D * s) * 2
    return None


def survey_step_bytes(inp, stats):
    """SURVEY.md §8d cfg3 figure for one fwd+bwd step, in the reference's data layout:
    B*H*W*(60 + 8D + 13K + u*(8 + 13*kbar)) + B*F*(164 + 36D), u = uncovered fraction and
    kbar = mean used soft-mask slots (+ terminator) over uncovered pixels, both measured."""
    B, H, W, F = inp['fvz'].shape[0], inp['H'], inp['W'], inp['F']
    D, K = 3, 30
    u, kbar = stats['uncovered'], stats['mean_slots']
    return int(B * H * W * (60 + 8 * D + 13 * K + u * (8 + 13 * kbar)) + B * F * (164 + 36 * D))


# kernels launched by each timed op (the roofline's traffic sums their PMC bytes)
OP_KERNELS = {
    'dibr_soft_mask_forward': ('bin_faces_kernel<float, kl::SoftSrc', 'tile_bucket_kernel', 'tile_order_kernel',
                               'soft_tile_fwd_kernel<float'),
    'dibr_soft_mask_backward': ('soft_bwd_plan_kernel', 'soft_tile_bwd_kernel<float'),
    'dibr_rasterize_forward': ('raster_bin_kernel<float, 2>', 'tile_bucket_kernel', 'tile_order_kernel',
                               'raster_tile_kernel<float'),
    'dibr_forward': ('raster_bin_kernel<float, 2>', 'tile_bucket2_kernel', 'tile_order2_kernel', 'raster_tile_kernel<float',
                     'soft_tile_fwd_kernel<float'),
    'dibr_rasterize_backward': ('rasterize_bwd_gather_kernel<float', 'rasterize_bwd_bigface_kernel<float'),
}


def pmc_traffic(op):
    """HBM bytes per call of `op` from the committed PMC summary (scripts/pmc_traffic.py), or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'pmc_traffic.json')
    if op not in OP_KERNELS or not os.path.exists(path):
        return None
    kern = json.load(open(path))['kernels']
    total, found = 0, 0
    for pref in OP_KERNELS[op]:
        for name, v in kern.items():
            if pref in name:
                total += v['hbm_bytes']
                found += 1
                break
    return total if found == len(OP_KERNELS[op]) else None


def timed_loop(fn, steps, world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def cpu_baseline(inp, row_step):
    """The C oracle (1 thread) on all the rank's views, every `row_step`-th pixel row:
    rasterize fwd, soft mask fwd, soft mask bwd, rasterize bwd."""
    import numpy as np
    from oracle import oracle as orc
    A = lambda t: t.detach().cpu().numpy()  # noqa: E731
    fvz, fvi, feat, fnz = (A(inp[k]) for k in ('fvz', 'fvi', 'feat', 'fnz'))
    H, W = inp['H'], inp['W']
    orc.lib().or_set_row_step(row_step)
    try:
        t0 = time.perf_counter()
        of, oi, ow = orc.rasterize(H, W, fvz, fvi, feat, valid_faces=fnz >= 0)
        fm, bb = orc.soft_mask_bboxes(fvi, 0.02, 1000.)
        om, op, oci, oct_ = orc.dibr_soft_mask_forward(fm, bb, oi, 7000., 30, 1000.)
        orc.dibr_soft_mask_backward(np.ones_like(om), om, oi, op, oci, oct_, fm, 7000., 1000.)
        orc.rasterize_backward(np.ones_like(of), oi, ow, fvi, feat, 1e-8)
        dt = time.perf_counter() - t0
    finally:
        orc.lib().or_set_row_step(1)
    rows = len(range(0, H, row_step)) * fvz.shape[0]
    return rows * W / dt / 1e6, rows * W, dt


def p2m_bench(device, steps):
    g = torch.Generator().manual_seed(0)
    pts = torch.randn((100000, 3), generator=g).to(device)
    fv = torch.randn((20000, 3, 3), generator=g).to(device)
    d = torch.empty(100000, device=device)
    i = torch.empty(100000, dtype=torch.long, device=device)
    t = torch.empty(100000, dtype=torch.int32, device=device)
    f = lambda: kal._C.metrics.unbatched_triangle_distance_forward_cuda(pts, fv, d, i, t)  # noqa: E731
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / steps
    return 100000 * 20000 / (ms * 1e-3) / 1e6, ms


def _event_ms(fn, steps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def deftet_bench(inp, steps, knum=8):
    """deftet_sparse_render fwd+bwd on the cfg3 mesh and views: every
    pixel centre of the 512x512 grid, depth range = the mesh's z span, knum=8 (a covered pixel
    of the sphere holds its front and back faces)."""
    fvz, fvi, feat, H, W = inp['fvz'], inp['fvi'], inp['feat'], inp['H'], inp['W']
    B, dev = fvz.shape[0], fvz.device
    x = (2 * torch.arange(W, device=dev, dtype=torch.float32) + 1 - W) / W
    y = (H - 2 * torch.arange(H, device=dev, dtype=torch.float32) - 1.) / H
    pix = torch.stack([x.view(1, -1).expand(H, W), y.view(-1, 1).expand(H, W)], -1).reshape(1, -1, 2)
    pix = pix.expand(B, -1, -1).contiguous()
    zmin, zmax = fvz.reshape(B, -1).min(1)[0], fvz.reshape(B, -1).max(1)[0]
    rr = torch.stack([zmin - 1e-2, zmax + 1e-2], -1).unsqueeze(1).expand(-1, H * W, -1).contiguous()
    fvi_r = fvi.detach().clone().requires_grad_(True)
    feat_r = feat.detach().clone().requires_grad_(True)
    g = torch.rand((B, H * W, knum, feat.shape[-1]), generator=torch.Generator().manual_seed(2)).to(dev)
    render = kal.render.mesh.deftet_sparse_render

    def fwd():
        return render(pix, rr, fvz, fvi_r, feat_r, knum)

    def step():
        out, _ = fwd()
        torch.autograd.grad(out, [fvi_r, feat_r], g)

    ms_fwd = _event_ms(lambda: fwd(), steps)
    ms = _event_ms(step, steps)
    _, idx = fwd()
    hits = int((idx >= 0).sum())
    return {'metric': 'deftet_sparse_render fwd+bwd Mpixels/s (4 views, 512x512, 50k faces, knum=8, f32)',
            'value': round(B * H * W / (ms * 1e-3) / 1e6, 1), 'ms': round(ms, 3), 'fwd_ms': round(ms_fwd, 3),
            'hits': hits}


def check_sign_bench(device, steps, n_points=1000000):
    """check_sign: the cfg3 sphere (50k faces) vs 1M points in [-1,1]^3."""
    verts, faces = uv_sphere(126, 200, device)
    g = torch.Generator().manual_seed(3)
    pts = (torch.rand((1, n_points, 3), generator=g) * 2 - 1).to(device)
    v = verts.unsqueeze(0).contiguous()
    ms = _event_ms(lambda: kal.ops.mesh.check_sign(v, faces, pts), steps)
    return {'metric': 'check_sign Mpoints/s (1M points vs 50k-face sphere, f32)',
            'value': round(n_points / (ms * 1e-3) / 1e6, 1), 'ms': round(ms, 3),
            'nominal_mpairs_per_s': round(n_points * faces.shape[0] / (ms * 1e-3) / 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--cpu-row-step', type=int, default=2)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-p2m', action='store_true')
    ap.add_argument('--no-extra', action='store_true', help='skip the deftet / check_sign sub-benches')
    ap.add_argument('--eager', action='store_true', help='time the eager step only (no HIP graph capture)')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl')
    device = torch.device('cuda', local if world > 1 else 0)
    torch.cuda.set_device(device)

    views_per_rank = 4
    views = views_for_rank(rank, world, views_per_rank)
    inp = dibr_inputs(views, device)
    step = lambda: dibr_step(inp, world)  # noqa: E731
    for _ in range(args.warmup):
        step()
    # workload statistics for the algorithmic byte counts
    with torch.no_grad():
        _, fidx = kal.render.mesh.rasterize(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'] >= 0)
        fm = inp['fvi'] * 1000.
        bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
        _, _, cidx, _ = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, fidx, 7000., 30, 1000.)
        unc = fidx < 0
        used = (cidx >= 0).sum(-1)
        slot_reads = int((torch.clamp(used + 1, max=30) * unc).sum())
        stats = dict(valid_faces=int((inp['fnz'] >= 0).sum()), slot_reads=slot_reads, hits=int(used.sum()),
                     uncovered=float(unc.float().mean()), mean_slots=float(used[unc].float().mean()))
    # eager pass: per-op HIP-event timing for the roofline, and the eager rate
    timer = _native.OpTimer()
    _native.set_timer(timer)
    eager_elapsed = timed_loop(step, args.steps, world)
    _native.set_timer(None)
    eager_elapsed = max_over_ranks(eager_elapsed, device, world)
    ops_ms = timer.summary_ms()
    pixels = views_per_rank * inp['H'] * inp['W'] * world * args.steps
    eager_value = pixels / eager_elapsed / 1e6
    mode = 'eager'
    elapsed = eager_elapsed
    if not args.eager:
        gstep, gout = graphed_step(inp, world)
        ref = dibr_step(inp, world)
        gstep()
        torch.cuda.synchronize()
        # the replayed graph must reproduce the eager step (forward bit-exact, grads to float order)
        ok = torch.equal(gout[4], ref[3]) and torch.equal(gout[3], ref[2]) and \
            torch.allclose(gout[1], ref[0], rtol=1e-4, atol=1e-5) and torch.allclose(gout[2], ref[1], rtol=1e-4, atol=1e-5)
        if not ok:
            raise RuntimeError('graph replay differs from the eager step')
        for _ in range(args.warmup):
            gstep()
        elapsed = max_over_ranks(timed_loop(gstep, args.steps, world), device, world)
        mode = 'hip_graph'
    value = pixels / elapsed / 1e6
    result = None
    if rank == 0:
        ops_ms = {k: v for k, v in ops_ms.items() if op_bytes(k, inp, stats)}
        dom = max(ops_ms, key=ops_ms.get)
        dbytes = op_bytes(dom, inp, stats)
        achieved = dbytes / (ops_ms[dom] * 1e-3) / 1e9
        ops_report = {k: {'ms': round(v, 4), 'GB/s': (round(op_bytes(k, inp, stats) / (v * 1e-3) / 1e9, 1)
                                                     if op_bytes(k, inp, stats) else None)}
                      for k, v in ops_ms.items()}
        result = {
            'metric': 'DIB-R 512^2 fwd+bwd Mpixels/s + point_to_mesh Mpairs/s, 1/2/4/8 GPU',
            'value': round(value, 2), 'unit': 'Mpixels/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic (seeded UV sphere, 4 views/GPU)',
            'config': {'workload': 'dibr_rasterization fwd+bwd, batch=4/GPU, 50k-face mesh, 512x512, K=30',
                       'global_batch': views_per_rank * world, 'height': 512, 'width': 512, 'faces': 50000,
                       'parallelism': f'batch-sharded x{world} (RCCL all_gather of per-shard losses)'},
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(dom),
                         'bytes_per_launch': dbytes, 'avg_launch_ms': round(ops_ms[dom], 4),
                         'note': 'algorithmic bytes of the compact soft-mask state (the reference layout would '
                                 'move ' + str(op_bytes('dibr_soft_mask_forward_cuda', inp, stats)) + ' B per call); '
                                 'the op is latency-bound, not HBM-bound (DESIGN.md section 5)',
                         'survey_formula': {
                             'scope': 'whole fwd+bwd step, SURVEY.md 8d cfg3 bytes (reference layout)',
                             'bytes_per_step': survey_step_bytes(inp, stats),
                             'achieved': round(survey_step_bytes(inp, stats) / (elapsed / args.steps) / 1e9, 1),
                             'frac': round(survey_step_bytes(inp, stats) / (elapsed / args.steps) / 1e9
                                           / HBM_PEAK_GBS, 4)}},
            'ops': ops_report,
            'workload_stats': stats,
            'mode': mode,
            'eager': {'value': round(eager_value, 2), 'ms_per_step': round(eager_elapsed / args.steps * 1e3, 4)},
        }
    if not args.no_p2m and rank == 0:
        mp, ms = p2m_bench(device, max(3, args.steps // 4))
        result['p2m'] = {'metric': 'point_to_mesh Mpairs/s (100k pts x 20k faces, fwd)', 'value': round(mp, 1),
                         'ms': round(ms, 3),
                         'roofline': {'bound': 'valu', 'flop_per_pair': 50,
                                      'achieved_tflops': round(mp * 1e6 * 50 / 1e12, 2),
                                      'peak_tflops': FP32_PEAK_TFLOPS,
                                      'frac': round(mp * 1e6 * 50 / 1e12 / FP32_PEAK_TFLOPS, 4)}}
    if not args.no_extra and rank == 0:
        result['deftet'] = deftet_bench(inp, max(3, args.steps // 4))
        result['check_sign'] = check_sign_bench(device, max(3, args.steps // 4))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rate, npx, dt = cpu_baseline(inp, args.cpu_row_step)
        result['cpu_baseline'] = {'value': round(rate, 5), 'unit': 'Mpixels/s', 'cores': 1, 'kind': 'port',
                                  'sample': f'C oracle, the {views_per_rank} views, every {args.cpu_row_step}th row of '
                                            f'512x512 ({npx} px, fwd+bwd, {dt:.1f} s)'}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
