"""bench.py -- DIB-R fwd+bwd throughput (Mpixels/s) on MI355X, plus point_to_mesh_distance
(Mpairs/s) and the other BASELINE.json configs as sub-lines.

Headline (``--config cfg3``, the default; BASELINE.json configs[2]),
per rank: UV sphere 126 lat x 200 lon = 50,000 faces, radius 0.9*(1+0.01*N(0,1)) per vertex
(seed 0); 4 views (azimuth 2*pi*i/(4N), distance 3, look-at 0, up +y, fovy pi/4); features
D=3 = [uv, 1]; dibr_rasterization(512, 512, ..., sigmainv=7000, boxlen=0.02, knum=30,
multiplier=1000, eps=1e-8); loss = <feat, g_feat> + <soft_mask, g_mask> with g ~ U[0,1]
(seed 1); backward to face_vertices_image and face_features.  One step = that forward +
backward over the rank's views.  ``--config cfg5`` (configs[4]): 8 views per rank at
1024x1024, 64 views over 8 GPUs.

Multi-GPU: one process per GPU.  Under torchrun (the driver's N>1 launch) the ranks come
from the environment and WORLD_SIZE must equal --gpus.  Run directly with --gpus N > 1, this
script starts the N rank processes itself (before anything touches the GPU) and exits with
their status.  Views are sharded contiguously (weak scaling), per-shard losses are
all-gathered over RCCL each step; time = max over ranks.

Sub-lines: p2m (configs[1], points split over the ranks, faces replicated,
outputs all-gathered, face gradient all-reduced), cfg4 (voxelgrid R=512 + mesh_to_spc L=9
on a 200k-face sphere), raytrace (the cfg4 SPC, 512^2 rays), cfg1 (sided_distance 2k x 2k),
deftet and check_sign; a full-size parity block (the GPU step against the C oracle on a row
sample) and CPU baselines (1 thread and all threads, median of 5, samples stated).
"""
import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'kaolin-windows_amd'))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector peak
METRIC = 'DIB-R 512^2 fwd+bwd Mpixels/s + point_to_mesh Mpairs/s, 1/2/4/8 GPU'
CONFIGS = {
    'cfg3': dict(views=4, H=512, W=512, row_step=2,
                 workload='dibr_rasterization fwd+bwd, batch=4/GPU, 50k-face mesh, 512x512, K=30'),
    'cfg5': dict(views=8, H=1024, W=1024, row_step=16,
                 workload='dibr_rasterization fwd+bwd, batch=8/GPU (64 @ 8 GPUs), 50k-face mesh, 1024x1024, K=30'),
}


# ----------------------------------------------------------------------------- launcher
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', choices=sorted(CONFIGS), default='cfg3')
    ap.add_argument('--device', choices=['cuda', 'cpu'], default='cuda',
                    help='cpu: gloo self-test of the launcher and the sharded p2m path (no GPU)')
    ap.add_argument('--cpu-row-step', type=int, default=None, help='oracle row sample (default per config)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-p2m', action='store_true')
    ap.add_argument('--no-extra', action='store_true', help='skip the cfg4 / raytrace / cfg1 / deftet / check_sign legs')
    ap.add_argument('--eager', action='store_true', help='time the eager step only (no HIP graph capture)')
    ap.add_argument('--collectives', action='store_true',
                    help='N=1: initialise a one-rank RCCL group and keep the loss all_gather (and the p2m leg\'s '
                         'gathers / face-gradient all_reduce) in the timed steps, as the N-GPU job times them')
    return ap.parse_args(argv)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    rendezvous on 127.0.0.1) and return the worst exit status.  The parent makes no GPU call:
    each child is a fresh interpreter."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


# ----------------------------------------------------------------------------- workloads
def uv_sphere(n_lat, n_lon, device, dtype=None, seed=0, radius=0.9, noise=0.01):
    import torch
    dtype = dtype or torch.float32
    lat = torch.linspace(0, math.pi, n_lat + 1, dtype=torch.float64)[1:-1]
    lon = torch.arange(n_lon, dtype=torch.float64) * (2 * math.pi / n_lon)
    ring = torch.stack([torch.sin(lat)[:, None] * torch.cos(lon)[None], torch.cos(lat)[:, None].expand(-1, n_lon),
                        torch.sin(lat)[:, None] * torch.sin(lon)[None]], -1).reshape(-1, 3)
    verts = torch.cat([torch.tensor([[0., 1., 0.]], dtype=torch.float64), ring,
                       torch.tensor([[0., -1., 0.]], dtype=torch.float64)])
    g = torch.Generator().manual_seed(seed)
    verts = verts * (radius * (1 + noise * torch.randn((verts.shape[0], 1), generator=g, dtype=torch.float64)))
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
    import torch
    import kaolin as kal
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


def collectives_on():
    """An initialised process group (N > 1, or N = 1 with --collectives): the step's collectives run."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def gather_losses(loss, world):
    """The step's only collective: all_gather of the per-shard scalar losses (RCCL whenever a
    process group is initialised, at N = 1 too under --collectives), waited for in its own step.
    (r06: issuing it asynchronously and waiting for it after the next step's kernels were queued
    measured slower at N = 1 on RCCL -- 0.2105 / 0.2261 against 0.1959 / 0.1968 ms per step,
    profiles/r06/r06g_collectives_ab.txt -- so the plain form stays.)"""
    from kaolin.distributed import gather_losses as gl
    return gl(loss) if collectives_on() else loss.detach().reshape(1)


def max_over_ranks(elapsed, device, world):
    return max(per_rank(elapsed, device, world))


def per_rank(elapsed, device, world):
    """Every rank's elapsed time (all_gather over the initialised process group)."""
    if world == 1:
        return [elapsed]
    import torch
    import torch.distributed as dist
    from kaolin.distributed import _all_gather  # (host copies under gloo: the shared-GPU rehearsal)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    _all_gather(out, t, None)
    return [float(x) for x in out]


def process_group_info(world):
    """What the initialised process group says (not the environment): world size, backend."""
    import torch.distributed as dist
    if not collectives_on():
        return {'initialized': False, 'world_size': 1, 'backend': None}
    return {'initialized': True, 'world_size': dist.get_world_size(), 'backend': str(dist.get_backend())}


def _sync(device):
    import torch
    if device.type == 'cuda':
        torch.cuda.synchronize(device)


def timed_loop(fn, steps, world, device=None):
    import torch
    import torch.distributed as dist
    device = device or torch.device('cuda', torch.cuda.current_device())
    if world > 1:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync(device)
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def progress(msg):
    """One line per leg on stderr (a long run keeps showing signs of life)."""
    print(f'[bench {time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def cpu_info():
    model = None
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    # the "all threads" CPU legs use the process's share of the host: OMP_NUM_THREADS when set (the
    # GPU box sets it to its 16-CPU share; os.cpu_count() there reports the whole machine's CPUs,
    # which this job may not use), else the CPUs the process may run on
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    all_threads = int(os.environ.get('OMP_NUM_THREADS') or affinity or 1)
    return {'model': model, 'visible_cpus': os.cpu_count(), 'affinity_cpus': affinity,
            'threads_used_for_nproc_leg': all_threads,
            'threads_source': 'OMP_NUM_THREADS (the job\'s CPU share)' if os.environ.get('OMP_NUM_THREADS')
            else 'sched_getaffinity'}


def median_time(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def torch_cpu_legs(fn, units, unit_scale, reps=5):
    """Median of `reps` runs of fn on 1 thread and on all threads -> {threads: rate}."""
    import torch
    prev = torch.get_num_threads()
    out = {}
    try:
        for nt in sorted({1, cpu_info()['threads_used_for_nproc_leg']}):
            torch.set_num_threads(nt)
            fn()  # warm
            out[str(nt)] = round(units / median_time(fn, reps) / unit_scale, 4)
    finally:
        torch.set_num_threads(prev)
    return out


# ----------------------------------------------------------------------------- DIB-R step
def loss_dot2(a, ga, b, gb, inp):
    """L = <a, ga> + <b, gb> in one launch (kl_loss_dot2: fp64 accumulation, deterministic; two
    torch.dot calls plus their add were four launches, ~25 us per step)."""
    import torch
    from kaolin import _native
    if 'loss_ws' not in inp:
        inp['loss_ws'] = torch.zeros(_native.lib().kl_loss_dot2_workspace_bytes(), dtype=torch.uint8, device=a.device)
    out = torch.empty(1, dtype=torch.float32, device=a.device)
    _native.check(_native.lib().kl_loss_dot2(_native.ptr(a), _native.ptr(ga), a.numel(), _native.ptr(b),
                                             _native.ptr(gb), b.numel(), _native.ptr(inp['loss_ws']),
                                             _native.ptr(out), _native.stream_of(a.device)), 'kl_loss_dot2')
    return out[0]


def dibr_compute(inp, g_feat=None, g_mask=None):
    """dibr_rasterization forward + the loss L = <features, g_feat> + <soft_mask, g_mask> + backward
    (everything but the collective).  dL/dfeatures = g_feat and dL/dsoft_mask = g_mask exactly, so the
    backward is driven with them directly (torch.autograd.backward) -- the same gradients as
    L.backward() without the broadcast kernels of the sum's backward; L itself is two dot products
    (one fused launch, loss_dot2)."""
    import torch
    import kaolin as kal
    g_feat = inp['g_feat'] if g_feat is None else g_feat
    g_mask = inp['g_mask'] if g_mask is None else g_mask
    fvi = inp['fvi'].detach().requires_grad_(True)
    feat = inp['feat'].detach().requires_grad_(True)
    feats, mask, idx = kal.render.mesh.dibr_rasterization(inp['H'], inp['W'], inp['fvz'], fvi, feat, inp['fnz'],
                                                          sigmainv=7000, boxlen=0.02, knum=30, multiplier=1000,
                                                          eps=1e-8)
    loss = loss_dot2(feats.detach(), g_feat, mask.detach(), g_mask, inp)
    torch.autograd.backward([feats, mask], [g_feat, g_mask])
    return loss, fvi.grad, feat.grad, mask, idx, feats


def dibr_step(inp, world):
    out = dibr_compute(inp)
    if collectives_on():  # per-shard losses all-gathered over RCCL / xGMI
        gather_losses(out[0], world)
    return out


def graphed_step(inp, world):
    """The same step with dibr_compute captured once in a HIP graph (its launches replayed as
    one); the loss all_gather stays an eager RCCL call.  Inputs are static buffers, as in a
    training loop that copies each batch into them."""
    import torch
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
        if collectives_on():
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
    if name == 'dibr_soft_mask_backward':
        # compact state: read grad, mask, hits per px + one record per hit + faces; add into grad (B,F,3,2)
        return px * (s + s + 1) + stats['hits'] * (4 + s) + B * F * 6 * s * 2
    if name == 'dibr_rasterize_forward':
        # write idx/weights/features; read (valid mask + z + image coords) of all faces + features of valid ones
        return px * (8 + 3 * s + D * s) + B * F * (1 + 3 * s + 6 * s) + nv * 3 * D * s
    if name == 'dibr_forward':
        # both of the above in one call: the faces are read once for both
        return (op_bytes('dibr_rasterize_forward', inp, stats) + op_bytes('dibr_soft_mask_forward', inp, stats)
                - B * F * 6 * s)
    if name in ('rasterize_backward_cuda', 'dibr_rasterize_backward'):
        return px * (8 + 3 * s + D * s) + B * F * (6 * s + 3 * D * s) * 2
    if name == 'dibr_backward':
        return (op_bytes('dibr_rasterize_backward', inp, stats) + op_bytes('dibr_soft_mask_backward', inp, stats)
                - B * F * 6 * s * 2)
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
    # (the _C soft mask's tile-path kernel shares the name up to its BboxSrc source: match the SoftSrc one)
    'dibr_forward': ('raster_bin_word_kernel<float, 2', 'tile_countorder_chip_kernel', 'raster_tile_kernel<float',
                     'soft_tile_fwd_kernel<float, kl::SoftSrc'),
    'dibr_backward': ('rasterize_bwd_gather2_kernel<float', 'soft_tile_bwd_kernel<float'),
}


# the sub-lines' kernels, each launched once per timed call (hipCUB's sorts / scans, shared by several
# legs, are left out of their traffic: `traffic_scope` says so)
SUB_KERNELS = {
    'deftet': ('deftet_tilebox_kernel', 'deftet_fwd_kernel', 'deftet_resolve_slots_kernel', 'deftet_bwd_keys_kernel',
               'deftet_bwd_gather_kernel'),
    'check_sign': ('cs_prep_kernel', 'cs_bin_kernel<false', 'cs_pcount_kernel', 'cs_units_kernel',
                   'cs_bin_kernel<true', 'cs_pscatter_kernel', 'cs_cell_check_kernel', 'cs_finalize_kernel'),
    'cfg1_sided': ('sided_fwd_kernel<float', 'sided_combine_kernel<float'),
    'soft_mask_C': ('bin_faces_kernel<float, kl::BboxSrc', 'soft_tile_fwd_kernel<float, kl::BboxSrc'),
}


def pmc_traffic(op, config):
    """HBM bytes per call of `op` from the committed PMC summary of the config's workload
    (scripts/pmc_traffic.py: profiles/pmc_traffic.json for the cfg3 step, pmc_traffic_cfg5.json for
    cfg5, pmc_traffic_sub.json for the sub-lines), or None when a kernel of the op is missing from it."""
    name = 'pmc_traffic.json' if config == 'cfg3' else f'pmc_traffic_{config}.json'
    if op in SUB_KERNELS:  # the sub-lines' passes ran over the bench's extra legs (their own summary)
        name = 'pmc_traffic_sub.json'
    path = os.path.join(ROOT, 'profiles', name)
    kernels = OP_KERNELS.get(op) or SUB_KERNELS.get(op)
    if not kernels or not os.path.exists(path):
        return None
    kern = json.load(open(path))['kernels']
    total, found = 0, 0
    for pref in kernels:
        for name, v in kern.items():
            if pref in name:
                total += v['hbm_bytes']
                found += 1
                break
    return total if found == len(kernels) else None


def roofline_hbm(nbytes, ms, op, model, config='cfg3'):
    """A sub-line's HBM roofline: algorithmic bytes per call / its mean call time, PMC traffic beside."""
    ach = nbytes / (ms * 1e-3) / 1e9
    return {'bound': 'hbm', 'achieved': round(ach, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(ach / HBM_PEAK_GBS, 4), 'bytes_per_call': int(nbytes), 'bytes_model': model,
            'traffic': pmc_traffic(op, config),
            'traffic_scope': 'sum of the kernels ' + ', '.join(SUB_KERNELS.get(op, OP_KERNELS.get(op, ())))}


def roofline_valu(flops, ms, model):
    ach = flops / (ms * 1e-3) / 1e12
    return {'bound': 'valu', 'achieved': round(ach, 4), 'peak': FP32_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(ach / FP32_PEAK_TFLOPS, 6), 'flops_per_call': int(flops), 'flops_model': model}


def workload_stats(inp):
    """Per-run counts for the algorithmic byte model: valid faces, soft-mask hits, uncovered
    fraction and mean used slots (from the _C contract's slot tensors, outside the timed region)."""
    import torch
    import kaolin as kal
    with torch.no_grad():
        _, fidx = kal.render.mesh.rasterize(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'] >= 0)
        fm = inp['fvi'] * 1000.
        bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
        _, _, cidx, _ = kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, fidx, 7000., 30, 1000.)
        unc = fidx < 0
        used = (cidx >= 0).sum(-1)
        stats = dict(valid_faces=int((inp['fnz'] >= 0).sum()), hits=int(used.sum()),
                     uncovered=float(unc.float().mean()), mean_slots=float(used[unc].float().mean()))
        del cidx
    torch.cuda.empty_cache()
    return stats


def dibr_parity_and_cpu(inp, row_step):
    """The C oracle (1 thread) on every `row_step`-th pixel row of all the rank's views: rasterize
    fwd, soft mask fwd, soft mask bwd, rasterize bwd with the bench's own upstream gradients.  Timed
    as the CPU baseline, then compared with the GPU step: forward rows bit-exact / max-abs, and the
    GPU backward driven by the same gradients restricted to the sampled rows (a pixel's gradient
    terms depend only on that pixel) against the oracle's gradients."""
    import numpy as np
    import torch
    from oracle import oracle as orc
    A = lambda t: t.detach().cpu().numpy()  # noqa: E731
    fvz, fvi, feat, fnz = (A(inp[k]) for k in ('fvz', 'fvi', 'feat', 'fnz'))
    gf, gm = A(inp['g_feat']), A(inp['g_mask'])
    H, W = inp['H'], inp['W']
    orc.lib().or_set_row_step(row_step)
    try:
        t0 = time.perf_counter()
        of, oi, ow = orc.rasterize(H, W, fvz, fvi, feat, valid_faces=fnz >= 0)
        fm, bb = orc.soft_mask_bboxes(fvi, 0.02, 1000.)
        om, op, oci, oct_ = orc.dibr_soft_mask_forward(fm, bb, oi, 7000., 30, 1000.)
        gi_s = orc.dibr_soft_mask_backward(gm, om, oi, op, oci, oct_, fm, 7000., 1000.)
        gi_r, gf_r = orc.rasterize_backward(gf, oi, ow, fvi, feat, 1e-8)
        dt = time.perf_counter() - t0
    finally:
        orc.lib().or_set_row_step(1)
    rows = np.arange(0, H, row_step)
    npx = len(rows) * W * fvz.shape[0]
    # GPU: full forward, backward restricted to the sampled rows
    rmask = torch.zeros((1, H, 1), device=inp['fvz'].device)
    rmask[:, rows] = 1
    _, gfvi, gfeat, mask, idx, feats = dibr_compute(inp, inp['g_feat'] * rmask.unsqueeze(-1), inp['g_mask'] * rmask)
    torch.cuda.synchronize()
    # the soft-mask backward's parity on identical saved values: the GPU forward's mask and
    # probabilities (equal to the oracle's to expf ulps, reported as max_abs_mask)
    from kaolin import _fused
    _, state = _fused.soft_mask_forward_compact(inp['fvi'], idx, 7000., 0.02, 30, 1000.)
    _, _, gp = orc.decode_compact(A(state.hits), A(state.rec_face), A(state.rec_prob), 30, rows=rows)
    orc.lib().or_set_row_step(row_step)
    try:
        gi_s = orc.dibr_soft_mask_backward(gm, A(mask), oi, gp, oci, oct_, fm, 7000., 1000.)
    finally:
        orc.lib().or_set_row_step(1)
    gi_o, gfe_o = gi_r + gi_s, gf_r
    gi_g, gfe_g = A(gfvi), A(gfeat)
    scale_i = float(np.abs(gi_o).max())
    parity = {
        'sample': f'every {row_step}th row of {fvz.shape[0]} views at {H}x{W} ({npx} px), oracle = C restatement',
        'face_idx_equal': bool(np.array_equal(A(idx)[:, rows], oi[:, rows])),
        'max_abs_feat': float(np.abs(A(feats)[:, rows] - of[:, rows]).max()),
        'max_abs_mask': float(np.abs(A(mask)[:, rows] - om[:, rows]).max()),
        'max_abs_grad_fvi': float(np.abs(gi_g - gi_o).max()),
        'max_abs_grad_feat': float(np.abs(gfe_g - gfe_o).max()),
        'max_abs_grad_fvi_reference_magnitude': scale_i,
        'grad_fvi_elems_over_1e-5': int((np.abs(gi_g - gi_o) > 1e-5).sum()),
        'grad_fvi_equal': bool(np.array_equal(gi_g, gi_o)),
        'grad_feat_equal': bool(np.array_equal(gfe_g, gfe_o)),
        'grad_note': 'both sides sum the float terms in double and round once; the soft-mask '
                     'backward runs on the GPU forward\'s saved mask / probabilities',
    }
    # the same sample on all threads (OpenMP over pixel rows; the backward's double sums added
    # with atomics): the parity above is the 1-thread run's
    nt = cpu_info()['threads_used_for_nproc_leg']
    dt_n = None
    if nt > 1:
        orc.lib().or_set_row_step(row_step)
        orc.lib().or_set_threads(nt)
        try:
            t0 = time.perf_counter()
            of2, oi2, ow2 = orc.rasterize(H, W, fvz, fvi, feat, valid_faces=fnz >= 0)
            om2, op2, oci2, oct2 = orc.dibr_soft_mask_forward(fm, bb, oi2, 7000., 30, 1000.)
            orc.dibr_soft_mask_backward(gm, om2, oi2, op2, oci2, oct2, fm, 7000., 1000.)
            orc.rasterize_backward(gf, oi2, ow2, fvi, feat, 1e-8)
            dt_n = time.perf_counter() - t0
        finally:
            orc.lib().or_set_threads(1)
            orc.lib().or_set_row_step(1)
    by_threads = {'1': round(npx / dt / 1e6, 5)}
    if dt_n:
        by_threads[str(nt)] = round(npx / dt_n / 1e6, 5)
    best = max(by_threads, key=lambda k: by_threads[k])
    cpu = {'value': by_threads[best], 'unit': 'Mpixels/s', 'cores': int(best), 'kind': 'port', 'by_threads': by_threads,
           'sample': f'C oracle (restatement of the reference CUDA path), {fvz.shape[0]} views, every {row_step}th '
                     f'row of {H}x{W} ({npx} px), fwd+bwd; 1 thread {dt:.1f} s'
                     + (f', {nt} threads (OpenMP over pixel rows) {dt_n:.2f} s' if dt_n else '')}
    return parity, cpu


def dibr_headline(args, world, rank, device):
    import torch
    import kaolin as kal  # noqa: F401
    from kaolin import _native
    cfg = CONFIGS[args.config]
    inp = dibr_inputs(views_for_rank(rank, world, cfg['views']), device, cfg['H'], cfg['W'])
    step = lambda: dibr_step(inp, world)  # noqa: E731
    for _ in range(args.warmup):
        step()
    stats = workload_stats(inp)
    inp['stats'] = stats
    # eager pass with per-op HIP events (the roofline's op durations), then the eager rate
    # without them (the events and their Python cost are not part of the step)
    timer = _native.OpTimer()
    _native.set_timer(timer)
    timed_loop(step, args.steps, world, device)
    _native.set_timer(None)
    ops_ms = timer.summary_ms()
    eager_times = per_rank(timed_loop(step, args.steps, world, device), device, world)
    eager_elapsed = max(eager_times)
    pixels = cfg['views'] * cfg['H'] * cfg['W'] * world * args.steps
    mode, elapsed = 'eager', eager_elapsed
    graph_elapsed = None
    if not args.eager:
        gstep, gout = graphed_step(inp, world)
        ref = dibr_step(inp, world)
        gstep()
        torch.cuda.synchronize()
        # the replayed graph must reproduce the eager step: forward bit-exact; gradients bit-exact
        # (the float terms sum exactly in double), save the documented one-ulp allowance where a
        # face's terms span more than ~2^29 -- at most 1 element in 10^4 (tests/dibr_util.py)
        ok = torch.equal(gout[4], ref[4]) and torch.equal(gout[3], ref[3])
        replay_grad_diffs = 0
        for a, b in ((gout[1], ref[1]), (gout[2], ref[2])):
            ne = a != b
            n = int(ne.sum())
            replay_grad_diffs += n
            if n:
                ulps = (a[ne].view(torch.int32).long() - b[ne].view(torch.int32).long()).abs().max()
                ok = ok and n <= max(1, a.numel() // 10000) and int(ulps) <= 1
        if not ok:
            raise RuntimeError('graph replay differs from the eager step')
        replay_check = {'forward_bit_equal': True, 'grad_elements_not_bit_equal': replay_grad_diffs}
        for _ in range(args.warmup):
            gstep()
        graph_times = per_rank(timed_loop(gstep, args.steps, world, device), device, world)
        graph_elapsed = max(graph_times)
        # the headline is the step in the faster of its two execution modes (same work, same
        # outputs: the replay is checked against the eager step above); the other is reported
        # beside it.  Eager can win: the graph's replay of ~10 small launches adds gaps the eager
        # stream, its host far ahead of the GPU, does not.
        if graph_elapsed <= eager_elapsed:
            elapsed, mode, rank_times = graph_elapsed, 'hip_graph', graph_times
        else:
            elapsed, mode, rank_times = eager_elapsed, 'eager', eager_times
    else:
        rank_times = eager_times
        replay_check = None
    pg = process_group_info(world)
    if pg['world_size'] != world:
        raise RuntimeError(f'process group has {pg["world_size"]} ranks, WORLD_SIZE says {world}')
    value = pixels / elapsed / 1e6
    if rank != 0:
        return None, inp
    ops_ms = {k: v for k, v in ops_ms.items() if op_bytes(k, inp, stats)}
    dom = max(ops_ms, key=ops_ms.get)
    dbytes = op_bytes(dom, inp, stats)
    achieved = dbytes / (ops_ms[dom] * 1e-3) / 1e9
    ops_report = {k: {'ms': round(v, 4), 'bytes': op_bytes(k, inp, stats),
                      'GB/s': round(op_bytes(k, inp, stats) / (v * 1e-3) / 1e9, 1)} for k, v in ops_ms.items()}
    sb = survey_step_bytes(inp, stats)
    result = {
        'metric': METRIC, 'value': round(value, 2), 'unit': 'Mpixels/s', 'n_gpus': pg['world_size'], 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'data': f'synthetic (seeded UV sphere, {cfg["views"]} views/GPU)',
        'config': {'workload': cfg['workload'], 'config': args.config, 'global_batch': cfg['views'] * world,
                   'height': cfg['H'], 'width': cfg['W'], 'faces': 50000,
                   'parallelism': f'batch-sharded x{world} (RCCL all_gather of per-shard losses)'
                                  + ('' if pg['initialized'] else ' -- N=1 without a process group: no collective in the step')},
        'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(dom, args.config),
                     'bytes_per_launch': dbytes, 'avg_launch_ms': round(ops_ms[dom], 4),
                     'note': 'algorithmic bytes of the compact soft-mask state (the reference layout would move '
                             + str(op_bytes('dibr_soft_mask_forward_cuda', inp, stats)) + ' B per call in the soft '
                             'mask alone); the op is latency-bound, not HBM-bound (DESIGN.md section 5)',
                     'survey_formula': {
                         'scope': 'whole fwd+bwd step, SURVEY.md 8d cfg3 bytes (reference layout)',
                         'bytes_per_step': sb, 'achieved': round(sb / (elapsed / args.steps) / 1e9, 1),
                         'frac': round(sb / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}},
        'ops': ops_report, 'workload_stats': stats, 'mode': mode, 'graph_replay_check': replay_check,
        'process_group': dict(pg, per_rank_ms_per_step=[round(t / args.steps * 1e3, 4) for t in rank_times],
                              devices_visible=torch.cuda.device_count()),
        'eager': {'value': round(pixels / eager_elapsed / 1e6, 2),
                  'ms_per_step': round(eager_elapsed / args.steps * 1e3, 4)},
        'hip_graph': None if graph_elapsed is None else {'value': round(pixels / graph_elapsed / 1e6, 2),
                                                         'ms_per_step': round(graph_elapsed / args.steps * 1e3, 4)},
    }
    return result, inp


# ----------------------------------------------------------------------------- prepare_vertices
def prepare_leg(device, steps, views=4):
    """prepare_vertices (render/mesh/utils.py:128-175) fwd + bwd on the
    cfg3 mesh and views, vertices and camera requiring grad: the fused HIP path
    (csrc/prepare.hip) against the reference's torch chain of ops on the same GPU."""
    import torch
    import kaolin as kal
    from kaolin.render.mesh.utils import _prepare_vertices_torch
    verts, faces = uv_sphere(126, 200, device)
    B, V, F = views, verts.shape[0], faces.shape[0]
    az = torch.tensor(views_for_rank(0, 1, views), dtype=torch.float32, device=device)
    cam = torch.stack([3 * torch.sin(az), torch.zeros_like(az), 3 * torch.cos(az)], -1)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(
        cam, torch.zeros_like(cam), torch.tensor([[0., 1., 0.]], device=device).repeat(B, 1))
    proj = kal.render.camera.generate_perspective_projection(math.pi / 4).to(device)
    v = verts.unsqueeze(0).repeat(B, 1, 1).requires_grad_(True)
    rot, trans = rot.requires_grad_(True), trans.requires_grad_(True)
    g = torch.Generator().manual_seed(3)
    grads = [torch.rand(s, generator=g).to(device) for s in ((B, F, 3, 3), (B, F, 3, 2), (B, F, 3))]

    def run(fn):
        out = fn(v, faces, proj, rot, trans, None)
        torch.autograd.backward(out, grads)
        v.grad = rot.grad = trans.grad = None
    fused = lambda: run(lambda *a: kal.render.mesh.prepare_vertices(*a[:5]))  # noqa: E731
    chain = lambda: run(_prepare_vertices_torch)  # noqa: E731
    ms_f = _wall_ms(fused, max(5, steps))
    ms_t = _wall_ms(chain, max(5, steps))
    # parity at bench size: max-abs of the fused path against the reference's own f32 chain
    # (torch ops on the same GPU) and of both against float64, outputs and vertex / camera grads
    res = {}
    for name, fn, dt in (('fused', lambda *a: kal.render.mesh.prepare_vertices(*a[:5]), torch.float32),
                         ('chain', _prepare_vertices_torch, torch.float32),
                         ('f64', _prepare_vertices_torch, torch.float64)):
        lv = [x.detach().to(dt).requires_grad_(True) for x in (v, rot, trans)]
        out = fn(lv[0], faces, proj.to(dt), lv[1], lv[2], None)
        torch.autograd.backward(out, [g.to(dt) for g in grads])
        res[name] = [o.detach().double() for o in out] + [x.grad.double() for x in lv]
    names = ['face_vertices_camera', 'face_vertices_image', 'face_normals', 'grad_vertices', 'grad_rot',
             'grad_trans']
    mx = lambda a, b: float((a - b).abs().max())  # noqa: E731
    parity = {n: {'fused_vs_f32_chain': mx(res['fused'][k], res['chain'][k]),
                  'fused_vs_f64': mx(res['fused'][k], res['f64'][k]),
                  'f32_chain_vs_f64': mx(res['chain'][k], res['f64'][k])} for k, n in enumerate(names)}
    v.grad = rot.grad = trans.grad = None
    # forward: vertices + faces read, three outputs written; backward: the three grads read,
    # the per-vertex double sums (5 x 8 B, atomics), the vertices re-read, grad_vertices written
    fwd_bytes = B * V * 12 + F * 24 + B * F * (36 + 24 + 12)
    bwd_bytes = B * F * (36 + 24 + 12) + F * 24 + B * V * 12 + B * V * 40 * 2 + B * V * 12
    nb = fwd_bytes + bwd_bytes
    return {'metric': 'prepare_vertices fwd+bwd ms (4 views, 50k-face mesh, vertices + camera grads, f32)',
            'ms': round(ms_f, 4), 'torch_chain_ms': round(ms_t, 4), 'speedup': round(ms_t / ms_f, 2),
            'bytes': nb, 'roofline': {'bound': 'hbm', 'achieved': round(nb / (ms_f * 1e-3) / 1e9, 1),
                                      'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                      'frac': round(nb / (ms_f * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            'timing': 'wall clock per fwd+bwd incl. Python / autograd (median of runs)',
            'parity_max_abs': parity}


# ----------------------------------------------------------------------------- tutorial loop
def tutorial_setup(device, views=4, H=512, W=512, tex=512):
    """The reference's own caller (examples/tutorial/dibr_tutorial.ipynb cells 8-14) at cfg3 size:
    the cfg3 sphere (50k faces) as the optimised mesh, 4 cameras (camera_transform form), a
    (1,3,tex,tex) texture map, Adam on the vertices + centre shift and on the texture.  Ground
    truth: a synthetic seeded image and a silhouette (no dataset on the box)."""
    import torch
    import kaolin as kal
    verts, faces = uv_sphere(126, 200, device)
    F = faces.shape[0]
    u = torch.atan2(verts[:, 2], verts[:, 0]) / (2 * math.pi) + 0.5
    vv = torch.acos(torch.clamp(verts[:, 1] / verts.norm(dim=1), -1, 1)) / math.pi
    face_uvs = kal.ops.mesh.index_vertices_by_faces(torch.stack([u, vv], -1)[None], faces).contiguous()
    az = torch.tensor(views_for_rank(0, 1, views), dtype=torch.float32, device=device)
    cam = torch.stack([3 * torch.sin(az), torch.zeros_like(az), 3 * torch.cos(az)], -1)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(
        cam, torch.zeros_like(cam), torch.tensor([[0., 1., 0.]], device=device).repeat(views, 1))
    cam_transform = torch.cat([rot.transpose(1, 2), -(trans[:, None] @ rot.transpose(1, 2))], 1).contiguous()
    cam_proj = kal.render.camera.generate_perspective_projection(math.pi / 4).to(device)
    g = torch.Generator().manual_seed(4)
    st = dict(
        faces=faces, face_uvs=face_uvs, cam_transform=cam_transform, cam_proj=cam_proj, B=views, H=H, W=W, F=F,
        vertices=verts[None].clone().requires_grad_(True),
        shift=torch.zeros((3,), dtype=torch.float32, device=device, requires_grad=True),
        texture=torch.rand((1, 3, tex, tex), generator=g).to(device).requires_grad_(True),
        gt_image=torch.rand((views, H, W, 3), generator=g).to(device),
        gt_uv=torch.rand((views, H, W, 2), generator=g).to(device),
        gt_mask=(torch.rand((views, H, W), generator=g) > 0.5).float().to(device))
    st['vopt'] = torch.optim.Adam([st['vertices'], st['shift']], lr=5e-4)
    st['topt'] = torch.optim.Adam([st['texture']], lr=1e-2)
    return st


def _tutorial_render(st):
    """render() of dibr_tutorial.ipynb cell 12 up to the rasterizer: center_points + shift,
    prepare_vertices(camera_transform=...), dibr_rasterization with the feature LIST
    [face_uvs, ones] -> (uv map, hard mask), soft mask."""
    import torch
    import kaolin as kal
    B = st['B']
    vb = kal.ops.pointcloud.center_points(st['vertices']) + st['shift']
    fvc, fvi, fn = kal.render.mesh.prepare_vertices(vb.repeat(B, 1, 1), st['faces'], st['cam_proj'],
                                                    camera_transform=st['cam_transform'])
    attrs = [st['face_uvs'].repeat(B, 1, 1, 1), torch.ones((B, st['F'], 3, 1), device=fvc.device)]
    (coords, mask), soft_mask, _ = kal.render.mesh.dibr_rasterization(
        st['H'], st['W'], fvc[:, :, :, -1], fvi, attrs, fn[:, :, -1], rast_backend='cuda')
    return coords, mask, soft_mask


def tutorial_shape_step(st):
    """The tutorial's call shape: prepare_vertices -> dibr_rasterization(list
    [uv, ones]) -> L1 + mask_iou -> backward, eager.  L1 is on the rasterized features (uv map x
    hard mask against a target); the texture lookup and the optimiser are in tutorial_step."""
    import torch
    import kaolin as kal
    coords, mask, soft_mask = _tutorial_render(st)
    l1 = torch.mean(torch.abs(coords * mask - st['gt_uv']))
    loss = l1 + kal.metrics.render.mask_iou(soft_mask, st['gt_mask'])
    loss.backward()
    st['vertices'].grad = st['shift'].grad = None
    return loss


def tutorial_step(st):
    """One whole iteration of dibr_tutorial.ipynb cell 14 (render() of cell 12 inlined): zero_grad,
    the render above, texture_mapping (bilinear), clamp(image * mask), L1 image loss + mask_iou,
    backward, both Adam steps.  The tutorial's laplacian regulariser (a dense V x V matmul, off the
    rendering path) is left out."""
    import torch
    import kaolin as kal
    B = st['B']
    st['vopt'].zero_grad()
    st['topt'].zero_grad()
    coords, mask, soft_mask = _tutorial_render(st)
    image = kal.render.mesh.texture_mapping(coords, st['texture'].repeat(B, 1, 1, 1), mode='bilinear')
    image = torch.clamp(image * mask, 0., 1.)
    image_loss = torch.mean(torch.abs(image - st['gt_image']))
    mask_loss = kal.metrics.render.mask_iou(soft_mask, st['gt_mask'])
    loss = image_loss * 1. + mask_loss * 1.
    loss.backward()
    st['vopt'].step()
    st['topt'].step()
    return loss


def tutorial_leg(device, steps, warmup=3):
    """The tutorial's call shape, eager (the caller the reference's users run): `value`; with the
    DIB-R fwd+bwd's own HIP-event time beside it, and the whole tutorial iteration (texture lookup,
    optimiser) as `full_iteration`."""
    import torch
    from kaolin import _native
    st = tutorial_setup(device)
    px = st['B'] * st['H'] * st['W']
    for _ in range(warmup):
        tutorial_shape_step(st)
    ms = _wall_ms(lambda: tutorial_shape_step(st), steps)
    # steady-state throughput: the loop without a sync per step (as bench's eager line)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tutorial_shape_step(st)
    torch.cuda.synchronize()
    ms_loop = (time.perf_counter() - t0) / steps * 1e3
    timer = _native.OpTimer()
    _native.set_timer(timer)
    for _ in range(5):
        tutorial_shape_step(st)
    _native.set_timer(None)
    ops = {k: round(v, 4) for k, v in timer.summary_ms().items()}
    # the same step captured once in a HIP graph and replayed (the caller's torch ops and autograd
    # included): what is left of the step without the eager host path
    ms_graph = None
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                tutorial_shape_step(st)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            tutorial_shape_step(st)
        for _ in range(warmup):
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            graph.replay()
        torch.cuda.synchronize()
        ms_graph = (time.perf_counter() - t0) / steps * 1e3
    except RuntimeError as e:  # reported, not fatal: the eager line is the tutorial's own shape
        ms_graph = f'capture failed: {e}'
    for _ in range(warmup):
        tutorial_step(st)
    ms_full = _wall_ms(lambda: tutorial_step(st), max(3, steps // 2))
    return {'metric': 'DIB-R tutorial call shape Mpixels/s, eager: prepare_vertices -> dibr_rasterization([uv, ones]) '
                      '-> L1 + mask_iou -> backward (4 views x 512^2, 50k faces)',
            'value': round(px / (ms_loop * 1e-3) / 1e6, 2), 'ms_per_step': round(ms_loop, 4),
            'ms_per_step_synced': round(ms, 4), 'native_op_ms': ops,
            'graph': ({'value': round(px / (ms_graph * 1e-3) / 1e6, 2), 'ms_per_step': round(ms_graph, 4),
                       'what': 'the same step captured once in a HIP graph and replayed (loss ops and autograd '
                               'included)'} if isinstance(ms_graph, float) else ms_graph),
            'full_iteration': {'ms': round(ms_full, 4), 'value': round(px / (ms_full * 1e-3) / 1e6, 2),
                               'what': 'dibr_tutorial.ipynb cell 14 minus the laplacian term: + texture_mapping '
                                       '(bilinear, 512^2 texture), clamp, L1 image loss, both Adam steps'},
            'timing': 'value: back-to-back eager steps between two synchronizes (as the headline eager line); '
                      'ms_per_step_synced: median with a synchronize per step'}


# ----------------------------------------------------------------------------- p2m (cfg2)
def p2m_inputs(device):
    import torch
    g = torch.Generator().manual_seed(0)
    pts = torch.randn((100000, 3), generator=g)
    fv = torch.randn((20000, 3, 3), generator=g)
    gd = torch.rand((100000,), generator=torch.Generator().manual_seed(1))
    return pts.to(device), fv.to(device), gd.to(device)


def p2m_leg(device, world, rank, steps, points=None, face_vertices=None, grad=None):
    """cfg2: 100k points vs 20k faces, points split contiguously over the ranks, faces
    replicated, outputs all-gathered (kaolin.distributed.sharded_point_to_mesh_distance).
    Timed: forward (+ gather), and forward + backward (+ face-gradient all_reduce)."""
    import torch
    from kaolin.distributed import shard_bounds, sharded_point_to_mesh_distance
    if points is None:
        points, face_vertices, grad = p2m_inputs(device)
    P, F = points.shape[0], face_vertices.shape[0]
    lo, hi = shard_bounds(P, rank, world)
    local = points[lo:hi].contiguous()

    def fwd():
        with torch.no_grad():
            return sharded_point_to_mesh_distance(local, face_vertices)

    lp = local.detach().requires_grad_(True)
    fvr = face_vertices.detach().requires_grad_(True)

    def fwd_bwd():
        lp.grad = None
        fvr.grad = None
        d, _, _ = sharded_point_to_mesh_distance(lp, fvr)
        d.backward(grad)

    out = fwd()
    fwd_bwd()
    t_f = max_over_ranks(timed_loop(fwd, steps, world, device), device, world) / steps
    t_fb = max_over_ranks(timed_loop(fwd_bwd, steps, world, device), device, world) / steps
    res = {'metric': 'point_to_mesh Mpairs/s (100k pts x 20k faces, fwd; points sharded over ranks)',
           'value': round(P * F / t_f / 1e6, 1), 'ms': round(t_f * 1e3, 4),
           'fwd_bwd': {'value': round(P * F / t_fb / 1e6, 1), 'ms': round(t_fb * 1e3, 4)},
           'n_ranks': world, 'points_per_rank': hi - lo, 'faces': F,
           'roofline': p2m_roofline(P, F, t_f)}
    return res, out, (lp.grad, fvr.grad)


def p2m_roofline(P, F, t_f):
    """p2m forward against the FP32 VALU peak.  `frac` prices the EXECUTED FP32 work: the kernel
    evaluates only the pairs its bounds cannot skip (r05: the wave-level bound, then a per-point bound
    whose passing pairs are evaluated one per lane), and the committed counter profile
    (profiles/r05_p2m_pmc.json: probe + SQ_INSTS_VALU_{ADD,MUL,FMA}_F32 passes on this round's kernel;
    r04's file for the r04 kernel) counts the flops one call executes; their rate at this call's time
    is the achieved figure.  The nominal figure (P*F x 50 flop) is beside it."""
    nominal = P * F * 50 / t_f / 1e12
    r = {'bound': 'valu', 'unit': 'TFLOP/s', 'peak': FP32_PEAK_TFLOPS,
         'nominal': {'flop_per_pair': 50, 'achieved': round(nominal, 2), 'frac': round(nominal / FP32_PEAK_TFLOPS, 4),
                     'note': 'nominal pairs (P*F); pruned pairs are not evaluated'}}
    name = 'r05_p2m_pmc.json' if os.path.exists(os.path.join(ROOT, 'profiles', 'r05_p2m_pmc.json')) else 'r04_p2m_pmc.json'
    path = os.path.join(ROOT, 'profiles', name)
    if P == 100000 and F == 20000 and os.path.exists(path):
        pm = json.load(open(path))
        executed = pm['executed_fp32_flop'] / t_f / 1e12
        r.update(achieved=round(executed, 2), frac=round(executed / FP32_PEAK_TFLOPS, 4),
                 executed_fp32_flop_per_call=pm['executed_fp32_flop'])
        r['measured'] = {'source': f'profiles/{name} (cfg2, one rank; this round\'s p2m_fwd_kernel)',
                         'evaluated_pair_fraction': pm['wave_face_pairs']['evaluated_fraction'],
                         'point_face_pairs_evaluated': pm['wave_face_pairs'].get('point_face_pairs_evaluated'),
                         'valu_insts_per_evaluated_wave_face_pair': pm['valu_insts_per_evaluated_wave_face_pair'],
                         'valu_issue_busy': pm['valu_issue_busy_est'],
                         'wait_any_fraction': pm['wait_any_fraction_of_wave_cycles']}
    else:
        r.update(achieved=r['nominal']['achieved'], frac=r['nominal']['frac'], note='no counter profile for this size: '
                 'nominal pairs')
    return r


def p2m_parity(points, face_vertices, out, n_sample=2000):
    """Oracle check of the sharded result on a point sample (C restatement of the reference
    CUDA kernel): forward bit-exact; face gradient of the sample via the oracle backward."""
    import numpy as np
    from oracle import oracle as orc
    A = lambda t: t.detach().cpu().numpy()  # noqa: E731
    P = points.shape[0]
    sel = np.linspace(0, P - 1, n_sample).astype(np.int64)
    od, oi, ot = orc.unbatched_triangle_distance_forward(A(points)[sel], A(face_vertices))
    d, i, t = (A(x) for x in out)
    return {'sample': f'{n_sample} evenly spaced points of {P} vs all {face_vertices.shape[0]} faces',
            'dist_equal': bool(np.array_equal(d[sel], od)), 'face_idx_equal': bool(np.array_equal(i[sel], oi)),
            'dist_type_equal': bool(np.array_equal(t[sel], ot))}


def p2m_cpu_legs(points, face_vertices, n_points=200):
    """The reference's CPU path for point_to_mesh_distance (its naive torch evaluation, restated in
    kaolin.metrics.trianglemesh) on the first n_points points vs all faces, fwd, 1 and all threads."""
    import torch
    from kaolin.metrics.trianglemesh import _unbatched_naive_point_to_mesh_distance as naive
    p = points[:n_points].cpu()
    fv = face_vertices.cpu()

    def run():
        with torch.no_grad():
            naive(p, fv)
    rates = torch_cpu_legs(run, n_points * fv.shape[0], 1e6)
    return {'unit': 'Mpairs/s', 'kind': 'port', 'by_threads': rates,
            'sample': f'first {n_points} points x {fv.shape[0]} faces (fwd, median of 5; rate extrapolates linearly '
                      'in points)'}


# ----------------------------------------------------------------------------- cfg1 sided
def sided_leg(device, steps):
    """cfg1: sided_distance on two random 2k-point clouds: the HIP kernel, and the reference's
    CPU path (its torch `_sided_distance`, restated in kaolin.metrics.pointcloud) on the host."""
    import torch
    import kaolin as kal
    from kaolin.metrics.pointcloud import _sided_distance
    g = torch.Generator().manual_seed(0)
    p1, p2 = torch.rand((1, 2048, 3), generator=g), torch.rand((1, 2048, 3), generator=g)
    d1, d2 = p1.to(device), p2.to(device)
    ms = _event_ms(lambda: kal.metrics.pointcloud.sided_distance(d1, d2), steps)
    dist, _ = kal.metrics.pointcloud.sided_distance(d1, d2)
    ref = _sided_distance(p1, p2)
    rates = torch_cpu_legs(lambda: _sided_distance(p1, p2), 2048 * 2048, 1e6)
    nbytes = 2 * 2048 * 12 + 2048 * (4 + 8)  # both clouds read, dist + idx written
    return {'metric': 'sided_distance Mpairs/s (2048 x 2048, f32, fwd)', 'value': round(2048 * 2048 / (ms * 1e-3) / 1e6, 1),
            'ms': round(ms, 4), 'parity_vs_cpu_reference_path': {'max_abs': float((dist.cpu() - ref).abs().max())},
            'roofline': dict(roofline_valu(8 * 2048 * 2048, ms, 'SURVEY.md 8d cfg1: 8 FP32 flop per pair (3 sub, '
                                           '3 mul, 2 add), 2048 x 2048 pairs'),
                             hbm=roofline_hbm(nbytes, ms, 'cfg1_sided', 'p1 and p2 read (12 B per point), dist 4 + '
                                                                        'idx 8 B per p1 point written'),
                             note='a 30 us call: launch- and latency-bound, far from either roof'),
            'cpu': {'unit': 'Mpairs/s', 'kind': 'port', 'by_threads': rates,
                    'sample': 'full 2048 x 2048 (median of 5)', 'survey_reference_8_threads': 152.0}}


# ----------------------------------------------------------------------------- cfg4
def cfg4_inputs(device):
    verts, faces = uv_sphere(251, 400, device, radius=0.95, noise=0.0)
    assert faces.shape[0] == 200000
    return verts, faces


def cfg4_leg(device, steps):
    """cfg4: trianglemeshes_to_voxelgrids at R=512 and unbatched_mesh_to_spc at L=9 on the
    200k-face sphere (radius 0.95), with the SURVEY.md §8d byte counts."""
    import torch
    import kaolin as kal
    from kaolin import _native
    verts, faces = cfg4_inputs(device)
    V, F, R, L = verts.shape[0], faces.shape[0], 512, 9
    vb = verts.unsqueeze(0).contiguous()
    fv = kal.ops.mesh.index_vertices_by_faces(vb, faces)[0].contiguous()
    vox = lambda: kal.ops.conversions.trianglemeshes_to_voxelgrids(vb, faces, R)  # noqa: E731
    spc = lambda: kal.ops.conversions.unbatched_mesh_to_spc(fv, L)  # noqa: E731
    grid = vox()
    n_occ = int(grid.count_nonzero())
    del grid
    octree, fidx, bary = spc()
    counts = (torch.zeros(16, dtype=torch.int64)).numpy()
    import ctypes
    nlev = _native.lib().kl_mesh_to_spc_level_counts(ctypes.c_void_p(counts.ctypes.data), 16)
    N = [int(x) for x in counts[:nlev]]
    nodes = int(octree.shape[0])
    leaves = int(fidx.shape[0])
    n_steps = max(3, steps // 4)
    ms_vox = _wall_ms(vox, n_steps)
    # the host-sized subdivision (one count read per level) beside the default device-counted one
    from kaolin.ops.conversions import trianglemesh as _tm
    _tm.HOST_SIZED = True
    try:
        grid_h = vox()
        ms_vox_host = _wall_ms(vox, n_steps)
    finally:
        _tm.HOST_SIZED = False
    vox_equal = bool(torch.equal(grid_h, vox()))
    del grid_h
    ms_spc = _wall_ms(spc, n_steps)
    vox_bytes = 4 * R ** 3 + 12 * V + 24 * F
    # SURVEY.md §8d (the reference's algorithm, sort and dedup included): an effective rate only
    survey_spc_bytes = sum(28 * n for n in N) + sum(16 * n for n in N[1:]) + N[-1] * (32 + 36 + 8) + 9 * nodes
    spc_bytes = m2s_build_bytes(N, F, nodes, leaves)
    return {'metric': 'cfg4: trianglemeshes_to_voxelgrids R=512 + unbatched_mesh_to_spc L=9, 200k-face sphere (f32)',
            'voxelgrid': {'ms': round(ms_vox, 3), 'occupied': n_occ, 'bytes': vox_bytes,
                          'host_sized': {'ms': round(ms_vox_host, 3), 'equal': vox_equal},
                          'roofline': {'bound': 'hbm', 'achieved': round(vox_bytes / (ms_vox * 1e-3) / 1e9, 1),
                                       'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                       'frac': round(vox_bytes / (ms_vox * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}},
            'mesh_to_spc': {'ms': round(ms_spc, 3), 'nodes': nodes, 'leaves': leaves, 'proposals_per_level': N,
                            'bytes': survey_spc_bytes,
                            # headline: SURVEY.md §8d's formula, comparable across rounds; the
                            # bytes this build's algorithm moves are the secondary build_model
                            'roofline': {'bound': 'hbm', 'achieved': round(survey_spc_bytes / (ms_spc * 1e-3) / 1e9, 1),
                                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                         'frac': round(survey_spc_bytes / (ms_spc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                         'bytes_source': 'SURVEY.md §8d (the reference algorithm: sort, dedup) -- an '
                                                         'effective rate: this build moves none of those bytes',
                                         'build_model': {
                                             'bytes': spc_bytes,
                                             'achieved': round(spc_bytes / (ms_spc * 1e-3) / 1e9, 1),
                                             'frac': round(spc_bytes / (ms_spc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                             'model': 'the node-rank algorithm (spc.hip): per pair its key, face, '
                                                      'triangle, node point and scan entry, child pairs written, '
                                                      '~31 B per node for the level scans, 52 B per leaf'}}},
            'timing': 'wall clock per call (median of runs); voxelgrid: device-counted levels, one status read; '
                      'voxelgrid.host_sized: incl. its per-level host count reads; mesh_to_spc: the node-rank '
                      'levels, one host read of the counts after them',
            'spc': (octree, fidx, bary)}


def m2s_build_bytes(N, F, nodes, leaves):
    """Bytes the node-rank mesh_to_spc (csrc/spc.hip, m2s_*_kernel) moves at cfg4, from its per-level
    proposal counts N (N[0] = F faces; N[l] = 8 x the passing (node, face) pairs of level l - 1):
    the root test reads every triangle (36 B) and writes its passing pairs (8 B); each level's
    node kernel reads a pair (key + face 8 B), its triangle (36 B), its node's point (8 B), scan
    entry (4 B) and parent octree byte (1 B), and writes the passing children's pairs (8 B) and
    child flags (1 B); the level scans read each node's child slots (8 B) and write its octree
    byte, scan entry, its children's points and cleared slots (~31 B per node over the levels);
    the leaves read their 8 least-face slots (32 B) and write face index and barycentrics (16 B),
    plus the last level's least-face atomics (4 B per leaf)."""
    pairs = [n // 8 for n in N[1:]]  # pairs of levels 0 .. L-1
    b = F * 36 + pairs[0] * 8
    for lvl in range(1, len(N)):
        b += pairs[lvl - 1] * (8 + 36 + 8 + 4 + 1)
        if lvl < len(pairs):
            b += pairs[lvl] * (8 + 1)
    return b + nodes * 31 + leaves * (32 + 16 + 4)


def cfg4_cpu_leg(device, stride=32):
    """The reference's voxelgrid algorithm on the host (its torch subdivision, restated in
    kaolin.ops.conversions as the CPU path) on every `stride`-th face of the cfg4 mesh at R=512,
    extrapolated linearly to all faces."""
    import torch
    import kaolin as kal
    verts, faces = cfg4_inputs('cpu')
    sub = faces[::stride].contiguous()
    vb = verts.unsqueeze(0)
    o = torch.min(vb, dim=1)[0]
    s = torch.max(torch.max(vb, dim=1)[0] - o, dim=1)[0]
    run = lambda: kal.ops.conversions.trianglemeshes_to_voxelgrids(vb, sub, 512, o, s)  # noqa: E731
    rates = torch_cpu_legs(run, 1.0, 1.0, reps=3)
    return {'unit': 'meshes/s (extrapolated)', 'kind': 'port',
            'by_threads': {k: round(v / stride, 6) for k, v in rates.items()},
            'sample': f'every {stride}th face ({sub.shape[0]} of {faces.shape[0]}) at R=512, median of 3, time x{stride} '
                      '(extrapolated); the reference itself took 55.9 s per mesh on 8 threads (BASELINE.md)'}


# ----------------------------------------------------------------------------- raytrace
def raytrace_leg(device, steps, spc_tuple):
    """North-star raytrace row: the cfg4 SPC (level 9), 512x512 pinhole rays from z=+3 toward
    the z=0 square [-1,1]^2 (SURVEY.md §8d byte model with the per-level hit counts)."""
    import torch
    import kaolin as kal
    octree = spc_tuple[0]
    lengths = torch.tensor([octree.shape[0]], dtype=torch.int32)
    L, pyr, exsum = kal.ops.spc.scan_octrees(octree, lengths)
    pts = kal.ops.spc.generate_points(octree, pyr, exsum)
    n = 512
    xs = (torch.arange(n, device=device, dtype=torch.float32) + 0.5) / n * 2 - 1
    tgt = torch.stack([xs.view(1, -1).expand(n, n), xs.view(-1, 1).expand(n, n), torch.zeros(n, n, device=device)], -1)
    o = torch.tensor([0., 0., 3.], device=device).expand(n * n, 3).contiguous()
    d = tgt.reshape(-1, 3) - o
    d = (d / d.norm(dim=-1, keepdim=True)).contiguous()
    rt = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L)  # noqa: E731
    ridx, pidx, depth = rt()
    hits = int(ridx.shape[0])
    per_level = [int(kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, lv,
                                                        return_depth=False)[0].shape[0]) for lv in range(L + 1)]
    ms = _wall_ms(rt, max(3, steps // 4))
    # the fixed-capacity march (kl_raytrace_fixed: no host count read, graph-capturable), capacity
    # above every level's candidates (a hit node's children before their own test, <= 8 each)
    cap = 8 * max(per_level) + 64
    rtf = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L, capacity=cap)  # noqa: E731
    fr, fp, fd, fres = rtf()
    fixed_equal = (fres.tolist() == [hits, 0] and torch.equal(fr[:hits], ridx) and torch.equal(fp[:hits], pidx)
                   and torch.equal(fd[:hits], depth))
    ms_fixed = _event_ms(rtf, max(3, steps // 4))
    R = n * n
    # SURVEY.md §8d's raytrace model (kept as survey_formula)
    survey_bytes = 24 * R + sum(31 * per_level[lv] + 8 * (per_level[lv + 1] if lv + 1 <= L else 0)
                                for lv in range(L + 1)) + per_level[L] * (16 + 4)
    # the hit-list march (spc.hip rth_count_kernel / rth_write_kernel; lists of HIT nodes): level 0's
    # list is the R rays at the root (8 B written); per level l < L, the count pass reads each listed
    # node's nugget 8 B, ray 24 B, octree byte 1 B, exsum 4 B and its children's points (6 B per
    # candidate: the popcount of the node's octree byte) and writes a mask byte (the tiles' totals,
    # 4 B per 256 nodes, are left out); the write pass reads the mask (1 B) and, per node, nugget 8 +
    # octree 1 + exsum 4 + point 6 + ray origin 12 B, and writes 8 B per hit child; the target level's
    # hits also re-read their point 6 B and ray direction 12 B for the depth (4 B written)
    cand = [R]
    for lv in range(L):
        _, pidx = kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, lv, return_depth=False)
        cand.append(int(_popcount_u8(octree[pidx.long()]).sum()))
    listed = [R] + per_level[1:L]
    nbytes = 8 * R + sum(n * (8 + 24 + 1 + 4 + 1 + 1 + 8 + 1 + 4 + 6 + 12) + 6 * cand[lv + 1] +
                         8 * per_level[lv + 1] for lv, n in enumerate(listed)) + per_level[L] * (6 + 12 + 4)
    return {'metric': 'unbatched_raytrace Mrays/s (cfg4 SPC level 9, 512x512 rays, depth)',
            'value': round(R / (ms * 1e-3) / 1e6, 2), 'ms': round(ms, 4), 'hits': hits, 'hits_per_level': per_level,
            'bytes': survey_bytes, 'timing': 'wall clock per call incl. its one host read and allocator calls',
            'fixed_capacity': {'value': round(R / (ms_fixed * 1e-3) / 1e6, 2), 'ms': round(ms_fixed, 4),
                               'capacity': cap, 'equal_to_host_sized': bool(fixed_equal),
                               'timing': 'HIP events over back-to-back calls (nothing read back)'},
            'candidates_per_level': cand,
            # headline: SURVEY.md §8d's formula (comparable across rounds); this build's bytes beside it
            'roofline': {'bound': 'hbm', 'achieved': round(survey_bytes / (ms * 1e-3) / 1e9, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(survey_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         'bytes_source': 'SURVEY.md §8d raytrace model with the per-level hit counts',
                         'build_model': {'bytes': nbytes,
                                         'achieved': round(nbytes / (ms * 1e-3) / 1e9, 1),
                                         'frac': round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                         'model': 'the hit-list march: per listed hit node its nugget, ray, octree '
                                                  'byte, exsum, its children\'s points and mask byte, the write '
                                                  'pass\'s reads and 8 B per hit child; per target hit its point and '
                                                  'ray again + depth'}}}


def _popcount_u8(t):
    """per-entry popcounts of a uint8 tensor (numpy)"""
    import numpy as np
    return np.unpackbits(t.cpu().numpy().astype(np.uint8).reshape(-1, 1), axis=1).sum(1)


# ----------------------------------------------------------------------------- deftet / check_sign
def _event_ms(fn, steps):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def _wall_ms(fn, steps):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def deftet_bench(inp, steps, knum=8):
    """deftet_sparse_render fwd+bwd on the cfg3 mesh and views: every
    pixel centre of the 512x512 grid, depth range = the mesh's z span, knum=8 (a covered pixel
    of the sphere holds its front and back faces)."""
    import torch
    import kaolin as kal
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
    out, idx = fwd()
    hits = int((idx >= 0).sum())
    nb = lambda t: t.numel() * t.element_size()  # noqa: E731
    F = fvz.shape[1]
    # compulsory traffic of one fwd + bwd: the inputs read once (pixels, ranges, the faces' z, image
    # coordinates and features), the outputs written once (slot features and face ids); the backward
    # reads the upstream gradient and the saved slots, and writes both face gradients
    nbytes = (nb(pix) + nb(rr) + nb(fvz) + nb(fvi) + nb(feat) + nb(out) + nb(idx)
              + nb(g) + nb(idx) + B * F * 3 * 4 + nb(fvi) + nb(feat))
    return {'metric': f'deftet_sparse_render fwd+bwd Mpixels/s ({B} views, {H}x{W}, 50k faces, knum=8, f32)',
            'value': round(B * H * W / (ms * 1e-3) / 1e6, 1), 'ms': round(ms, 3), 'fwd_ms': round(ms_fwd, 3),
            'hits': hits,
            'roofline': roofline_hbm(nbytes, ms, 'deftet', 'compulsory: inputs read once, slot outputs written '
                                     'once, backward reads grad + saved slots and writes the face gradients')}


def check_sign_bench(device, steps, n_points=1000000):
    """check_sign: the cfg3 sphere (50k faces) vs 1M points in [-1,1]^3."""
    import torch
    import kaolin as kal
    verts, faces = uv_sphere(126, 200, device)
    g = torch.Generator().manual_seed(3)
    pts = (torch.rand((1, n_points, 3), generator=g) * 2 - 1).to(device)
    v = verts.unsqueeze(0).contiguous()
    ms = _event_ms(lambda: kal.ops.mesh.check_sign(v, faces, pts), steps)
    nbytes = n_points * (12 + 1) + v.numel() * 4 + faces.numel() * 8
    return {'metric': 'check_sign Mpoints/s (1M points vs 50k-face sphere, f32)',
            'value': round(n_points / (ms * 1e-3) / 1e6, 1), 'ms': round(ms, 3),
            'nominal_mpairs_per_s': round(n_points * faces.shape[0] / (ms * 1e-3) / 1e6, 1),
            'roofline': roofline_hbm(nbytes, ms, 'check_sign', 'compulsory: points 12 B read + 1 B written, the mesh '
                                     'read once; the cell lists the kernels build and re-read are not counted')}


def soft_mask_c_leg(inp, steps):
    """The reference's _C contract soft-mask forward (dibr_soft_mask_forward_cuda: the (B,H,W,K) prob /
    idx / type slot tensors, what the reference's own tests and direct _C callers use) on the cfg3
    views, timed with HIP events; bytes by op_bytes (SURVEY.md 8d's soft-mask term)."""
    import torch
    import kaolin as kal
    stats = inp['stats']
    with torch.no_grad():
        _, fidx = kal.render.mesh.rasterize(inp['H'], inp['W'], inp['fvz'], inp['fvi'], inp['feat'], inp['fnz'] >= 0)
        fm = inp['fvi'] * 1000.
        bb = torch.cat([fm.min(-2)[0] - 20., fm.max(-2)[0] + 20.], -1).contiguous()
    fwd = lambda: kal._C.render.mesh.dibr_soft_mask_forward_cuda(fm, bb, fidx, 7000., 30, 1000.)  # noqa: E731
    ms = _event_ms(fwd, steps)
    nbytes = op_bytes('dibr_soft_mask_forward_cuda', inp, stats)
    B, H, W = inp['fvz'].shape[0], inp['H'], inp['W']
    torch.cuda.empty_cache()
    return {'metric': 'dibr_soft_mask_forward_cuda (_C contract, K=30 slot tensors) Mpixels/s, cfg3 views',
            'value': round(B * H * W / (ms * 1e-3) / 1e6, 1), 'ms': round(ms, 4),
            'roofline': roofline_hbm(nbytes, ms, 'soft_mask_C', 'SURVEY.md 8d soft fwd: sel 8 + mask 4 + K x (prob 4 '
                                     '+ idx 8 + type 1) per px, fvi 24 + bbox 16 per face')}


# ----------------------------------------------------------------------------- CPU self-test
def cpu_selftest(args, world, rank):
    """--device cpu: the launcher, the rendezvous, the sharded p2m leg (CPU path of
    point_to_mesh_distance) with its gather / all_reduce, and the max-over-ranks timing, on
    gloo.  The gathered result is checked against the unsharded op on every rank."""
    import torch
    import kaolin as kal
    dev = torch.device('cpu')
    g = torch.Generator().manual_seed(0)
    pts, fv = torch.randn((203, 3), generator=g), torch.randn((37, 3, 3), generator=g)
    grad = torch.rand((203,), generator=g)
    res, out, (gl, gfv) = p2m_leg(dev, world, rank, max(1, args.steps), pts, fv, grad)
    p = pts.clone().requires_grad_(True)
    f = fv.clone().requires_grad_(True)
    d, i, t = kal.metrics.trianglemesh.point_to_mesh_distance(p[None], f[None])
    d.backward(grad[None])
    from kaolin.distributed import shard_bounds
    lo, hi = shard_bounds(pts.shape[0], rank, world)
    ok = (torch.equal(out[0], d[0].detach()) and torch.equal(out[1], i[0]) and torch.equal(out[2], t[0])
          and torch.equal(gl, p.grad[lo:hi]) and torch.allclose(gfv, f.grad, rtol=1e-5, atol=1e-6))
    flags = [None] * world if world > 1 else [ok]
    if world > 1:
        import torch.distributed as dist
        dist.all_gather_object(flags, ok)
    if rank == 0:
        res['parity_all_ranks'] = all(flags)
        emit({'metric': 'cpu self-test (sharded point_to_mesh_distance over gloo)', 'n_ranks': world,
              'steps': args.steps, 'p2m': res})
    return 0 if all(flags) else 1


# ----------------------------------------------------------------------------- main
_LINE_OUT = None


def emit(obj):
    """The one JSON line, on the process's original stdout (library chatter went to stderr)."""
    out = _LINE_OUT or sys.stdout
    out.write(json.dumps(obj) + '\n')
    out.flush()


def _guard_stdout():
    """Send everything written to fd 1 from here on to stderr, keeping the original stdout for the
    JSON line: RCCL prints its version banner on stdout at communicator setup (seen on the GPU box,
    gpurun_out/r06a), once per rank under torchrun, and the driver reads rank 0's stdout as ONE line."""
    global _LINE_OUT
    if _LINE_OUT is None:
        sys.stdout.flush()
        _LINE_OUT = os.fdopen(os.dup(1), 'w')
        os.dup2(2, 1)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, argv)
    _guard_stdout()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        print(f'bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to time a different job',
              file=sys.stderr)
        return 2
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    import torch.distributed as dist
    if args.device == 'cpu':
        if world > 1:
            dist.init_process_group('gloo')
        try:
            return cpu_selftest(args, world, rank)
        finally:
            if world > 1:
                dist.destroy_process_group()
    # KAOLIN_BENCH_SHARED_GPU=1: a rehearsal of the N-rank flow on a box with fewer GPUs (ranks share
    # the devices round-robin, gloo instead of RCCL: RCCL takes one rank per GPU) -- the job's
    # timings are then not the N-GPU job's and the line says so in process_group.backend
    shared = os.environ.get('KAOLIN_BENCH_SHARED_GPU') == '1'
    if shared:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device('cuda', local)
    if os.environ.get('KAOLIN_DEV_FLAGS'):  # development A/B timing only (kl_dev_set_flags); unset in the product run
        import ctypes
        from kaolin import _native
        lib = _native.lib()
        lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
        lib.kl_dev_set_flags(int(os.environ['KAOLIN_DEV_FLAGS'], 0))
    if os.environ.get('KAOLIN_DEV_PARAMS'):  # "index=value,..." (kl_dev_set_param), development sweeps only
        import ctypes
        from kaolin import _native
        lib = _native.lib()
        lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
        for kv in os.environ['KAOLIN_DEV_PARAMS'].split(','):
            k, v = kv.split('=')
            lib.kl_dev_set_param(int(k), int(v))
    if world == 1 and args.collectives:  # a one-rank RCCL group on 127.0.0.1 (no launcher)
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(_free_port()))
        dist.init_process_group('nccl', device_id=device, rank=0, world_size=1)
    if world > 1:
        if shared:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=device)
    progress(f'rank {rank}/{world}: DIB-R {args.config} headline')
    result, inp = dibr_headline(args, world, rank, device)
    if not args.no_p2m:
        progress('p2m leg')
        p2m_res, p2m_out, p2m_grads = p2m_leg(device, world, rank, max(5, args.steps // 2))
        if rank == 0:
            result['p2m'] = p2m_res
            pts, fv, _ = p2m_inputs(device)
            result['p2m']['parity'] = p2m_parity(pts, fv, p2m_out)
            if world == 1 and not args.no_cpu_baseline:
                progress('p2m cpu leg')
                result['p2m']['cpu'] = p2m_cpu_legs(pts, fv)
    if rank == 0 and not args.no_extra:
        progress('cfg4 leg')
        c4 = cfg4_leg(device, args.steps)
        spc_tuple = c4.pop('spc')
        result['cfg4'] = c4
        progress('raytrace leg')
        result['raytrace'] = raytrace_leg(device, args.steps, spc_tuple)
        del spc_tuple
        progress('cfg1 sided leg')
        result['cfg1_sided'] = sided_leg(device, max(5, args.steps))
        if world == 1 and not args.no_cpu_baseline:
            progress('cfg4 cpu leg')
            result['cfg4']['cpu'] = cfg4_cpu_leg(device)
        progress('deftet / check_sign legs')
        if args.config == 'cfg3':
            result['deftet'] = deftet_bench(inp, max(3, args.steps // 4))
        result['check_sign'] = check_sign_bench(device, max(3, args.steps // 4))
        if args.config == 'cfg3':
            progress('_C soft mask leg')
            result['soft_mask_C'] = soft_mask_c_leg(inp, max(5, args.steps // 2))
        progress('prepare_vertices leg')
        result['prepare_vertices'] = prepare_leg(device, args.steps)
        if args.config == 'cfg3':
            progress('tutorial loop leg')
            result['tutorial'] = tutorial_leg(device, max(10, args.steps))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        row_step = args.cpu_row_step or CONFIGS[args.config]['row_step']
        progress(f'DIB-R parity + cpu baseline (oracle, every {row_step}th row)')
        parity, cpu = dibr_parity_and_cpu(inp, row_step)
        result['parity'] = parity
        result['cpu_baseline'] = cpu
        result['cpu_host'] = cpu_info()
    if rank == 0:
        emit(result)
    if collectives_on():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
