"""Host cost of the tutorial-shape eager step (bench.tutorial_shape_step), piece by piece
(development aid): each piece is called N times back to back with no sync, so the loop time is the
host's (the GPU trails); then a cProfile of whole steps.  usage: python scripts/dev/tutorial_host.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kaolin as kal  # noqa: E402


def host_us(fn, n=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def main():
    st = bench.tutorial_setup('cuda')
    B = st['B']
    vb = (kal.ops.pointcloud.center_points(st['vertices']) + st['shift']).detach()
    fvc, fvi, fn = kal.render.mesh.prepare_vertices(vb.repeat(B, 1, 1), st['faces'], st['cam_proj'],
                                                    camera_transform=st['cam_transform'])
    attrs = [st['face_uvs'].repeat(B, 1, 1, 1), torch.ones((B, st['F'], 3, 1), device='cuda')]
    fz, fn2 = fvc[:, :, :, -1].contiguous(), fn[:, :, -1].contiguous()
    pieces = {
        'step (fwd+bwd)': lambda: bench.tutorial_shape_step(st),
        'render (fwd only)': lambda: bench._tutorial_render(st),
        'center+shift+repeat': lambda: (kal.ops.pointcloud.center_points(st['vertices']) + st['shift']).repeat(B, 1, 1),
        'prepare_vertices': lambda: kal.render.mesh.prepare_vertices(vb.repeat(B, 1, 1), st['faces'], st['cam_proj'],
                                                                     camera_transform=st['cam_transform']),
        'attrs (repeat + ones)': lambda: [st['face_uvs'].repeat(B, 1, 1, 1), torch.ones((B, st['F'], 3, 1), device='cuda')],
        'dibr_rasterization(list)': lambda: kal.render.mesh.dibr_rasterization(512, 512, fz, fvi, attrs, fn2,
                                                                                rast_backend='cuda'),
        'mask_iou': lambda: kal.metrics.render.mask_iou(fz.new_ones((B, 512, 512)), st['gt_mask']),
    }
    for k, f in pieces.items():
        h, w = host_us(f)
        print(f'{k:28s} host {h:8.1f} us   wall {w:8.1f} us', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        bench.tutorial_shape_step(st)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
