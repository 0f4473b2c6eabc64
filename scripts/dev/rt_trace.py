"""cfg4 raytrace (level 9 SPC of the 200k-face sphere, 512^2 rays) after warm-up, for a rocprofv3
--kernel-trace of its kernels in order (development aid): python scripts/dev/rt_trace.py [calls]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import kaolin as kal
    verts, faces = bench.cfg4_inputs('cuda')
    fv = kal.ops.mesh.index_vertices_by_faces(verts[None], faces)[0].contiguous()
    octree = kal.ops.conversions.unbatched_mesh_to_spc(fv, 9)[0]
    lengths = torch.tensor([octree.shape[0]], dtype=torch.int32)
    L, pyr, exsum = kal.ops.spc.scan_octrees(octree, lengths)
    pts = kal.ops.spc.generate_points(octree, pyr, exsum)
    n = 512
    xs = (torch.arange(n, device='cuda', dtype=torch.float32) + 0.5) / n * 2 - 1
    tgt = torch.stack([xs.view(1, -1).expand(n, n), xs.view(-1, 1).expand(n, n), torch.zeros(n, n, device='cuda')], -1)
    o = torch.tensor([0., 0., 3.], device='cuda').expand(n * n, 3).contiguous()
    d = tgt.reshape(-1, 3) - o
    d = (d / d.norm(dim=-1, keepdim=True)).contiguous()
    rt = lambda: kal.render.spc.unbatched_raytrace(octree, pts, pyr[0], exsum, o, d, L)  # noqa: E731
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for _ in range(k):
        out = rt()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        out = rt()
    e.record()
    torch.cuda.synchronize()
    print(f'raytrace {s.elapsed_time(e) / 10:.4f} ms, hits {out[0].shape[0]}', flush=True)


if __name__ == '__main__':
    main()
