"""cfg4 mesh_to_spc (L=9, 200k-face sphere) after warm-up, for a rocprofv3 --kernel-trace of its kernels in
order (development aid): python scripts/dev/m2s_trace.py [calls]"""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for _ in range(n):
        out = kal.ops.conversions.unbatched_mesh_to_spc(fv, 9)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        out = kal.ops.conversions.unbatched_mesh_to_spc(fv, 9)
    e.record()
    torch.cuda.synchronize()
    print(f'mesh_to_spc {s.elapsed_time(e) / 10:.4f} ms, nodes {out[0].shape[0]}', flush=True)


if __name__ == '__main__':
    main()
