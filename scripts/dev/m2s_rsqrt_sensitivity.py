"""How many of mesh_to_spc's separating-axis decisions at cfg4 (200k-face sphere, L=9) can the
edge normalisation's rounding flip?  The reference uses CUDA's double rsqrt (1 ulp, not
correctly rounded; mesh_to_spc_cuda.cu:123-125, spc_math.h:240-243), this build 1.0 / sqrt.
CPU only (the oracle's counter, OpenMP); writes profiles/r03_m2s_rsqrt_sensitivity.json."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'kaolin-windows_amd')]

import bench  # noqa: E402
from oracle import oracle as orc  # noqa: E402

verts, faces = bench.cfg4_inputs('cpu')
fv = verts[faces].numpy()
t0 = time.time()
res = orc.m2s_rsqrt_sensitivity(fv, 9)
res.update(mesh='cfg4 UV sphere 251x400 (200,000 faces), radius 0.95', level=9, seconds=round(time.time() - t0, 1))
print(json.dumps(res))
with open(os.path.join(ROOT, 'profiles', 'r03_m2s_rsqrt_sensitivity.json'), 'w') as f:
    json.dump(res, f, indent=1)
