"""kaolin (MI355X): Kaolin 0.14's differentiable-rendering / 3D-conversion hot path,
re-implemented for AMD Instinct MI355X (gfx950) behind the reference's Python API.

Scope: DIB-R rasterize + soft mask (fwd/bwd), point_to_mesh_distance,
sided_distance (+ chamfer / f_score), trianglemeshes_to_voxelgrids,
unbatched_mesh_to_spc, scan_octrees / generate_points, unbatched_raytrace.
GPU tensors run through libkaolin_hip.so (hand-written HIP, C ABI); the two front-ends the
reference runs on CPU (point_to_mesh_distance, trianglemeshes_to_voxelgrids) keep a torch CPU path.
"""
__version__ = '0.14.0+mi355x'

from . import _C  # noqa: F401
from . import ops  # noqa: F401
from . import metrics  # noqa: F401
from . import render  # noqa: F401
from . import utils  # noqa: F401
from . import distributed  # noqa: F401
