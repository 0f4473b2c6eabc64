from .spc import scan_octrees, generate_points  # noqa: F401
from .points import points_to_morton, morton_to_points, unbatched_points_to_octree  # noqa: F401
