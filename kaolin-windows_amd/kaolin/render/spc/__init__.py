from .raytrace import (unbatched_raytrace, mark_pack_boundaries, mark_first_hit, diff, sum_reduce,  # noqa: F401
                       cumsum, cumprod, exponential_integration)
