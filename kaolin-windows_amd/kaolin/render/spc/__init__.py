from .raytrace import unbatched_raytrace, mark_pack_boundaries, mark_first_hit  # noqa: F401
