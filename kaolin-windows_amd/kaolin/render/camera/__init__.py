from .legacy import (generate_perspective_projection, generate_rotate_translate_matrices,  # noqa: F401
                     rotate_translate_points, perspective_camera)
