from .mesh import index_vertices_by_faces  # noqa: F401
from .trianglemesh import face_normals  # noqa: F401
from .check_sign import check_sign  # noqa: F401
