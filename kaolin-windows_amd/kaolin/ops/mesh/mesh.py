"""Input preparation used by the hot path (kaolin/ops/mesh/mesh.py:25-46)."""
import torch


def index_vertices_by_faces(vertices_features, faces):
    r"""Per-vertex features (B, V, K) -> per-face-vertex features (B, F, n, K)."""
    assert vertices_features.ndim == 3, \
        "vertices_features: expected a (batch_size, num_points, knum) tensor"
    assert faces.ndim == 2, "faces: expected a (num_faces, num_vertices) tensor"
    inp = vertices_features.unsqueeze(2).expand(-1, -1, faces.shape[-1], -1)
    indices = faces[None, ..., None].expand(vertices_features.shape[0], -1, -1, vertices_features.shape[-1])
    return torch.gather(input=inp, index=indices, dim=1)
