"""face_normals (kaolin/ops/mesh/trianglemesh.py:313-336), used to build DIB-R's
``face_normals_z`` input."""
import torch


def face_normals(face_vertices, unit=False):
    if face_vertices.shape[-2] != 3:
        raise NotImplementedError("face_normals: triangle meshes only (3 vertices per face)")
    edges_dist0 = face_vertices[:, :, 1] - face_vertices[:, :, 0]
    edges_dist1 = face_vertices[:, :, 2] - face_vertices[:, :, 0]
    normals = torch.cross(edges_dist0, edges_dist1, dim=2)
    if unit:
        length = normals.norm(dim=2, keepdim=True)
        normals = normals / (length + 1e-10)
    return normals
