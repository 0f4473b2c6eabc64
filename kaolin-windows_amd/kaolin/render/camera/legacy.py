"""Legacy camera helpers used only to PREPARE rasterizer inputs (kaolin/render/camera/legacy.py:22-159).
Pure PyTorch: not part of the accelerated path."""
from math import tan

import torch


def rotate_translate_points(points, camera_rot, camera_trans):
    translated_points = points - camera_trans.view(-1, 1, 3)
    return torch.matmul(translated_points, camera_rot.permute(0, 2, 1))


def generate_rotate_translate_matrices(camera_position, look_at, camera_up_direction):
    """Look-at camera frame (legacy.py:40-83): rows x, y, -z with z = normalize(look_at - pos)."""
    fwd = look_at - camera_position
    fwd = fwd / (fwd.norm(dim=1, keepdim=True) + 1e-10)
    up = camera_up_direction
    if up.shape[0] < fwd.shape[0]:
        up = up.repeat(fwd.shape[0], 1)
    elif up.shape[0] > fwd.shape[0]:
        fwd = fwd.repeat(up.shape[0], 1)
    right = torch.cross(fwd, up, dim=1)
    right = right / (right.norm(dim=1, keepdim=True) + 1e-10)
    true_up = torch.cross(right, fwd, dim=1)
    true_up = true_up / (true_up.norm(dim=1, keepdim=True) + 1e-10)
    return torch.stack([right, true_up, -fwd], dim=1), camera_position


def perspective_camera(points, camera_proj):
    projected_points = points * camera_proj.view(-1, 1, 3)
    return projected_points[:, :, :2] / projected_points[:, :, 2:3]


def generate_perspective_projection(fovyangle, ratio=1.0, dtype=torch.float):
    tanfov = tan(fovyangle / 2.0)
    return torch.tensor([[1.0 / (ratio * tanfov)], [1.0 / tanfov], [-1]], dtype=dtype)
