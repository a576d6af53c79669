"""Geometry helpers on the GN calib path (mirror of mast3r_slam/geometry.py:37-42, 107-123).

``constrain_points_to_ray`` keeps only each canonical point's depth and re-projects it
along its pixel's ray through K, as solve_GN_calib does before the op
(global_opt.py:172).
"""
from __future__ import annotations

import torch


def get_pixel_coords(b, img_size, device, dtype):
    h, w = img_size
    v, u = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    uv = torch.stack((u, v), dim=-1)[None].repeat(b, 1, 1, 1)
    return uv.to(device=device, dtype=dtype)


def backproject(p, z, K):
    """pixels p[...,2], depth z[...,1] -> points z * ((u-cx)/fx, (v-cy)/fy, 1)."""
    x = (p[..., 0] - K[0, 2]) / K[0, 0]
    y = (p[..., 1] - K[1, 2]) / K[1, 1]
    ray = torch.stack((x, y, torch.ones_like(x)), dim=-1).to(K.dtype)
    return z * ray


def constrain_points_to_ray(img_size, Xs, K):
    uv = get_pixel_coords(Xs.shape[0], img_size, device=Xs.device, dtype=Xs.dtype)
    uv = uv.view(*Xs.shape[:-1], 2)
    return backproject(uv, Xs[..., 2:3], K)
