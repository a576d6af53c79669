"""Iterative projective matching -- caller of the two matching ops.

Mirror of mast3r_slam/matching.py:8-90 (same function names, arguments and outputs):

* ``prep_for_iter_proj``: normalised ray image + its gradient packed to 9 channels,
  normalised target rays, identity or warm-start initial pixels (matching.py:25-49);
* ``match_iterative_proj``: iter_proj -> ``p.long()`` truncation -> 3D occlusion test on
  the PRE-refine pixels -> refine_matches on fp16 descriptors -> linear index
  (matching.py:52-90).

On HIP tensors ``match_iterative_proj`` runs as ONE op (``mast3r_slam_backends.match_iterative_proj``:
prep, iter_proj, occlusion, refine and the linear index in four launches, the glue's float ops in
the reference's host arithmetic); ``fused=False`` runs the torch glue below around the two
reference ops instead (its normalize / conv2d round as torch's GPU kernels do).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import mast3r_slam_backends

from .config import config as _global_config
from .image import img_gradient


def match(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=None):
    return match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init, cfg=cfg)


def pixel_to_lin(p1, w):
    """(u, v) -> u + w*v  (matching.py:13-15)."""
    return p1[..., 0] + w * p1[..., 1]


def lin_to_pixel(idx_1_to_2, w):
    """u + w*v -> (u, v)  (matching.py:18-22)."""
    return torch.stack((idx_1_to_2 % w, idx_1_to_2 // w), dim=-1)


def prep_for_iter_proj(X11, X21, idx_1_to_2_init):
    b, h, w, _ = X11.shape
    rays = F.normalize(X11, dim=-1).permute(0, 3, 1, 2)  # [b,3,h,w]
    gx, gy = img_gradient(rays)
    rays_with_grad = torch.cat((rays, gx, gy), dim=1).permute(0, 2, 3, 1).contiguous()

    pts3d_norm = F.normalize(X21.view(b, -1, 3), dim=-1)

    if idx_1_to_2_init is None:
        idx_1_to_2_init = torch.arange(h * w, device=X11.device)[None, :].repeat(b, 1)
    p_init = lin_to_pixel(idx_1_to_2_init, w).float()
    return rays_with_grad, pts3d_norm, p_init


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=None, fused=None, contract=None):
    """``contract``: iter_proj's FMA-contraction convention (default: the reference build's,
    mast3r_slam_backends.CONTRACT)."""
    cfg = (cfg if cfg is not None else _global_config)["matching"]
    b, h, w = X21.shape[:3]
    device = X11.device
    if fused is None:
        fused = device.type == "cuda" and hasattr(mast3r_slam_backends, "match_iterative_proj")
    if fused:
        idx_1_to_2, valid = mast3r_slam_backends.match_iterative_proj(
            X11.contiguous(), X21.contiguous(), D11.contiguous(), D21.contiguous(),
            None if idx_1_to_2_init is None else idx_1_to_2_init.contiguous(),
            cfg["max_iter"], cfg["lambda_init"], cfg["convergence_thresh"], cfg["dist_thresh"],
            cfg["radius"], cfg["dilation_max"], contract=contract,
        )
        return idx_1_to_2, valid

    rays_with_grad, pts3d_norm, p_init = prep_for_iter_proj(X11, X21, idx_1_to_2_init)
    p1, valid_proj2 = mast3r_slam_backends.iter_proj(
        rays_with_grad, pts3d_norm, p_init,
        cfg["max_iter"], cfg["lambda_init"], cfg["convergence_thresh"],
        **({} if contract is None else {"contract": contract}),
    )
    p1 = p1.long()

    # occlusion: the matched 3D point must lie near the query point (pre-refine p1)
    bi = torch.arange(b, device=device)[:, None].expand(b, h * w)
    X11_at_p1 = X11[bi, p1[..., 1], p1[..., 0], :].reshape(b, h, w, 3)
    dists2 = torch.linalg.norm(X11_at_p1 - X21, dim=-1)
    valid_proj2 = valid_proj2 & (dists2 < cfg["dist_thresh"]).view(b, -1)

    if cfg["radius"] > 0:
        (p1,) = mast3r_slam_backends.refine_matches(
            D11.half(), D21.view(b, h * w, -1).half(), p1, cfg["radius"], cfg["dilation_max"]
        )

    idx_1_to_2 = pixel_to_lin(p1, w)
    return idx_1_to_2, valid_proj2.unsqueeze(-1)
