"""Keyframe point-map state (mirror of mast3r_slam/frame.py:17-108).

``Frame`` keeps the reference's fields (frame_id, img, T_WC, X_canon, C, N, N_updates, K) and
``update_pointmap`` follows frame.py:41-105 mode by mode.  The per-point modes
(weighted_pointmap -- the default, base.yaml:32 -- indep_conf, recent, first) run as one
fused HIP pass (``mast3r_slam_backends.pointmap_update``, keyframe.hip), optionally fused with
the Sim3 transform the tracker applies to the observation (tracker.py:98-99); best_score and
weighted_spherical stay torch expressions as in the reference.  Like the other ops there is
no CPU path for the fused modes.
"""
from __future__ import annotations

import torch

import mast3r_slam_backends

from .config import config as _global_config
from .global_opt import PoseBatch


class Frame:
    def __init__(self, frame_id=0, img=None, T_WC=None, X_canon=None, C=None, K=None, cfg=None):
        self.frame_id = frame_id
        self.img = img
        self.T_WC = T_WC if T_WC is not None else PoseBatch(_identity())
        self.X_canon = X_canon
        self.C = C
        self.N = 0
        self.N_updates = 0
        self.K = K
        self.score = None
        self._cfg = cfg

    @property
    def cfg(self):
        return (self._cfg if self._cfg is not None else _global_config)["tracking"]

    def get_score(self, C):  # frame.py:33-39
        return torch.median(C) if self.cfg["filtering_score"] == "median" else torch.mean(C)

    def update_pointmap(self, X, C, T=None):
        """frame.py:41-105; ``T`` (Sim3 data) transforms X first, as tracker.py:98 does."""
        mode = self.cfg["filtering_mode"]
        if self.N == 0:  # :44-51
            self.X_canon = _act_copy(X, T)
            self.C = C.clone()
            self.N = 1
            self.N_updates = 1
            if mode == "best_score":
                self.score = self.get_score(C)
            return
        if mode == "first":  # :53-57
            if self.N_updates == 1:
                mast3r_slam_backends.pointmap_update("recent", self.X_canon, self.C, X, C, T)
                self.N = 1
        elif mode == "recent":  # :58-61
            mast3r_slam_backends.pointmap_update("recent", self.X_canon, self.C, X, C, T)
            self.N = 1
        elif mode == "best_score":  # :62-68
            new_score = self.get_score(C)
            if new_score > self.score:
                self.X_canon = _act_copy(X, T)
                self.C = C.clone()
                self.N = 1
                self.score = new_score
        elif mode == "indep_conf":  # :69-73
            mast3r_slam_backends.pointmap_update("indep_conf", self.X_canon, self.C, X, C, T)
            self.N = 1
        elif mode == "weighted_pointmap":  # :74-77
            mast3r_slam_backends.pointmap_update("weighted_pointmap", self.X_canon, self.C, X, C, T)
            self.N += 1
        elif mode == "weighted_spherical":  # :78-102
            X = _act_copy(X, T)

            def to_sph(P):
                r = torch.linalg.norm(P, dim=-1, keepdim=True)
                x, y, z = torch.tensor_split(P, 3, dim=-1)
                return torch.cat((r, torch.atan2(y, x), torch.acos(z / r)), dim=-1)

            def to_cart(S):
                r, phi, theta = torch.tensor_split(S, 3, dim=-1)
                return torch.cat((r * torch.sin(theta) * torch.cos(phi),
                                  r * torch.sin(theta) * torch.sin(phi), r * torch.cos(theta)), dim=-1)

            sph = ((self.C * to_sph(self.X_canon)) + (C * to_sph(X))) / (self.C + C)
            self.X_canon = to_cart(sph)
            self.C = self.C + C
            self.N += 1
        else:
            raise ValueError(f"unknown filtering_mode {mode!r}")
        self.N_updates += 1

    def get_average_conf(self):  # frame.py:107-108
        return self.C / self.N if self.C is not None else None


def _identity():
    d = torch.zeros((1, 8))
    d[0, 6] = 1.0
    d[0, 7] = 1.0
    return d


def _act_copy(X, T):
    if T is None:
        return X.clone()
    out = torch.empty_like(X)
    C0 = torch.zeros((X.shape[0], 1), dtype=X.dtype, device=X.device)
    mast3r_slam_backends.pointmap_update("recent", out, C0, X.contiguous(), C0.clone(), T)
    return out
