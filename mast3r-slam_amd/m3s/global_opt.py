"""Factor-graph side of the GN op (mirror of mast3r_slam/global_opt.py:12-213).

``FactorGraph`` keeps the reference's edge store (ii, jj, idx_ii2jj, idx_jj2ii,
valid_match_j/i, Q_ii2jj/jj2ii), builds the two-way edge set exactly like
``prep_two_way_edges`` (:104-110), stacks poses/points/confidences of the unique
keyframes in sorted-id order (``get_poses_points``, :112-119) and hands the op the same
positional arguments (``solve_GN_rays`` :121-158, ``solve_GN_calib`` :160-213; checked
against the reference in tests/test_glue_golden.py).  ``Twc`` is updated in place by
the op and written back with ``frames.update_T_WCs``.

The network half of ``add_factors`` (MASt3R symmetric decoding, :30-52) is outside the
hot path; ``add_matched_factors`` takes its outputs and applies the reference's
Q-combination and match-fraction gating (:53-99).

``frames`` is duck-typed like the reference's SharedKeyframes: ``frames[i]`` returns an
object with ``X_canon``, ``T_WC.data``, ``get_average_conf()`` and ``img``; plus
``update_T_WCs(T, idx)``.  ``KeyframeStore`` is a device-resident implementation.
"""
from __future__ import annotations

import torch

import mast3r_slam_backends

from .config import config as _global_config
from .geometry import constrain_points_to_ray


class PoseBatch:
    """Stand-in for the lietorch.Sim3 container the reference passes around: ``.data``
    is ``[N,1,8]`` = ``[t(3), q(4, xyzw), s]`` (lietorch embedding)."""

    def __init__(self, data):
        self.data = data

    def __getitem__(self, k):
        return PoseBatch(self.data[k])


class _KeyframeView:
    def __init__(self, store, i):
        self._s, self._i = store, i

    @property
    def X_canon(self):
        return self._s.X[self._i]

    @property
    def T_WC(self):
        return PoseBatch(self._s.T_WC[self._i])

    @property
    def img(self):
        return self._s.img_placeholder

    def get_average_conf(self):
        return self._s.C[self._i] / self._s.n_obs[self._i]


class KeyframeStore:
    """Fixed-capacity device-resident keyframe buffers (the layout the GN op reads:
    X [cap,HW,3], T_WC [cap,1,8], C [cap,HW,1]) -- cf. frame.py:220-327."""

    def __init__(self, capacity, h, w, device="cuda"):
        hw = h * w
        self.h, self.w = h, w
        self.X = torch.zeros((capacity, hw, 3), device=device)
        self.C = torch.zeros((capacity, hw, 1), device=device)
        self.n_obs = torch.ones((capacity,), device=device)
        self.T_WC = torch.zeros((capacity, 1, 8), device=device)
        self.T_WC[:, 0, 6] = 1.0
        self.T_WC[:, 0, 7] = 1.0
        self.img_placeholder = torch.zeros((3, h, w), device="cpu")
        self.size = 0

    def append(self, X, C, T_WC):
        k = self.size
        self.X[k] = X
        self.C[k] = C
        self.T_WC[k, 0] = T_WC
        self.size += 1
        return k

    def __len__(self):
        return self.size

    def __getitem__(self, i):
        return _KeyframeView(self, int(i))

    def update_T_WCs(self, T_WCs, idx):
        self.T_WC[idx] = T_WCs.data


class FactorGraph:
    def __init__(self, model, frames, K=None, device="cuda", cfg=None):
        self.model = model
        self.frames = frames
        self.device = device
        self.cfg = (cfg if cfg is not None else _global_config)["local_opt"]
        empty = lambda dt: torch.as_tensor([], dtype=dt, device=device)
        self.ii = empty(torch.long)
        self.jj = empty(torch.long)
        self.idx_ii2jj = empty(torch.long)
        self.idx_jj2ii = empty(torch.long)
        self.valid_match_j = empty(torch.bool)
        self.valid_match_i = empty(torch.bool)
        self.Q_ii2jj = empty(torch.float32)
        self.Q_jj2ii = empty(torch.float32)
        self.window_size = self.cfg["window_size"]
        self.K = K

    # -- edge construction after the network (global_opt.py:53-99) -------------------
    def add_matched_factors(self, ii, jj, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii,
                            Qjj, Qji, Qij, min_match_frac, is_reloc=False):
        # Qj/Qi and the per-pair valid counts in one HIP pass (edges.hip; :53-67)
        Qj, Qi, counts = mast3r_slam_backends.edge_confidence(
            idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij, self.cfg["Q_conf"])
        frac_j = counts[:, 0] / (valid_match_j.shape[1] * valid_match_j.shape[2])
        frac_i = counts[:, 1] / (valid_match_i.shape[1] * valid_match_i.shape[2])

        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        # both directions must pass, except consecutive keyframes (always kept)
        invalid = (torch.minimum(frac_j, frac_i) < min_match_frac) & ~(ii_t == (jj_t - 1))
        if is_reloc and invalid.any():
            return False
        keep = ~invalid
        cat = torch.cat
        self.ii = cat([self.ii, ii_t[keep]])
        self.jj = cat([self.jj, jj_t[keep]])
        self.idx_ii2jj = cat([self.idx_ii2jj, idx_i2j[keep]])
        self.idx_jj2ii = cat([self.idx_jj2ii, idx_j2i[keep]])
        self.valid_match_j = cat([self.valid_match_j, valid_match_j[keep]])
        self.valid_match_i = cat([self.valid_match_i, valid_match_i[keep]])
        self.Q_ii2jj = cat([self.Q_ii2jj, Qj[keep]])
        self.Q_jj2ii = cat([self.Q_jj2ii, Qi[keep]])
        return bool(keep.sum() > 0)

    # -- the solve (global_opt.py:101-213) ---------------------------------------------
    def get_unique_kf_idx(self):
        return torch.unique(torch.cat([self.ii, self.jj]), sorted=True)

    def prep_two_way_edges(self):
        ii = torch.cat((self.ii, self.jj), dim=0)
        jj = torch.cat((self.jj, self.ii), dim=0)
        idx_ii2jj = torch.cat((self.idx_ii2jj, self.idx_jj2ii), dim=0)
        valid_match = torch.cat((self.valid_match_j, self.valid_match_i), dim=0)
        Q_ii2jj = torch.cat((self.Q_ii2jj, self.Q_jj2ii), dim=0)
        return ii, jj, idx_ii2jj, valid_match, Q_ii2jj

    def get_poses_points(self, unique_kf_idx):
        kfs = [self.frames[i] for i in unique_kf_idx]
        Xs = torch.stack([kf.X_canon for kf in kfs])
        T_WCs = PoseBatch(torch.stack([kf.T_WC.data for kf in kfs]))
        Cs = torch.stack([kf.get_average_conf() for kf in kfs])
        return Xs, T_WCs, Cs

    def _prepare(self):
        pin = self.cfg["pin"]
        unique_kf_idx = self.get_unique_kf_idx()
        if unique_kf_idx.numel() <= pin:
            return None
        Xs, T_WCs, Cs = self.get_poses_points(unique_kf_idx)
        return pin, unique_kf_idx, Xs, T_WCs, Cs

    def solve_GN_rays(self, backend=None):
        be = backend or mast3r_slam_backends
        prep = self._prepare()
        if prep is None:
            return
        pin, unique_kf_idx, Xs, T_WCs, Cs = prep
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        c = self.cfg
        pose_data = T_WCs.data[:, 0, :]  # a view: the op updates T_WCs in place
        be.gauss_newton_rays(
            pose_data, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q_ii2jj,
            c["sigma_ray"], c["sigma_dist"], c["C_conf"], c["Q_conf"], c["max_iters"],
            c["delta_norm"],
        )
        self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])

    def solve_GN_calib(self, backend=None):
        be = backend or mast3r_slam_backends
        prep = self._prepare()
        if prep is None:
            return
        pin, unique_kf_idx, Xs, T_WCs, Cs = prep
        height, width = self.frames[0].img.shape[-2:]
        Xs = constrain_points_to_ray((height, width), Xs, self.K)
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        c = self.cfg
        pose_data = T_WCs.data[:, 0, :]
        be.gauss_newton_calib(
            pose_data, Xs, Cs, self.K, ii, jj, idx_ii2jj, valid_match, Q_ii2jj, height, width,
            c["pixel_border"], c["depth_eps"], c["sigma_pixel"], c["sigma_depth"], c["C_conf"],
            c["Q_conf"], c["max_iters"], c["delta_norm"],
        )
        self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])
