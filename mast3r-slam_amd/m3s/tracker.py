"""Frame tracker's pose optimisation (mirror of mast3r_slam/tracker.py:15-266).

``FrameTracker`` keeps the reference's method names and argument meaning; the Gauss-Newton
loops ``opt_pose_ray_dist_sim3`` (:173-214) and ``opt_pose_calib_sim3`` (:216-266) run as ONE
op on the GPU (``mast3r_slam_backends.track_sim3``: hand-written HIP, track.hip) instead of
~30 torch kernels, a host sync and a Cholesky per iteration.  Poses are lietorch Sim3
``.data`` tensors ([1,8] = t, q xyzw, s) wrapped in ``PoseBatch``.  A non positive-definite
system raises ``mast3r_slam_backends.CholeskyError`` (a RuntimeError), which ``track``
catches like the reference (:72-93).

``track_matched`` is ``track`` (:28-127) after the network: it takes the outputs of
``mast3r_match_asymmetric`` (not on this path) and does the confidence combination,
validity gating, pose optimisation, keyframe point-map update and keyframe selection.
"""
from __future__ import annotations

import torch

import mast3r_slam_backends

from .config import config as _global_config
from .frame import Frame
from .geometry import constrain_points_to_ray, get_pixel_coords
from .global_opt import PoseBatch


class FrameTracker:
    def __init__(self, model=None, frames=None, device="cuda", cfg=None, use_calib=None):
        full = cfg if cfg is not None else _global_config
        self.cfg = full["tracking"]
        self.use_calib = full.get("use_calib", False) if use_calib is None else use_calib
        self.model = model
        self.keyframes = frames
        self.device = device
        self.reset_idx_f2k()

    def reset_idx_f2k(self):
        self.idx_f2k = None

    # -- tracker.py:129-154 -------------------------------------------------------------
    def get_points_poses(self, frame, keyframe, idx_f2k, img_size, use_calib, K=None):
        Xf, Xk = frame.X_canon, keyframe.X_canon
        T_WCf, T_WCk = frame.T_WC, keyframe.T_WC
        Cf, Ck = frame.get_average_conf(), keyframe.get_average_conf()
        meas_k = valid_meas_k = None
        if use_calib:
            Xf = constrain_points_to_ray(img_size, Xf[None], K).squeeze(0)
            Xk = constrain_points_to_ray(img_size, Xk[None], K).squeeze(0)
            uv_k = get_pixel_coords(1, img_size, device=Xf.device, dtype=Xf.dtype).view(-1, 2)
            meas_k = torch.cat((uv_k, torch.log(Xk[..., 2:3])), dim=-1)
            valid_meas_k = Xk[..., 2:3] > self.cfg["depth_eps"]
            meas_k[~valid_meas_k.repeat(1, 3)] = 0.0
        return Xf[idx_f2k], Xk, T_WCf, T_WCk, Cf[idx_f2k], Ck, meas_k, valid_meas_k

    # -- tracker.py:173-266 -------------------------------------------------------------
    def opt_pose_ray_dist_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid):
        c = self.cfg
        Tf, Tr, self.last_iters, self.last_cost = mast3r_slam_backends.track_sim3(
            "rays", Xf.contiguous(), Xk.contiguous(), _data(T_WCf), _data(T_WCk),
            Qk.contiguous(), valid.contiguous(), c["sigma_ray"], c["sigma_dist"], c["huber"],
            c["max_iters"], c["rel_error"], c["delta_norm"])
        return PoseBatch(Tf), PoseBatch(Tr)

    def opt_pose_calib_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K,
                            img_size):
        c = self.cfg
        Tf, Tr, self.last_iters, self.last_cost = mast3r_slam_backends.track_sim3(
            "calib", Xf.contiguous(), None, _data(T_WCf), _data(T_WCk), Qk.contiguous(),
            valid.contiguous(), c["sigma_pixel"], c["sigma_depth"], c["huber"], c["max_iters"],
            c["rel_error"], c["delta_norm"], meas_k=meas_k.contiguous(),
            valid_meas_k=valid_meas_k.contiguous(), K=K.contiguous(), img_size=img_size,
            pixel_border=c["pixel_border"], z_eps=c["depth_eps"])
        return PoseBatch(Tf), PoseBatch(Tr)

    # -- tracker.py:28-127 after mast3r_match_asymmetric ----------------------------------
    def track_matched(self, frame, keyframe, idx_f2k, valid_match_k, Xff, Cff, Qff, Xkf, Ckf, Qkf):
        """Returns (new_kf, [X_k, C_k, X_f, C_f, Qkf, Qff] | [], try_reloc) like track()."""
        self.idx_f2k = idx_f2k.clone()
        idx_f2k = idx_f2k[0]
        valid_match_k = valid_match_k[0]
        Qk = torch.sqrt(Qff[idx_f2k] * Qkf)
        frame.update_pointmap(Xff, Cff)
        img_size = frame.img.shape[-2:]
        K = keyframe.K if self.use_calib else None
        Xf, Xk, T_WCf, T_WCk, Cf, Ck, meas_k, valid_meas_k = self.get_points_poses(
            frame, keyframe, idx_f2k, img_size, self.use_calib, K)
        valid_opt = valid_match_k & (Cf > self.cfg["C_conf"]) & (Ck > self.cfg["C_conf"]) & \
            (Qk > self.cfg["Q_conf"])
        valid_kf = valid_match_k & (Qk > self.cfg["Q_conf"])
        if valid_opt.sum() / valid_opt.numel() < self.cfg["min_match_frac"]:
            return False, [], True
        try:
            if not self.use_calib:
                T_WCf, T_CkCf = self.opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid_opt)
            else:
                T_WCf, T_CkCf = self.opt_pose_calib_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid_opt,
                                                         meas_k, valid_meas_k, K, img_size)
        except RuntimeError:
            return False, [], True
        frame.T_WC = T_WCf
        if isinstance(keyframe, Frame):  # the transform fused into the point-map update
            keyframe.update_pointmap(Xkf, Ckf, T=_data(T_CkCf))
        else:
            keyframe.update_pointmap(_act(T_CkCf, Xkf), Ckf)
        n_valid = valid_kf.sum()
        match_frac_k = n_valid / valid_kf.numel()
        unique_frac_f = torch.unique(idx_f2k[valid_match_k[:, 0]]).shape[0] / valid_kf.numel()
        new_kf = min(match_frac_k, unique_frac_f) < self.cfg["match_frac_thresh"]
        if new_kf:
            self.reset_idx_f2k()
        return new_kf, [keyframe.X_canon, keyframe.get_average_conf(), frame.X_canon,
                        frame.get_average_conf(), Qkf, Qff], False


def _data(T):
    d = T.data if hasattr(T, "data") and not isinstance(T, torch.Tensor) else T
    return d.reshape(1, 8).contiguous()


def _act(T, p):
    """lietorch Sim3 act (s R p + t) on [..., 3] points, T data [1,8]."""
    d = _data(T)[0]
    t, q, s = d[0:3], d[3:7], d[7]
    u, w = q[:3].expand_as(p), q[3]
    uv = 2.0 * torch.cross(u, p, dim=-1)
    return s * (p + w * uv + torch.cross(u, uv, dim=-1)) + t
