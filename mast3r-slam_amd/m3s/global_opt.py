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

``DeviceFactorGraph`` is the same factor graph without the
per-solve copies: edges live in a device-resident two-way store (``EdgeStore``: forward and
backward halves, grown by doubling, appended in place) handed to the op as its two halves
(the op's ``second_half``), and, when the graph's keyframes are a contiguous range of a
``KeyframeStore``, poses / points / average confidences are views of the store's buffers
(the op updates the store's poses in place; the ray-constrained points and C / N are kept
per keyframe by the store, recomputed only when a keyframe changes).
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
    X [cap,HW,3], T_WC [cap,1,8], C [cap,HW,1]) -- cf. frame.py:220-327.

    Derived per-keyframe buffers for the zero-copy solve (DeviceFactorGraph): ``C_avg`` = C / N
    (get_average_conf, frame.py) and, with ``K``, ``X_ray`` = the points constrained to their
    pixel rays (geometry.py:37-42, what solve_GN_calib computes per call, global_opt.py:172).
    They are kept current by ``append`` / ``set_keyframe`` / ``refresh``; code that writes
    X / C / n_obs directly calls ``refresh(k)`` (the reference-compatible FactorGraph reads
    only X / C / n_obs / T_WC and needs nothing)."""

    def __init__(self, capacity, h, w, device="cuda", K=None):
        hw = h * w
        self.h, self.w = h, w
        self.X = torch.zeros((capacity, hw, 3), device=device)
        self.C = torch.zeros((capacity, hw, 1), device=device)
        self.n_obs = torch.ones((capacity,), device=device)
        self.T_WC = torch.zeros((capacity, 1, 8), device=device)
        self.T_WC[:, 0, 6] = 1.0
        self.T_WC[:, 0, 7] = 1.0
        self.C_avg = torch.zeros((capacity, hw, 1), device=device)
        self.K = K
        self.X_ray = torch.zeros((capacity, hw, 3), device=device) if K is not None else None
        self.img_placeholder = torch.zeros((3, h, w), device="cpu")
        self.size = 0

    def refresh(self, k):
        """Recompute keyframe k's derived rows (C / N; the ray-constrained points)."""
        self.C_avg[k] = self.C[k] / self.n_obs[k]
        if self.X_ray is not None:
            self.X_ray[k] = constrain_points_to_ray((self.h, self.w), self.X[k:k + 1], self.K)[0]

    def set_keyframe(self, k, X=None, C=None, T_WC=None, n_obs=None):
        if X is not None:
            self.X[k] = X
        if C is not None:
            self.C[k] = C
        if T_WC is not None:
            self.T_WC[k, 0] = T_WC
        if n_obs is not None:
            self.n_obs[k] = n_obs
        self.refresh(k)

    def append(self, X, C, T_WC, n_obs=None):
        k = self.size
        self.size += 1
        self.set_keyframe(k, X, C, T_WC, n_obs)
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

    @staticmethod
    def _check_solved(be, pose_data):
        """Raise a deferred solver error of the call just made before its poses are written back
        (ADVICE r04): a timed-out factorisation restores Twc on the device, and this makes the
        caller see the error in the same solve_GN_* call, as the reference's synchronous op would
        (its driver synchronises the host every iteration, gn_kernels.cu:1199-1222)."""
        check = getattr(be, "gn_check", None)
        if check is not None and pose_data.is_cuda:
            check(pose_data.device)

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
        self._check_solved(be, pose_data)
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
        self._check_solved(be, pose_data)
        self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])


class EdgeStore:
    """Device-resident two-way edge store: the forward edges' (ii, jj, idx_ii2jj, valid_match_j,
    Q_ii2jj) and the backward edges' (idx_jj2ii, valid_match_i, Q_jj2ii) in capacity buffers that
    grow by doubling, so adding factors appends in place (the reference concatenates the whole
    store on every add_factors, global_opt.py:89-96, and again on every solve, :104-110)."""

    def __init__(self, hw, device, capacity=16):
        self.hw, self.device, self.E = hw, device, 0
        self._alloc(capacity)

    def _alloc(self, cap):
        d, hw = self.device, self.hw
        new = dict(
            ii=torch.zeros((cap,), dtype=torch.long, device=d),
            jj=torch.zeros((cap,), dtype=torch.long, device=d),
            idx_f=torch.zeros((cap, hw), dtype=torch.long, device=d),
            idx_b=torch.zeros((cap, hw), dtype=torch.long, device=d),
            valid_f=torch.zeros((cap, hw, 1), dtype=torch.bool, device=d),
            valid_b=torch.zeros((cap, hw, 1), dtype=torch.bool, device=d),
            Q_f=torch.zeros((cap, hw, 1), dtype=torch.float32, device=d),
            Q_b=torch.zeros((cap, hw, 1), dtype=torch.float32, device=d),
        )
        if self.E:
            for k, t in new.items():
                t[: self.E] = getattr(self, "_" + k)[: self.E]
        for k, t in new.items():
            setattr(self, "_" + k, t)
        self.capacity = cap

    def append(self, ii, jj, idx_i2j, idx_j2i, valid_j, valid_i, Qj, Qi):
        n = ii.shape[0]
        if self.E + n > self.capacity:
            self._alloc(max(2 * self.capacity, self.E + n))
        sl = slice(self.E, self.E + n)
        self._ii[sl], self._jj[sl] = ii, jj
        self._idx_f[sl], self._idx_b[sl] = idx_i2j, idx_j2i
        self._valid_f[sl], self._valid_b[sl] = valid_j, valid_i
        self._Q_f[sl], self._Q_b[sl] = Qj, Qi
        self.E += n

    def view(self, name):
        return getattr(self, "_" + name)[: self.E]

    def forward(self):
        return self.view("idx_f"), self.view("valid_f"), self.view("Q_f")

    def backward(self):
        return self.view("idx_b"), self.view("valid_b"), self.view("Q_b")


class DeviceFactorGraph(FactorGraph):
    """FactorGraph over an EdgeStore and a KeyframeStore, solving without per-call copies.

    The reference attributes (ii, jj, idx_ii2jj, idx_jj2ii, valid_match_j/i, Q_ii2jj/jj2ii)
    are read-only views of the store; prep_two_way_edges still returns the reference's
    concatenation for callers that want it.  The solve hands the op the same directed edges
    in the same order ([forward; backward], global_opt.py:104-110) as two halves, so its result
    is bitwise the reference-compatible FactorGraph's (tests/test_gpu_factor_graph.py)."""

    def __init__(self, model, frames, K=None, device="cuda", cfg=None):
        self.edges = None  # created at the first add (its point count comes from the matches)
        super().__init__(model, frames, K=K, device=device, cfg=cfg)

    def _edge_view(name, dtype):
        def get(s):
            if s.edges is None:
                return torch.as_tensor([], dtype=dtype, device=s.device)
            return s.edges.view(name)

        def put(s, v):  # the base __init__ assigns the empty reference attributes
            if v.numel():
                raise AttributeError("DeviceFactorGraph edges are added with add_matched_factors")

        return property(get, put)

    # the reference's edge attributes, as views of the store
    ii = _edge_view("ii", torch.long)
    jj = _edge_view("jj", torch.long)
    idx_ii2jj = _edge_view("idx_f", torch.long)
    idx_jj2ii = _edge_view("idx_b", torch.long)
    valid_match_j = _edge_view("valid_f", torch.bool)
    valid_match_i = _edge_view("valid_b", torch.bool)
    Q_ii2jj = _edge_view("Q_f", torch.float32)
    Q_jj2ii = _edge_view("Q_b", torch.float32)
    del _edge_view

    def add_edges(self, ii, jj, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qj, Qi):
        """Append already-gated edges (both directions) to the store."""
        if self.edges is None:
            self.edges = EdgeStore(idx_i2j.shape[1], self.device)
        self.edges.append(ii, jj, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qj, Qi)

    def add_matched_factors(self, ii, jj, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii,
                            Qjj, Qji, Qij, min_match_frac, is_reloc=False):
        Qj, Qi, counts = mast3r_slam_backends.edge_confidence(
            idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij, self.cfg["Q_conf"])
        frac_j = counts[:, 0] / (valid_match_j.shape[1] * valid_match_j.shape[2])
        frac_i = counts[:, 1] / (valid_match_i.shape[1] * valid_match_i.shape[2])
        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        invalid = (torch.minimum(frac_j, frac_i) < min_match_frac) & ~(ii_t == (jj_t - 1))
        if is_reloc and invalid.any():
            return False
        keep = ~invalid
        self.add_edges(ii_t[keep], jj_t[keep], idx_i2j[keep], idx_j2i[keep], valid_match_j[keep],
                       valid_match_i[keep], Qj[keep], Qi[keep])
        return bool(keep.sum() > 0)

    def _views(self, unique_kf_idx, calib):
        """Xs, Twc (store view, updated in place by the op) and Cs of the graph's keyframes:
        views when they are a contiguous range of a KeyframeStore, else stacked copies."""
        fr = self.frames
        u = unique_kf_idx
        lo, hi = int(u[0]), int(u[-1]) + 1
        if isinstance(fr, KeyframeStore) and hi - lo == u.numel() and (not calib or fr.X_ray is not None):
            Xs = (fr.X_ray if calib else fr.X)[lo:hi]
            return Xs, fr.T_WC[lo:hi, 0], fr.C_avg[lo:hi], True
        Xs, T_WCs, Cs = self.get_poses_points(u)
        if calib:
            height, width = fr[0].img.shape[-2:]
            Xs = constrain_points_to_ray((height, width), Xs, self.K)
        return Xs, T_WCs.data[:, 0, :], Cs, False

    def _solve(self, mode):
        pin = self.cfg["pin"]
        unique_kf_idx = self.get_unique_kf_idx()
        if unique_kf_idx.numel() <= pin:
            return
        calib = mode == mast3r_slam_backends.GN_CALIB
        Xs, pose_data, Cs, in_place = self._views(unique_kf_idx, calib)
        ii = torch.cat((self.ii, self.jj))  # 16 B per directed edge
        jj = torch.cat((self.jj, self.ii))
        c = self.cfg
        kw = {}
        if calib:
            height, width = self.frames[0].img.shape[-2:]
            s0, s1 = c["sigma_pixel"], c["sigma_depth"]
            kw = dict(K=self.K, height=height, width=width, pixel_border=c["pixel_border"],
                      z_eps=c["depth_eps"])
        else:
            s0, s1 = c["sigma_ray"], c["sigma_dist"]
        idx_f, valid_f, Q_f = self.edges.forward()
        # the op pins only pose 0 (num_fix = 1, gn_kernels.cu:741); the reference writes back
        # T_WCs[pin:] only (global_opt.py:158/213): with pin > 1 the store's rows 1..pin-1 must
        # keep their values when the op updates the store in place
        keep = pose_data[1:pin].clone() if in_place and pin > 1 else None
        mast3r_slam_backends._run_gn(
            mode, pose_data, Xs, Cs, ii, jj, idx_f, valid_f, Q_f, c["max_iters"], c["delta_norm"],
            s0, s1, c["C_conf"], c["Q_conf"], second_half=self.edges.backward(), **kw)
        self._check_solved(mast3r_slam_backends, pose_data)
        if keep is not None:
            pose_data[1:pin] = keep
        if not in_place:
            self.frames.update_T_WCs(PoseBatch(pose_data[pin:, None]), unique_kf_idx[pin:])

    def solve_GN_rays(self, backend=None):
        self._solve(mast3r_slam_backends.GN_RAYS)

    def solve_GN_calib(self, backend=None):
        self._solve(mast3r_slam_backends.GN_CALIB)
