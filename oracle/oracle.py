"""ctypes binding of the CPU oracle (oracle/m3s_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product path (mast3r-slam_amd/).
All functions take and return numpy arrays (C-contiguous).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libm3s_oracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


if not os.path.exists(LIB_PATH):
    build()

_lib = ctypes.CDLL(LIB_PATH)
_vp, _i64, _i, _f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float

_lib.oracle_iter_proj.argtypes = [_vp] * 5 + [_i64] * 4 + [_i, _f, _f, _i]
_lib.oracle_set_contract.argtypes = [_i]
_lib.oracle_get_contract.restype = _i
_lib.oracle_refine_matches_f16.argtypes = [_vp] * 4 + [_i64] * 5 + [_i, _i]
_lib.oracle_refine_matches_f32.argtypes = [_vp] * 4 + [_i64] * 5 + [_i, _i]
_lib.oracle_refine_matches_f64.argtypes = [_vp] * 4 + [_i64] * 5 + [_i, _i]
_lib.oracle_f32_to_f16.restype = ctypes.c_uint16
_lib.oracle_f32_to_f16.argtypes = [_f]
_lib.oracle_f16_to_f32.restype = _f
_lib.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
_lib.oracle_num_threads.restype = _i
_lib.oracle_set_num_threads.argtypes = [_i]
_lib.oracle_set_exact_sums.argtypes = [_i]
_lib.oracle_match_prep.argtypes = [_vp] * 3 + [_i64] * 3 + [_vp] * 3
_lib.oracle_match_post.argtypes = [_vp] * 4 + [_i64] * 3 + [_f, _vp, _vp]


class GNParams(ctypes.Structure):
    _fields_ = [
        ("mode", _i),
        ("sigma0", _f),
        ("sigma1", _f),
        ("C_thresh", _f),
        ("Q_thresh", _f),
        ("K", _f * 9),
        ("height", _i),
        ("width", _i),
        ("pixel_border", _i),
        ("z_eps", _f),
        ("max_iter", _i),
        ("delta_thresh", _f),
    ]


_P = ctypes.POINTER(GNParams)
_lib.oracle_gn_align.argtypes = [_P] + [_vp] * 8 + [_i64] * 3 + [_vp, _vp]
_lib.oracle_gn_residuals.argtypes = [_P] + [_vp] * 8 + [_i64] * 3 + [_vp] * 4
_lib.oracle_gn_assemble.argtypes = [_vp] * 4 + [_i64, _i64, _vp, _vp]
_lib.oracle_gn_system.argtypes = [_P] + [_vp] * 8 + [_i64] * 3 + [_vp, _vp]
_lib.oracle_cholesky_solve.argtypes = [_vp, _vp, _vp, _i64]
_lib.oracle_cholesky_solve.restype = _i
_lib.oracle_pose_retr.argtypes = [_vp, _vp, _i64, _i]
_lib.oracle_gauss_newton.argtypes = [_P] + [_vp] * 8 + [_i64] * 3 + [_vp]
_lib.oracle_gauss_newton.restype = _i
_lib.oracle_remap.argtypes = [_vp, _vp, _i64, _vp, _vp]
_lib.oracle_remap.restype = _i64
_lib.oracle_exp_sim3.argtypes = [_vp] * 4
_lib.oracle_retr_sim3.argtypes = [_vp] * 7
_lib.oracle_apply_sim3_adj_inv.argtypes = [_vp] * 5

MODES = {"points": 0, "rays": 1, "calib": 2}
# FMA contraction conventions (m3s_oracle.h / mast3r-slam_amd/csrc/contract.h): the reference's nvcc
# build fuses multiply-adds (NVCC, left product of a two-product sum; the default), NVCC_RIGHT the
# right product, OFF multiply-then-add
CONTRACT = {"nvcc": 0, "off": 1, "nvcc_right": 2}
CONTRACT_DEFAULT = "nvcc"


def _cm(contract):
    return CONTRACT[contract] if isinstance(contract, str) else int(contract)


class contract:
    """Context: the GN restatement's contraction convention (alignment kernels, Sim3 library,
    retraction) -- ``with contract("off"): ...``."""

    def __init__(self, cm):
        self.cm = _cm(cm)

    def __enter__(self):
        self.prev = _lib.oracle_get_contract()
        _lib.oracle_set_contract(self.cm)

    def __exit__(self, *a):
        _lib.oracle_set_contract(self.prev)


def _c(a, dtype):
    a = np.ascontiguousarray(a, dtype=dtype)
    return a


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def num_threads():
    return _lib.oracle_num_threads()


def set_num_threads(n):
    _lib.oracle_set_num_threads(int(n))


class exact_sums:
    """Context: the GN oracle sums the reference's float terms in double (a precision
    reference, not the reference's arithmetic)."""

    def __enter__(self):
        _lib.oracle_set_exact_sums(1)

    def __exit__(self, *a):
        _lib.oracle_set_exact_sums(0)


def f32_to_f16_bits(x: float) -> int:
    return _lib.oracle_f32_to_f16(float(x))


def f16_bits_to_f32(h: int) -> float:
    return _lib.oracle_f16_to_f32(int(h))


def iter_proj(rays, pts, p_init, max_iter, lambda_init, cost_thresh, contract=CONTRACT_DEFAULT):
    rays = _c(rays, np.float32)
    pts = _c(pts, np.float32)
    p_init = _c(p_init, np.float32)
    B, H, W, C = rays.shape
    assert C == 9
    N = p_init.shape[1]
    p_new = np.zeros((B, N, 2), np.float32)
    conv = np.zeros((B, N), np.uint8)
    _lib.oracle_iter_proj(_p(rays), _p(pts), _p(p_init), _p(p_new), _p(conv), B, H, W, N,
                          int(max_iter), float(lambda_init), float(cost_thresh), _cm(contract))
    return p_new, conv.astype(bool)


def match_prep(X11, X21, idx_init=None):
    """prep_for_iter_proj (matching.py:25-49) with the reference's host arithmetic
    -> rays_with_grad [B,H,W,9], pts3d_norm [B,HW,3], p_init [B,HW,2]."""
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    B, H, W, _ = X11.shape
    rays = np.zeros((B, H, W, 9), np.float32)
    pts = np.zeros((B, H * W, 3), np.float32)
    p_init = np.zeros((B, H * W, 2), np.float32)
    ii = None if idx_init is None else _c(idx_init, np.int64)
    _lib.oracle_match_prep(_p(X11), _p(X21), _p(ii) if ii is not None else None, B, H, W, _p(rays), _p(pts),
                           _p(p_init))
    return rays, pts, p_init


def match_iterative_proj(X11, X21, D11, D21, idx_init, max_iter, lambda_init, cost_thresh, dist_thresh,
                         radius, dilation_max, contract=CONTRACT_DEFAULT, return_pre=False):
    """The reference's match_iterative_proj (matching.py:52-90): glue with the host arithmetic,
    the oracle's iter_proj / refine_matches -> idx [B,HW] i64, valid [B,HW,1] bool."""
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    B, H, W, _ = X11.shape
    rays, pts, p_init = match_prep(X11, X21, idx_init)
    p_new, conv = iter_proj(rays, pts, p_init, max_iter, lambda_init, cost_thresh, contract)
    p1 = np.zeros((B, H * W, 2), np.int64)
    valid = np.zeros((B, H * W), np.uint8)
    conv8 = np.ascontiguousarray(conv.astype(np.uint8))
    _lib.oracle_match_post(_p(X11), _p(X21), _p(p_new), _p(conv8), B, H, W, float(dist_thresh), _p(p1),
                           _p(valid))
    p1_pre = p1
    if radius > 0:
        d11 = np.asarray(D11, np.float32).astype(np.float16)
        d21 = np.asarray(D21, np.float32).reshape(B, H * W, -1).astype(np.float16)
        p1 = refine_matches(d11, d21, p1, radius, dilation_max)
    out = (p1[..., 0] + W * p1[..., 1], valid.astype(bool)[..., None])
    if return_pre:  # + iter_proj's p_new and the truncated pre-refine pixels p.long()
        return out + (p_new, p1_pre)
    return out


def refine_matches(D11, D21, p1, radius, dilation_max):
    p1 = _c(p1, np.int64)
    B, H, W, F = D11.shape
    N = p1.shape[1]
    out = np.zeros((B, N, 2), np.int64)
    if D11.dtype == np.float16:
        d11 = _c(D11, np.float16).view(np.uint16)
        d21 = _c(D21, np.float16).view(np.uint16)
        _lib.oracle_refine_matches_f16(_p(d11), _p(d21), _p(p1), _p(out), B, H, W, N, F,
                                       int(radius), int(dilation_max))
    elif D11.dtype == np.float64:
        d11 = _c(D11, np.float64)
        d21 = _c(D21, np.float64)
        _lib.oracle_refine_matches_f64(_p(d11), _p(d21), _p(p1), _p(out), B, H, W, N, F,
                                       int(radius), int(dilation_max))
    else:
        d11 = _c(D11, np.float32)
        d21 = _c(D21, np.float32)
        _lib.oracle_refine_matches_f32(_p(d11), _p(d21), _p(p1), _p(out), B, H, W, N, F,
                                       int(radius), int(dilation_max))
    return out


def make_params(mode, sigma0, sigma1=0.0, C_thresh=0.0, Q_thresh=1.5, K=None, height=0,
                width=0, pixel_border=0, z_eps=0.0, max_iter=10, delta_thresh=1e-8):
    P = GNParams()
    P.mode = MODES[mode] if isinstance(mode, str) else int(mode)
    P.sigma0, P.sigma1 = sigma0, sigma1
    P.C_thresh, P.Q_thresh = C_thresh, Q_thresh
    if K is not None:
        K = np.asarray(K, np.float32).reshape(9)
        for k in range(9):
            P.K[k] = float(K[k])
    P.height, P.width, P.pixel_border = int(height), int(width), int(pixel_border)
    P.z_eps = z_eps
    P.max_iter = int(max_iter)
    P.delta_thresh = float(delta_thresh)
    return P


def remap(ii, jj):
    ii = _c(ii, np.int64)
    jj = _c(jj, np.int64)
    ie = np.zeros_like(ii)
    je = np.zeros_like(jj)
    nu = _lib.oracle_remap(_p(ii), _p(jj), ii.shape[0], _p(ie), _p(je))
    return ie, je, nu


def gn_align(P, Twc, Xs, Cs, ii_edge, jj_edge, idx, valid, Q):
    Twc, Xs, Cs = _c(Twc, np.float32), _c(Xs, np.float32), _c(Cs, np.float32)
    ii_edge, jj_edge, idx = _c(ii_edge, np.int64), _c(jj_edge, np.int64), _c(idx, np.int64)
    valid = _c(valid, np.uint8)
    Q = _c(Q, np.float32)
    N, HW = Xs.shape[0], Xs.shape[1]
    E = ii_edge.shape[0]
    Hs = np.zeros((4, E, 7, 7), np.float32)
    gs = np.zeros((2, E, 7), np.float32)
    _lib.oracle_gn_align(ctypes.byref(P), _p(Twc), _p(Xs), _p(Cs), _p(ii_edge), _p(jj_edge),
                         _p(idx), _p(valid), _p(Q), N, HW, E, _p(Hs), _p(gs))
    return Hs, gs


def gn_residuals(P, Twc, Xs, Cs, ii_edge, jj_edge, idx, valid, Q):
    """Per directed point-edge: T_ij Xj [E,HW,3], residuals [E,HW,4], robust weights [E,HW,4]
    (3-row modes: the 4th is 0) and the validity flag [E,HW] of the align kernels."""
    Twc, Xs, Cs = _c(Twc, np.float32), _c(Xs, np.float32), _c(Cs, np.float32)
    ii_edge, jj_edge, idx = _c(ii_edge, np.int64), _c(jj_edge, np.int64), _c(idx, np.int64)
    valid = _c(valid, np.uint8)
    Q = _c(Q, np.float32)
    N, HW = Xs.shape[0], Xs.shape[1]
    E = ii_edge.shape[0]
    X = np.zeros((E, HW, 3), np.float32)
    err = np.zeros((E, HW, 4), np.float32)
    w = np.zeros((E, HW, 4), np.float32)
    vo = np.zeros((E, HW), np.uint8)
    _lib.oracle_gn_residuals(ctypes.byref(P), _p(Twc), _p(Xs), _p(Cs), _p(ii_edge), _p(jj_edge),
                             _p(idx), _p(valid), _p(Q), N, HW, E, _p(X), _p(err), _p(w), _p(vo))
    return X, err, w, vo.astype(bool)


def gn_assemble(Hs, gs, ii_opt, jj_opt, N):
    Hs, gs = _c(Hs, np.float32), _c(gs, np.float32)
    ii_opt, jj_opt = _c(ii_opt, np.int64), _c(jj_opt, np.int64)
    n = 7 * (N - 1)
    H = np.zeros((n, n), np.float64)
    b = np.zeros((n,), np.float64)
    _lib.oracle_gn_assemble(_p(Hs), _p(gs), _p(ii_opt), _p(jj_opt), N, ii_opt.shape[0], _p(H), _p(b))
    return H, b


def gn_build_system(P, Twc, Xs, Cs, ii, jj, idx, valid, Q):
    """Dense normal equations of ONE iteration at the current Twc (reference SparseBlock), as
    gauss_newton forms them (under ``exact_sums()``: the exactly summed system, unrounded)."""
    ie, je, _ = remap(ii, jj)
    Twc, Xs, Cs = _c(Twc, np.float32), _c(Xs, np.float32), _c(Cs, np.float32)
    idx, valid, Q = _c(idx, np.int64), _c(valid, np.uint8), _c(Q, np.float32)
    N, HW = Xs.shape[0], Xs.shape[1]
    n = 7 * (N - 1)
    H = np.zeros((n, n), np.float64)
    b = np.zeros((n,), np.float64)
    _lib.oracle_gn_system(ctypes.byref(P), _p(Twc), _p(Xs), _p(Cs), _p(ie), _p(je), _p(idx), _p(valid),
                          _p(Q), N, HW, ie.shape[0], _p(H), _p(b))
    return H, b


def cholesky_solve(H, b):
    H = _c(H, np.float64).copy()
    b = _c(b, np.float64)
    x = np.zeros_like(b)
    rc = _lib.oracle_cholesky_solve(_p(H), _p(b), _p(x), b.shape[0])
    return x, rc


def gauss_newton(P, Twc, Xs, Cs, ii, jj, idx, valid, Q):
    """Returns (Twc_out, dx, iterations)."""
    Twc = _c(Twc, np.float32).copy()
    Xs, Cs = _c(Xs, np.float32), _c(Cs, np.float32)
    ii, jj, idx = _c(ii, np.int64), _c(jj, np.int64), _c(idx, np.int64)
    valid = _c(valid, np.uint8)
    Q = _c(Q, np.float32)
    N, HW = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    dx = np.zeros((max(N - 1, 0), 7), np.float32)
    it = _lib.oracle_gauss_newton(ctypes.byref(P), _p(Twc), _p(Xs), _p(Cs), _p(ii), _p(jj),
                                  _p(idx), _p(valid), _p(Q), N, HW, E, _p(dx))
    return Twc, dx, it


def exp_sim3(xi):
    xi = _c(xi, np.float32)
    t = np.zeros(3, np.float32)
    q = np.zeros(4, np.float32)
    s = np.zeros(1, np.float32)
    _lib.oracle_exp_sim3(_p(xi), _p(t), _p(q), _p(s))
    return t, q, s[0]


def retr_sim3(xi, pose):
    xi = _c(xi, np.float32)
    pose = _c(pose, np.float32)
    t, q, s = pose[:3].copy(), pose[3:7].copy(), pose[7:8].copy()
    t1 = np.zeros(3, np.float32)
    q1 = np.zeros(4, np.float32)
    s1 = np.zeros(1, np.float32)
    _lib.oracle_retr_sim3(_p(xi), _p(t), _p(q), _p(s), _p(t1), _p(q1), _p(s1))
    return np.concatenate([t1, q1, s1])


def apply_sim3_adj_inv(pose, X):
    pose = _c(pose, np.float32)
    X = _c(X, np.float32)
    t, q, s = pose[:3].copy(), pose[3:7].copy(), pose[7:8].copy()
    Y = np.zeros(7, np.float32)
    _lib.oracle_apply_sim3_adj_inv(_p(t), _p(q), _p(s), _p(X), _p(Y))
    return Y
