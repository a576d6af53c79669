"""mast3r_slam_backends -- MI355X-native drop-in for the reference's pybind11 module.

Same module name, same five ops, same positional signatures and return lists as the
reference (``/root/reference/mast3r_slam/backend/src/gn.cpp:116-123``; prototypes in
``gn.h:22-117``), so ``mast3r_slam/matching.py:60,79`` and ``global_opt.py:140,190``
call it unchanged.  Every op runs the hand-written gfx950 HIP kernels of
``libm3s_backend.so`` (C ABI: ``include/m3s_backend.h``) on torch's current HIP stream.

There is no CPU fallback: CPU tensors raise ``RuntimeError`` (the reference dispatches
unconditionally to ``*_cuda`` as well), and a missing library raises ``ImportError`` at
import time.
"""
from __future__ import annotations

import atexit
import ctypes
import os

import torch

__all__ = [
    "gn_debug_flags",
    "iter_proj",
    "refine_matches",
    "gauss_newton_points",
    "gauss_newton_rays",
    "gauss_newton_calib",
    "track_sim3",
    "CholeskyError",
    "pointmap_update",
    "edge_confidence",
    "gn_plan_info",
    "library_path",
    "set_gn_order",
    "set_gn_contract",
    "lib",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
library_path = os.environ.get(
    "M3S_BACKEND_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libm3s_backend.so")
)

if not os.path.exists(library_path):
    raise ImportError(
        f"mast3r_slam_backends: HIP backend library not found at {library_path}; "
        "build it with `make -C mast3r-slam_amd` (or __graft_entry__.build())"
    )

lib = ctypes.CDLL(library_path)

_c_int64 = ctypes.c_int64
_vp = ctypes.c_void_p
_f = ctypes.c_float
_i = ctypes.c_int

lib.m3s_last_error.restype = ctypes.c_char_p
lib.m3s_shutdown.restype = None
# pinned staging buffers / events are released here, while the HIP runtime is alive (not by
# exit-time destructors inside the library)
atexit.register(lib.m3s_shutdown)
lib.m3s_version.restype = ctypes.c_char_p
lib.m3s_iter_proj.argtypes = [_vp] * 5 + [_c_int64] * 4 + [_i, _f, _f, _vp]
lib.m3s_iter_proj_ex.argtypes = [_vp] * 5 + [_c_int64] * 4 + [_i, _f, _f, _i, _vp]
lib.m3s_refine_matches_f16.argtypes = [_vp] * 4 + [_c_int64] * 5 + [_i, _i, _vp]
lib.m3s_refine_matches_f32.argtypes = [_vp] * 4 + [_c_int64] * 5 + [_i, _i, _vp]
lib.m3s_refine_matches_f64.argtypes = [_vp] * 4 + [_c_int64] * 5 + [_i, _i, _vp]
lib.m3s_match_workspace_bytes.argtypes = [_c_int64] * 4
lib.m3s_match_workspace_bytes.restype = ctypes.c_size_t
lib.m3s_match_iterative_proj.argtypes = ([_vp] * 5 + [_c_int64] * 4 + [_i, _f, _f, _f, _i, _i, _i]
                                         + [_vp, _vp, _vp, ctypes.c_size_t, _vp])

# FMA-contraction convention of the parity paths (include/m3s_backend.h M3S_CONTRACT_*): the
# reference's nvcc build fuses multiply-adds ("nvcc": the left product of a two-product sum, the
# default); "nvcc_right" and "off" are variants for measuring the convention
CONTRACT = {"nvcc": 0, "off": 1, "nvcc_right": 2}


def _contract(c):
    if c is None:
        return CONTRACT["nvcc"]
    if c not in CONTRACT:
        raise ValueError(f"unknown contraction convention {c!r} (expected one of {sorted(CONTRACT)})")
    return CONTRACT[c]
lib.m3s_gn_workspace_bytes.restype = ctypes.c_size_t
lib.m3s_gn_workspace_bytes.argtypes = [_i, _c_int64, _c_int64, _c_int64, _c_int64]
lib.m3s_gn_plan_info.argtypes = [_vp, _vp, _c_int64, _c_int64, _vp, _vp, _vp, ctypes.c_int32]


class GNArgs(ctypes.Structure):
    """Mirror of ``m3s_gn_args`` (include/m3s_backend.h)."""

    _fields_ = [
        ("mode", _i),
        ("Twc", _vp),
        ("Xs", _vp),
        ("Cs", _vp),
        ("ii", _vp),
        ("jj", _vp),
        ("idx", _vp),
        ("valid", _vp),
        ("Q", _vp),
        ("N", _c_int64),
        ("HW", _c_int64),
        ("E_total", _c_int64),
        ("E_local", _c_int64),
        ("edge_offset", _c_int64),
        ("sigma0", _f),
        ("sigma1", _f),
        ("C_thresh", _f),
        ("Q_thresh", _f),
        ("K", _vp),
        ("height", _i),
        ("width", _i),
        ("pixel_border", _i),
        ("z_eps", _f),
        ("max_iter", _i),
        ("delta_thresh", _f),
        ("dx", _vp),
        ("ws", _vp),
        ("ws_bytes", ctypes.c_size_t),
        ("comm", _vp),
        ("stream", _vp),
        ("order", _i),
        ("idx_b", _vp),
        ("valid_b", _vp),
        ("Q_b", _vp),
        ("E_a", _c_int64),
        ("contract", _i),
    ]


lib.m3s_gauss_newton.argtypes = [ctypes.POINTER(GNArgs)]
lib.m3s_gn_check.argtypes = [_vp]
lib.m3s_gn_build_system.argtypes = [ctypes.POINTER(GNArgs), _vp, _vp]
lib.m3s_gn_edge_hessians.argtypes = [ctypes.POINTER(GNArgs), _vp, _vp]
lib.m3s_comm_get_unique_id.argtypes = [_vp]
lib.m3s_comm_init.argtypes = [_vp, _i, _i, ctypes.POINTER(_vp)]
lib.m3s_comm_destroy.argtypes = [_vp]
lib.m3s_comm_size.argtypes = [_vp, ctypes.POINTER(_i)]
# int (*)(void* user, double* buf, size_t count)
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(_i, _vp, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t)
lib.m3s_comm_init_host.argtypes = [HOST_ALLREDUCE_FN, _vp, _i, _i, ctypes.POINTER(_vp)]

GN_POINTS, GN_RAYS, GN_CALIB = 0, 1, 2

# Summation order of the GN normal equations (include/m3s_backend.h M3S_GN_ORDER_*):
# "default" lets the library decide (env M3S_GN_ORDER, else the fast packed path); "reference"
# reproduces the reference kernels' own float order and formulas (gn_refacc.hip).
GN_ORDERS = {"default": 0, "fast": 1, "reference": 2}
_gn_order = [0]


_gn_contract = [0]


def set_gn_contract(contract: str) -> str:
    """Select the FMA-contraction convention (``CONTRACT``) of the reference-order GN accumulate
    and the retraction for later gauss_newton_* calls; returns the previous."""
    prev = [k for k, v in CONTRACT.items() if v == _gn_contract[0]][0]
    _gn_contract[0] = _contract(contract)
    return prev


def set_gn_order(order: str) -> str:
    """Select the GN summation order for later gauss_newton_* calls; returns the previous."""
    if order not in GN_ORDERS:
        raise ValueError(f"unknown GN order {order!r} (expected one of {sorted(GN_ORDERS)})")
    prev = [k for k, v in GN_ORDERS.items() if v == _gn_order[0]][0]
    _gn_order[0] = GN_ORDERS[order]
    return prev

# ---------------------------------------------------------------------------------
# argument checks (the reference's TORCH_CHECK / packed_accessor32 behaviour)
# ---------------------------------------------------------------------------------

_DT_NAME = {
    torch.float32: "Float",
    torch.float16: "Half",
    torch.float64: "Double",
    torch.int64: "Long",
    torch.int32: "Int",
    torch.bool: "Bool",
    torch.uint8: "Byte",
}


def _check(t, name, dtype, ndim):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_contiguous():  # CHECK_CONTIGUOUS (gn.h:5)
        raise RuntimeError(f"{name} must be contiguous")
    dts = dtype if isinstance(dtype, tuple) else (dtype,)
    if t.dtype not in dts:
        raise RuntimeError(
            f"expected scalar type {_DT_NAME.get(dts[0], dts[0])} but found "
            f"{_DT_NAME.get(t.dtype, t.dtype)} ({name})"
        )
    if t.dim() != ndim:
        raise RuntimeError(f"packed_accessor32 expects {ndim} dims but tensor has {t.dim()} ({name})")


def _on_device(**tensors):
    """All tensors on one HIP device (checked after dtype/shape, like the accessors)."""
    dev = None
    for name, t in tensors.items():
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                f"{name} must be a HIP (cuda) tensor: mast3r_slam_backends has no CPU path"
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"{name} must be on {dev}, got {t.device}")
    return dev


def _raise(rc, what):
    if rc != 0:
        msg = lib.m3s_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg} (code {rc})")


def gn_plan_info(ii, jj, N):
    """The elimination plan gauss_newton_* builds for a pose graph (host only, no GPU;
    include/m3s_backend.h m3s_gn_plan_info).  ii, jj: the op's global keyframe ids (any int
    sequence / CPU tensor), N poses.  Returns a dict: solver ("fused" | "hybrid" | "multi" |
    None), rounds, eliminated, core_poses, core_unknowns_padded, pairs, plan_ints, core_fits,
    order (the poses round by round, then the core's) and round_ptr (each round's start in
    order, then the core's)."""
    import numpy as np

    ii = np.ascontiguousarray(np.asarray(ii, dtype=np.int64))
    jj = np.ascontiguousarray(np.asarray(jj, dtype=np.int64))
    if ii.shape != jj.shape or ii.ndim != 1:
        raise ValueError("ii and jj must be 1-D of equal length")
    info = np.zeros(8, dtype=np.int32)
    npose = max(int(N) - 1, 0)
    order = np.zeros(max(npose, 1), dtype=np.int32)
    cap = npose + 2
    rptr = np.zeros(cap, dtype=np.int32)
    rc = lib.m3s_gn_plan_info(ii.ctypes.data, jj.ctypes.data, ii.shape[0], int(N), info.ctypes.data,
                              order.ctypes.data, rptr.ctypes.data, cap)
    _raise(rc, "gn_plan_info")
    rounds = int(info[1])
    return {"solver": {0: "fused", 1: "hybrid", 2: "multi"}.get(int(info[0])), "rounds": rounds,
            "eliminated": int(info[2]), "core_poses": int(info[3]), "core_unknowns_padded": int(info[4]),
            "pairs": int(info[5]), "plan_ints": int(info[6]), "core_fits": bool(info[7]),
            "order": order[:npose].tolist(), "round_ptr": rptr[:rounds + 1].tolist()}


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# ---------------------------------------------------------------------------------
# matching ops
# ---------------------------------------------------------------------------------


def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh,
              contract=None):
    """gn.cpp:84-99 / matching_kernels.cu:279-316 -> [p_new f32[B,N,2], converged bool[B,N]].

    ``contract``: FMA-contraction convention (``CONTRACT``; default the reference build's)."""
    _check(rays_img_with_grad, "rays_img_with_grad", torch.float32, 4)
    _check(pts_3d_norm, "pts_3d_norm", torch.float32, 3)
    _check(p_init, "p_init", torch.float32, 3)
    dev = _on_device(rays_img_with_grad=rays_img_with_grad, pts_3d_norm=pts_3d_norm, p_init=p_init)
    B, H, W, C = rays_img_with_grad.shape
    if C != 9:
        raise RuntimeError(f"rays_img_with_grad must have 9 channels (ray, d/du, d/dv), got {C}")
    Bp, N = p_init.shape[0], p_init.shape[1]
    if p_init.shape[2] != 2 or pts_3d_norm.shape[2] != 3:
        raise RuntimeError("p_init must be [B,N,2] and pts_3d_norm [B,N,3]")
    if pts_3d_norm.shape[:2] != p_init.shape[:2] or Bp != B:
        raise RuntimeError("batch / point counts of rays_img_with_grad, pts_3d_norm, p_init differ")
    p_new = torch.zeros((Bp, N, 2), dtype=p_init.dtype, device=dev)
    converged = torch.zeros((Bp, N), dtype=torch.bool, device=dev)
    with torch.cuda.device(dev):
        rc = lib.m3s_iter_proj_ex(
            _ptr(rays_img_with_grad), _ptr(pts_3d_norm), _ptr(p_init), _ptr(p_new),
            _ptr(converged), B, H, W, N, int(max_iter), float(lambda_init),
            float(cost_thresh), _contract(contract), _stream(dev),
        )
    _raise(rc, "iter_proj")
    return [p_new, converged]


def refine_matches(D11, D21, p1, window_size, dilation_max):
    """gn.cpp:101-114 / matching_kernels.cu:84-116 -> [p1_new i64[B,N,2]].

    ``window_size`` is the search radius (config ``matching.radius``)."""
    # AT_DISPATCH_FLOATING_TYPES_AND_HALF (matching_kernels.cu:103): half, float, double
    _check(D11, "D11", (torch.float16, torch.float32, torch.float64), 4)
    _check(D21, "D21", D11.dtype, 3)
    _check(p1, "p1", torch.int64, 3)
    dev = _on_device(D11=D11, D21=D21, p1=p1)
    B, H, W, F = D11.shape
    Bq, N = p1.shape[0], p1.shape[1]
    if p1.shape[2] != 2 or D21.shape[0] != Bq or D21.shape[1] != N or D21.shape[2] != F or Bq != B:
        raise RuntimeError("refine_matches: expected D11 [B,H,W,F], D21 [B,N,F], p1 [B,N,2]")
    p1_new = torch.zeros((Bq, N, 2), dtype=p1.dtype, device=dev)
    fn = {torch.float16: lib.m3s_refine_matches_f16, torch.float32: lib.m3s_refine_matches_f32,
          torch.float64: lib.m3s_refine_matches_f64}[D11.dtype]
    with torch.cuda.device(dev):
        rc = fn(
            _ptr(D11), _ptr(D21), _ptr(p1), _ptr(p1_new), B, H, W, N, F,
            int(window_size), int(dilation_max), _stream(dev),
        )
    _raise(rc, "refine_matches")
    return [p1_new]


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init, max_iter, lambda_init, cost_thresh,
                         dist_thresh, radius, dilation_max, contract=None):
    """The whole Python matching caller (matching.py:52-90) as one op: prep_for_iter_proj,
    iter_proj, ``p.long()``, the occlusion test on the pre-refine pixels, refine_matches on the
    ``.half()`` descriptors and ``pixel_to_lin`` -> [idx i64[B,H*W], valid bool[B,H*W,1]].
    Extension op (not in the reference's module); the glue's float ops follow the reference's
    host arithmetic (csrc/match_glue.hip)."""
    _check(X11, "X11", torch.float32, 4)
    _check(X21, "X21", torch.float32, 4)
    _check(D11, "D11", torch.float32, 4)
    _check(D21, "D21", torch.float32, 4)
    if idx_1_to_2_init is not None:
        _check(idx_1_to_2_init, "idx_1_to_2_init", torch.int64, 2)
    dev = _on_device(X11=X11, X21=X21, D11=D11, D21=D21, idx_1_to_2_init=idx_1_to_2_init)
    B, H, W, _ = X11.shape
    F = D11.shape[3]
    if X11.shape[3] != 3 or X21.shape != X11.shape or D21.shape != D11.shape or D11.shape[:3] != (B, H, W):
        raise RuntimeError("match_iterative_proj: expected X11, X21 [B,H,W,3] and D11, D21 [B,H,W,F]")
    if idx_1_to_2_init is not None and tuple(idx_1_to_2_init.shape) != (B, H * W):
        raise RuntimeError("match_iterative_proj: idx_1_to_2_init must be [B,H*W]")
    idx = torch.empty((B, H * W), dtype=torch.int64, device=dev)
    valid = torch.empty((B, H * W, 1), dtype=torch.bool, device=dev)
    nbytes = int(lib.m3s_match_workspace_bytes(B, H, W, F))
    ws = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        rc = lib.m3s_match_iterative_proj(
            _ptr(X11), _ptr(X21), _ptr(D11), _ptr(D21), _ptr(idx_1_to_2_init), B, H, W, F,
            int(max_iter), float(lambda_init), float(cost_thresh), float(dist_thresh), int(radius),
            int(dilation_max), _contract(contract), _ptr(idx), _ptr(valid), _ptr(ws), nbytes,
            _stream(dev),
        )
    _raise(rc, "match_iterative_proj")
    return [idx, valid]


# ---------------------------------------------------------------------------------
# Gauss-Newton ops
# ---------------------------------------------------------------------------------


def _gn_common_checks(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, edge_local=None):
    _check(Twc, "Twc", torch.float32, 2)
    _check(Xs, "Xs", torch.float32, 3)
    _check(Cs, "Cs", torch.float32, 3)
    _check(ii, "ii", torch.int64, 1)
    _check(jj, "jj", torch.int64, 1)
    _check(idx_ii2jj, "idx_ii2jj", torch.int64, 2)
    _check(valid_match, "valid_match", torch.bool, 3)
    _check(Q, "Q", torch.float32, 3)
    dev = _on_device(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx_ii2jj=idx_ii2jj,
                     valid_match=valid_match, Q=Q)
    N, HW = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    El = E if edge_local is None else edge_local
    if Twc.shape != (N, 8) or Xs.shape[2] != 3 or Cs.shape != (N, HW, 1):
        raise RuntimeError("gauss_newton: expected Twc [N,8], Xs [N,HW,3], Cs [N,HW,1]")
    if jj.shape[0] != E:
        raise RuntimeError("gauss_newton: ii and jj differ in length")
    if idx_ii2jj.shape != (El, HW) or valid_match.shape != (El, HW, 1) or Q.shape != (El, HW, 1):
        raise RuntimeError(
            "gauss_newton: expected idx_ii2jj [E,HW], valid_match [E,HW,1], Q [E,HW,1]"
        )
    return dev, N, HW, E


def _run_gn(mode, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, max_iter, delta_thresh,
            sigma0, sigma1, C_thresh, Q_thresh, K=None, height=0, width=0, pixel_border=0,
            z_eps=0.0, comm=None, edge_offset=0, edge_total=None, second_half=None):
    """``second_half`` = (idx, valid, Q) of local directed edges E_a.. when the edges come as
    two tensors (a two-way edge store: forward then backward), E_a = len(idx_ii2jj)."""
    E_a = idx_ii2jj.shape[0]
    E_local = E_a
    if second_half is not None:
        idx_b, valid_b, Q_b = second_half
        _check(idx_b, "idx_ii2jj (second half)", torch.int64, 2)
        _check(valid_b, "valid_match (second half)", torch.bool, 3)
        _check(Q_b, "Q (second half)", torch.float32, 3)
        _on_device(idx_a=idx_ii2jj, idx_b=idx_b, valid_b=valid_b, Q_b=Q_b)
        E_b = idx_b.shape[0]
        if idx_b.shape[1:] != idx_ii2jj.shape[1:] or valid_b.shape != (E_b,) + valid_match.shape[1:] \
                or Q_b.shape != (E_b,) + Q.shape[1:]:
            raise RuntimeError("gauss_newton: second edge half shapes differ from the first")
        E_local = E_a + E_b
    dev, N, HW, E = _gn_common_checks(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, E_a)
    if E_local != E_a and edge_total is None and E_local != E:
        raise RuntimeError("gauss_newton: the two edge halves must cover len(ii) directed edges")
    if edge_total is not None and edge_total != E:
        raise RuntimeError("gauss_newton: edge_total must equal len(ii)")
    if K is not None:
        _check(K, "K", torch.float32, 2)
        _on_device(Twc=Twc, K=K)
        if K.shape != (3, 3):
            raise RuntimeError("K must be [3,3]")
    max_iter = int(max_iter)
    dx = torch.zeros((max(N - 1, 0), 7), dtype=torch.float32, device=dev)
    ws_bytes = lib.m3s_gn_workspace_bytes(mode, N, HW, E, E_local)
    ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=dev)
    a = GNArgs()
    a.mode = mode
    a.Twc, a.Xs, a.Cs = Twc.data_ptr(), Xs.data_ptr(), Cs.data_ptr()
    a.ii, a.jj = ii.data_ptr(), jj.data_ptr()
    a.idx, a.valid, a.Q = idx_ii2jj.data_ptr(), valid_match.data_ptr(), Q.data_ptr()
    a.N, a.HW, a.E_total, a.E_local, a.edge_offset = N, HW, E, E_local, int(edge_offset)
    a.sigma0, a.sigma1 = float(sigma0), float(sigma1)
    a.C_thresh, a.Q_thresh = float(C_thresh), float(Q_thresh)
    a.K = K.data_ptr() if K is not None else None
    a.height, a.width, a.pixel_border = int(height), int(width), int(pixel_border)
    a.z_eps = float(z_eps)
    a.max_iter = max_iter
    a.delta_thresh = float(delta_thresh)
    a.dx = dx.data_ptr()
    a.ws, a.ws_bytes = ws.data_ptr(), ws_bytes
    a.comm = comm
    a.order = _gn_order[0]
    a.contract = _gn_contract[0]
    if second_half is not None:
        a.idx_b, a.valid_b, a.Q_b = idx_b.data_ptr(), valid_b.data_ptr(), Q_b.data_ptr()
        a.E_a = E_a
    with torch.cuda.device(dev):
        a.stream = torch.cuda.current_stream(dev).cuda_stream
        rc = lib.m3s_gauss_newton(ctypes.byref(a))
    _raise(rc, "gauss_newton")
    # the reference returns an undefined tensor when no iteration ran
    return [dx if max_iter > 0 else None]


def gauss_newton_points(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_point, C_thresh,
                        Q_thresh, max_iter, delta_thresh):
    """gn.cpp:3-26 -> [dx].  Twc is updated in place."""
    return _run_gn(GN_POINTS, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, max_iter,
                   delta_thresh, sigma_point, 0.0, C_thresh, Q_thresh)


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist,
                      C_thresh, Q_thresh, max_iter, delta_thresh):
    """gn.cpp:28-52 -> [dx].  Twc is updated in place."""
    return _run_gn(GN_RAYS, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, max_iter,
                   delta_thresh, sigma_ray, sigma_dist, C_thresh, Q_thresh)


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width,
                       pixel_border, z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh,
                       max_iter, delta_thresh):
    """gn.cpp:54-82 -> [dx].  Twc is updated in place."""
    return _run_gn(GN_CALIB, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, max_iter,
                   delta_thresh, sigma_pixel, sigma_depth, C_thresh, Q_thresh, K=K,
                   height=height, width=width, pixel_border=pixel_border, z_eps=z_eps)


# ---------------------------------------------------------------------------------
# frame tracking (extension: the reference runs this loop in torch, tracker.py:173-266)
# ---------------------------------------------------------------------------------


class TrackArgs(ctypes.Structure):
    """Mirror of ``m3s_track_args`` (include/m3s_backend.h)."""

    _fields_ = [
        ("mode", _i),
        ("Xf", _vp),
        ("Xk", _vp),
        ("Qk", _vp),
        ("valid", _vp),
        ("meas_k", _vp),
        ("valid_meas", _vp),
        ("K", _vp),
        ("T_WCf", _vp),
        ("T_WCk", _vp),
        ("HW", _c_int64),
        ("height", _i),
        ("width", _i),
        ("pixel_border", _i),
        ("z_eps", ctypes.c_double),
        ("sigma0", ctypes.c_double),
        ("sigma1", ctypes.c_double),
        ("huber_k", ctypes.c_double),
        ("max_iters", _i),
        ("rel_error", ctypes.c_double),
        ("delta_norm", ctypes.c_double),
        ("check_every", _i),
        ("T_WCf_out", _vp),
        ("T_CkCf_out", _vp),
        ("info", _vp),
        ("cost", _vp),
        ("ws", _vp),
        ("ws_bytes", ctypes.c_size_t),
        ("stream", _vp),
    ]


lib.m3s_track_sim3.argtypes = [ctypes.POINTER(TrackArgs)]
lib.m3s_track_workspace_bytes.restype = ctypes.c_size_t
lib.m3s_track_workspace_bytes.argtypes = [_c_int64]
lib.m3s_track_last_result.argtypes = [_vp, _vp]


class CholeskyError(RuntimeError):
    """The 7x7 normal equations were not positive definite (torch.linalg.cholesky raises
    torch.linalg.LinAlgError, a RuntimeError, in the reference; tracker.py:91 catches it)."""


def track_sim3(mode, Xf, Xk, T_WCf, T_WCk, Qk, valid, sigma0, sigma1, huber_k, max_iters,
               rel_error, delta_norm, meas_k=None, valid_meas_k=None, K=None, img_size=None,
               pixel_border=0, z_eps=0.0, check_every=4):
    """Sim3 GN of one frame against its keyframe (tracker.py:173-266) on the GPU.

    mode "rays" (opt_pose_ray_dist_sim3) or "calib" (opt_pose_calib_sim3); Xf [HW,3] the
    gathered frame points, Xk [HW,3], Qk [HW,1], valid [HW,1] bool, T_WCf / T_WCk lietorch
    Sim3 data [1,8] (or [8]).  Returns (T_WCf [1,8], T_CkCf [1,8], iterations, cost).
    Raises CholeskyError when the normal equations are not positive definite."""
    m = GN_RAYS if mode == "rays" else GN_CALIB
    _check(Xf, "Xf", torch.float32, 2)
    _check(Qk, "Qk", torch.float32, 2)
    _check(valid, "valid", torch.bool, 2)
    T_WCf = T_WCf.reshape(-1)
    T_WCk = T_WCk.reshape(-1)
    _check(T_WCf, "T_WCf", torch.float32, 1)
    _check(T_WCk, "T_WCk", torch.float32, 1)
    HW = Xf.shape[0]
    if Xf.shape[1] != 3 or Qk.shape != (HW, 1) or valid.shape != (HW, 1) or T_WCf.numel() != 8 \
            or T_WCk.numel() != 8:
        raise RuntimeError("track_sim3: expected Xf [HW,3], Qk [HW,1], valid [HW,1], poses [8]")
    tens = dict(Xf=Xf, Qk=Qk, valid=valid, T_WCf=T_WCf, T_WCk=T_WCk)
    if m == GN_RAYS:
        _check(Xk, "Xk", torch.float32, 2)
        if Xk.shape != (HW, 3):
            raise RuntimeError("track_sim3: Xk must be [HW,3]")
        tens["Xk"] = Xk
    else:
        _check(meas_k, "meas_k", torch.float32, 2)
        _check(valid_meas_k, "valid_meas_k", torch.bool, 2)
        _check(K, "K", torch.float32, 2)
        if meas_k.shape != (HW, 3) or valid_meas_k.shape != (HW, 1) or K.shape != (3, 3):
            raise RuntimeError("track_sim3: expected meas_k [HW,3], valid_meas_k [HW,1], K [3,3]")
        tens.update(meas_k=meas_k, valid_meas_k=valid_meas_k, K=K)
    dev = _on_device(**tens)
    out_f = torch.empty((1, 8), dtype=torch.float32, device=dev)
    out_r = torch.empty((1, 8), dtype=torch.float32, device=dev)
    # the device-side info (4 int32) and cost (1 f64), one buffer (the result is read on the host
    # through m3s_track_last_result below)
    res = torch.empty((3,), dtype=torch.float64, device=dev)
    info, cost = res[:2].view(torch.int32), res[2:]
    ws_bytes = lib.m3s_track_workspace_bytes(HW)
    ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=dev)
    a = TrackArgs()
    a.mode = m
    a.Xf, a.Qk, a.valid = Xf.data_ptr(), Qk.data_ptr(), valid.data_ptr()
    a.Xk = Xk.data_ptr() if m == GN_RAYS else None
    if m == GN_CALIB:
        a.meas_k, a.valid_meas, a.K = meas_k.data_ptr(), valid_meas_k.data_ptr(), K.data_ptr()
        a.height, a.width = int(img_size[0]), int(img_size[1])
    a.T_WCf, a.T_WCk = T_WCf.data_ptr(), T_WCk.data_ptr()
    a.HW = HW
    a.pixel_border = int(pixel_border)
    a.z_eps = float(z_eps)
    a.sigma0, a.sigma1 = float(sigma0), float(sigma1)
    a.huber_k = float(huber_k)
    a.max_iters = int(max_iters)
    a.rel_error, a.delta_norm = float(rel_error), float(delta_norm)
    a.check_every = int(check_every)
    a.T_WCf_out, a.T_CkCf_out = out_f.data_ptr(), out_r.data_ptr()
    a.info, a.cost = info.data_ptr(), cost.data_ptr()
    a.ws, a.ws_bytes = ws.data_ptr(), ws_bytes
    with torch.cuda.device(dev):
        a.stream = torch.cuda.current_stream(dev).cuda_stream
        rc = lib.m3s_track_sim3(ctypes.byref(a))
    _raise(rc, "track_sim3")
    # the result from the call's pinned state copy (no second device round trip when the call
    # already saw its done flag); `info` / `cost` on the device hold the same values
    hinfo = (ctypes.c_int32 * 4)()
    hcost = ctypes.c_double()
    _raise(lib.m3s_track_last_result(ctypes.cast(hinfo, _vp), ctypes.cast(ctypes.pointer(hcost), _vp)),
           "track_last_result")
    it, failed = int(hinfo[0]), int(hinfo[2])
    if failed:
        raise CholeskyError("track_sim3: normal equations not positive definite "
                            f"(iteration {it + 1})")
    return out_f, out_r, it, float(hcost.value)


# ---------------------------------------------------------------------------------
# edge construction after matching (extension: global_opt.py:53-67 runs in torch)
# ---------------------------------------------------------------------------------

lib.m3s_edge_confidence.argtypes = [_vp] * 8 + [_f, _c_int64, _c_int64, _vp, _vp, _vp, _vp]


def edge_confidence(idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij, Q_conf):
    """global_opt.py:53-67 fused: returns (Qj [B,HW,1], Qi [B,HW,1], counts [B,2] int32) with
    counts = (#valid_j, #valid_i) per pair (the match-fraction numerators)."""
    _check(idx_i2j, "idx_i2j", torch.int64, 2)
    _check(idx_j2i, "idx_j2i", torch.int64, 2)
    B, HW = idx_i2j.shape
    for name, t in (("valid_match_j", valid_match_j), ("valid_match_i", valid_match_i)):
        _check(t, name, torch.bool, 3)
    for name, t in (("Qii", Qii), ("Qjj", Qjj), ("Qji", Qji), ("Qij", Qij)):
        _check(t, name, torch.float32, 3)
    for t in (valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij):
        if t.shape != (B, HW, 1):
            raise RuntimeError("edge_confidence: expected [B,HW,1] masks / confidences")
    if idx_j2i.shape != (B, HW):
        raise RuntimeError("edge_confidence: idx_i2j and idx_j2i differ in shape")
    dev = _on_device(idx_i2j=idx_i2j, idx_j2i=idx_j2i, valid_match_j=valid_match_j,
                     valid_match_i=valid_match_i, Qii=Qii, Qjj=Qjj, Qji=Qji, Qij=Qij)
    Qj = torch.empty((B, HW, 1), dtype=torch.float32, device=dev)
    Qi = torch.empty((B, HW, 1), dtype=torch.float32, device=dev)
    counts = torch.empty((B, 2), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        rc = lib.m3s_edge_confidence(_ptr(idx_i2j), _ptr(idx_j2i), _ptr(valid_match_j),
                                     _ptr(valid_match_i), _ptr(Qii), _ptr(Qjj), _ptr(Qji), _ptr(Qij),
                                     float(Q_conf), B, HW, _ptr(Qj), _ptr(Qi), _ptr(counts),
                                     _stream(dev))
    _raise(rc, "edge_confidence")
    return Qj, Qi, counts


# ---------------------------------------------------------------------------------
# keyframe point-map fusion (extension: frame.py:41-105 runs in torch in the reference)
# ---------------------------------------------------------------------------------

lib.m3s_pointmap_update.argtypes = [_i, _vp, _vp, _vp, _vp, _vp, _c_int64, _vp]
FILTER_MODES = {"weighted_pointmap": 0, "indep_conf": 1, "recent": 2}


def pointmap_update(mode, X, C, X_new, C_new, T=None):
    """In-place X [HW,3], C [HW,1] <- fuse(X, C, T.act(X_new), C_new) for filtering ``mode``
    (frame.py:58-77; T: optional Sim3 data [1,8] / [8], tracker.py:98-99)."""
    if mode not in FILTER_MODES:
        raise RuntimeError(f"pointmap_update: mode {mode!r} is not a per-point filtering mode")
    for name, t in (("X", X), ("X_new", X_new)):
        _check(t, name, torch.float32, 2)
    for name, t in (("C", C), ("C_new", C_new)):
        _check(t, name, torch.float32, 2)
    HW = X.shape[0]
    if X.shape != (HW, 3) or X_new.shape != (HW, 3) or C.shape != (HW, 1) or C_new.shape != (HW, 1):
        raise RuntimeError("pointmap_update: expected X, X_new [HW,3] and C, C_new [HW,1]")
    if T is not None:
        T = T.reshape(-1)
        _check(T, "T", torch.float32, 1)
        if T.numel() != 8:
            raise RuntimeError("pointmap_update: T must hold 8 floats")
    dev = _on_device(X=X, C=C, X_new=X_new, C_new=C_new, T=T)
    with torch.cuda.device(dev):
        rc = lib.m3s_pointmap_update(FILTER_MODES[mode], _ptr(T), _ptr(X_new), _ptr(C_new), _ptr(X),
                                     _ptr(C), HW, _stream(dev))
    _raise(rc, "pointmap_update")
    return X, C


def gn_check(device=None):
    """Raise the deferred error of this thread's last Gauss-Newton call, if any: a bounded
    device-side wait of its factorisation that timed out (include/m3s_backend.h m3s_gn_check).
    Synchronises the current stream of `device` (default: the current device)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    _raise(lib.m3s_gn_check(_stream(dev)), "gauss_newton")


def gn_debug_flags() -> dict:
    """Diagnostics of the last Gauss-Newton call made with env M3S_GN_DEBUG_FLAGS set (that call
    reads its device flags back): the accumulate path it took and its lagged-factor PCG solves
    (include/m3s_backend.h m3s_gn_debug_flags / m3s_gn_pcg_stats)."""
    f = (ctypes.c_int * 4)()
    lib.m3s_gn_debug_flags(f)
    q = (ctypes.c_int * 5)()
    lib.m3s_gn_pcg_stats(q)
    return {"done": f[0], "fail": f[1], "packed": bool(f[2]), "ray_constrained": bool(f[3]),
            "pcg_planned": bool(q[3]), "pcg_runs": q[0], "pcg_steps": q[1], "pcg_fallbacks": q[2],
            "pcg_from": q[4]}


def version() -> str:
    return lib.m3s_version().decode()
