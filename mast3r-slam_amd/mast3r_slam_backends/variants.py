"""Measurement-only refine_matches variants (lib/libm3s_variants.so, include/m3s_variants.h).

Not part of the drop-in op set: each variant returns the same matches as ``refine_matches``
(bit-exact, tested) and was measured slower than the product kernel on the bench data
(DESIGN.md section 4).  bench.py and the tests A/B them through this module."""
import ctypes
import os

import torch

from . import _check, _on_device, _ptr, _stream

LDS, MFMA, DOT2, LATTICE, BOX, PLANES = 1, 2, 3, 4, 5, 6  # M3S_REFINE_VARIANT_*

library_path = os.environ.get("M3S_VARIANTS_LIB", os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libm3s_variants.so"))
if not os.path.exists(library_path):
    raise ImportError(f"refine variants library not found at {library_path}; build with `make -C mast3r-slam_amd`")
lib = ctypes.CDLL(library_path)
lib.m3s_refine_variant_f16.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 5 + \
    [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.m3s_refine_variant_stats.argtypes = [ctypes.c_int, ctypes.c_void_p]
lib.m3s_refine_variant_stats.restype = None
lib.m3s_variants_last_error.restype = ctypes.c_char_p
lib.m3s_test_hold_cus.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]


def refine_matches_variant(kind, D11, D21, p1, window_size, dilation_max):
    """``refine_matches`` (fp16, F = 24, radius 3) computed by variant ``kind`` (LDS / MFMA / DOT2)."""
    _check(D11, "D11", (torch.float16,), 4)
    _check(D21, "D21", D11.dtype, 3)
    _check(p1, "p1", torch.int64, 3)
    dev = _on_device(D11=D11, D21=D21, p1=p1)
    B, H, W, F = D11.shape
    N = p1.shape[1]
    p1_new = torch.zeros((B, N, 2), dtype=p1.dtype, device=dev)
    with torch.cuda.device(dev):
        rc = lib.m3s_refine_variant_f16(int(kind), _ptr(D11), _ptr(D21), _ptr(p1), _ptr(p1_new), B, H, W, N, F,
                                        int(window_size), int(dilation_max), _stream(dev))
    if rc != 0:
        raise RuntimeError(f"refine variant {kind}: {lib.m3s_variants_last_error().decode()}")
    return [p1_new]


def variant_stats(enable=True):
    """Counters of the bound-and-rescore variants (MFMA, DOT2, LATTICE): (exactly re-scored, in-image
    candidates) since the previous call; ``enable`` switches the counting for later calls.
    ``mfma_issued()`` gives the lattice kernel's MFMA count of the same interval."""
    out = (ctypes.c_ulonglong * 3)()
    lib.m3s_refine_variant_stats(int(bool(enable)), ctypes.cast(out, ctypes.c_void_p))
    variant_stats.mfma = int(out[2])
    return int(out[0]), int(out[1])


def mfma_issued():
    return getattr(variant_stats, "mfma", 0)


def hold_cus(nblocks, lds_bytes, usec, stream):
    """Test hook: ``nblocks`` workgroups on ``stream`` (a torch.cuda.Stream) that each hold
    ``lds_bytes`` of LDS for ``usec`` microseconds -- CUs taken away from a concurrent launch."""
    rc = lib.m3s_test_hold_cus(int(nblocks), int(lds_bytes), int(usec), ctypes.c_void_p(stream.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"hold_cus: rc {rc}")
