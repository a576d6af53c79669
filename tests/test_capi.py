"""The C-ABI library loads, exports every symbol include/m3s_backend.h declares, and the
drop-in module validates arguments like the reference (no GPU needed, no compute calls)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "m3s_backend.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(m3s_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(backend):
    syms = declared_symbols()
    assert len(syms) >= 15, syms
    lib = ctypes.CDLL(backend.library_path)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_variants_library_exports_its_header():
    """The measurement-only refine variants (and the test hook) live in their own library (not the
    drop-in one)."""
    src = open(os.path.join(ROOT, "include", "m3s_variants.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    syms = sorted(set(re.findall(r"\b(m3s_[a-z0-9_]+)\s*\(", src)))
    assert len(syms) == 4, syms
    path = os.path.join(ROOT, "mast3r-slam_amd", "lib", "libm3s_variants.so")
    lib = ctypes.CDLL(path)
    assert all(hasattr(lib, s) for s in syms)
    product = ctypes.CDLL(os.path.join(ROOT, "mast3r-slam_amd", "lib", "libm3s_backend.so"))
    assert not any(hasattr(product, s) for s in syms)


def test_library_is_gfx950_code_object(backend):
    data = open(backend.library_path, "rb").read()
    assert b"gfx950" in data
    assert backend.version().endswith("gfx950")


def test_workspace_size_query(backend):
    f = backend.lib.m3s_gn_workspace_bytes
    small = f(1, 2, 64, 2, 2)
    big = f(2, 128, 384 * 512, 512, 512)
    assert 0 < small < big
    # cfg3: the per-call packed stream (8 B per directed point-edge) dominates, then the calib
    # depth / ray-table / inverse-depth arrays ((2N + 1) HW floats); the dense f64 matrices are
    # not part of it (sized per call by the solver actually used)
    HW = 384 * 512
    assert 8 * 512 * HW < big < 8 * 512 * HW + (2 * 128 + 1) * HW * 4 + 64 * 2**20
    # far beyond the dense-solve limit (1171 keyframes): still a valid (sparse-path) size
    huge = f(1, 4096, 64, 8192, 8192)
    assert 0 < huge < 64 * 2**20
    assert f(1, 0, 64, 2, 2) == 0  # invalid sizes


def test_cpu_tensors_are_rejected(backend):
    with pytest.raises(RuntimeError, match="no CPU path"):
        backend.iter_proj(torch.zeros(1, 4, 4, 9), torch.zeros(1, 16, 3), torch.zeros(1, 16, 2), 10, 1e-8, 1e-6)
    with pytest.raises(RuntimeError, match="no CPU path"):
        backend.refine_matches(torch.zeros(1, 4, 4, 24).half(), torch.zeros(1, 16, 24).half(),
                               torch.zeros(1, 16, 2, dtype=torch.long), 3, 5)
    N, HW, E = 3, 8, 4
    with pytest.raises(RuntimeError, match="no CPU path"):
        backend.gauss_newton_rays(torch.zeros(N, 8), torch.zeros(N, HW, 3), torch.zeros(N, HW, 1),
                                  torch.zeros(E, dtype=torch.long), torch.zeros(E, dtype=torch.long),
                                  torch.zeros(E, HW, dtype=torch.long), torch.zeros(E, HW, 1, dtype=torch.bool),
                                  torch.zeros(E, HW, 1), 0.003, 10.0, 0.0, 1.5, 10, 1e-8)


def test_contiguity_and_dtype_checks(backend):
    # the reference's CHECK_CONTIGUOUS message (gn.h:5) and accessor dtype errors
    x = torch.zeros(1, 4, 9, 4).permute(0, 1, 3, 2)
    with pytest.raises(RuntimeError, match="rays_img_with_grad must be contiguous"):
        backend.iter_proj(x, torch.zeros(1, 16, 3), torch.zeros(1, 16, 2), 10, 1e-8, 1e-6)
    with pytest.raises(RuntimeError, match="expected scalar type Float but found Double"):
        backend.iter_proj(torch.zeros(1, 4, 4, 9, dtype=torch.float64), torch.zeros(1, 16, 3),
                          torch.zeros(1, 16, 2), 10, 1e-8, 1e-6)
    with pytest.raises(RuntimeError, match="expected scalar type Long"):
        backend.refine_matches(torch.zeros(1, 4, 4, 24).half(), torch.zeros(1, 16, 24).half(),
                               torch.zeros(1, 16, 2, dtype=torch.int32), 3, 5)


def test_no_oracle_in_product_path():
    """The product package must never import the oracle (test infrastructure)."""
    pkg = os.path.join(ROOT, "mast3r-slam_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
                assert "libm3s_oracle" not in txt, f
