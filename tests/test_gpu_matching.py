"""GPU parity of the matching ops against the CPU oracle (bit-exact indices/flags).

The HIP kernels are called through the drop-in module (C ABI) on identical inputs; the
oracle is the checker.  Sizes: full 512x384 for B=1 (the tracking shape) and B=8 (add_factors'
batch), plus ragged / edge-case shapes.  iter_proj is bit-exact under every FMA-contraction
convention (CONTRACTS: the reference build's nvcc --fmad=true, the default; its right-product
variant; contraction off), each against the oracle in the same convention.
"""
import numpy as np
import pytest
import torch

from m3s import synth
from m3s.matching import prep_for_iter_proj

pytestmark = pytest.mark.gpu

CFG = dict(max_iter=10, lambda_init=1e-8, cost_thresh=1e-6)
CONTRACTS = ["nvcc", "nvcc_right", "off"]


def _iter_proj_both(backend, oracle, rays, pts, p_init, contract=None, **kw):
    c = dict(CFG, **kw)
    p_g, conv_g = backend.iter_proj(rays.cuda(), pts.cuda(), p_init.cuda(), c["max_iter"],
                                    c["lambda_init"], c["cost_thresh"], contract=contract)
    p_o, conv_o = oracle.iter_proj(rays.numpy(), pts.numpy(), p_init.numpy(), c["max_iter"],
                                   c["lambda_init"], c["cost_thresh"], contract=contract or "nvcc")
    return p_g.cpu().numpy(), conv_g.cpu().numpy(), p_o, conv_o


@pytest.mark.parametrize("contract", CONTRACTS)
@pytest.mark.parametrize("B,H,W,warm", [(1, 384, 512, False), (1, 384, 512, True), (2, 48, 64, False), (3, 5, 7, True)])
def test_iter_proj_bit_exact(backend, oracle, B, H, W, warm, contract):
    mp = synth.make_match_pair(B=B, H=H, W=W, seed=3 + H)
    rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init if warm else None)
    p_g, c_g, p_o, c_o = _iter_proj_both(backend, oracle, rays, pts, p_init, contract)
    # bit-exact floats and flags
    assert np.array_equal(p_g.view(np.uint32), p_o.view(np.uint32)), (
        f"{(p_g != p_o).sum()} of {p_o.size} coordinates differ")
    assert np.array_equal(c_g, c_o)
    # and the truncated match indices the caller uses (p.long())
    assert np.array_equal(p_g.astype(np.int64), p_o.astype(np.int64))


@pytest.mark.parametrize("warm", [False, True])
def test_iter_proj_bit_exact_b8_default_convention(backend, oracle, warm):
    """The bench's / add_factors' batch: 8 pairs at 512x384 under the default convention (the
    reference build's), bitwise; and the default equals an explicit contract="nvcc"."""
    mp = synth.make_match_pair(B=8, H=384, W=512, seed=11)
    rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init if warm else None)
    p_g, c_g, p_o, c_o = _iter_proj_both(backend, oracle, rays, pts, p_init)
    assert np.array_equal(p_g.view(np.uint32), p_o.view(np.uint32)), (p_g != p_o).sum()
    assert np.array_equal(c_g, c_o)
    p_n, c_n, _, _ = _iter_proj_both(backend, oracle, rays[:1], pts[:1], p_init[:1], "nvcc")
    assert np.array_equal(p_n.view(np.uint32), p_g[:1].view(np.uint32)) and np.array_equal(c_n, c_g[:1])


def test_iter_proj_edge_cases(backend, oracle):
    g = torch.Generator().manual_seed(0)
    B, H, W = 1, 16, 20
    rays = torch.randn((B, H, W, 9), generator=g)
    pts = torch.nn.functional.normalize(torch.randn((B, 50, 3), generator=g), dim=-1)
    # initial pixels far outside the image, on the border, and NaN
    p_init = torch.empty((B, 50, 2))
    p_init[0, :, 0] = torch.linspace(-100, 100, 50)
    p_init[0, :, 1] = torch.linspace(50, -50, 50)
    p_init[0, 3] = float("nan")
    for cm in CONTRACTS:
        for kw in (dict(), dict(max_iter=0), dict(max_iter=1), dict(lambda_init=10.0, cost_thresh=2.0)):
            p_g, c_g, p_o, c_o = _iter_proj_both(backend, oracle, rays, pts, p_init, cm, **kw)
            assert np.array_equal(p_g.view(np.uint32), p_o.view(np.uint32)), (cm, kw)
            assert np.array_equal(c_g, c_o), (cm, kw)


def test_iter_proj_empty(backend):
    rays = torch.zeros((0, 8, 8, 9), device="cuda")
    pts = torch.zeros((0, 64, 3), device="cuda")
    p = torch.zeros((0, 64, 2), device="cuda")
    p_new, conv = backend.iter_proj(rays, pts, p, 10, 1e-8, 1e-6)
    assert p_new.shape == (0, 64, 2) and conv.shape == (0, 64)


def _refine_both(backend, oracle, D11, D21, p1, radius=3, dmax=5, variant=None):
    """The product op (variant None) or a measurement-only variant (mast3r_slam_backends.variants)
    against the oracle."""
    if variant is None:
        (out_g,) = backend.refine_matches(D11.cuda(), D21.cuda(), p1.cuda(), radius, dmax)
    else:
        from mast3r_slam_backends import variants
        (out_g,) = variants.refine_matches_variant(variant, D11.cuda(), D21.cuda(), p1.cuda(), radius, dmax)
    out_o = oracle.refine_matches(D11.numpy(), D21.numpy(), p1.numpy(), radius, dmax)
    return out_g.cpu().numpy(), out_o


@pytest.mark.parametrize("dot2", [False, True])
@pytest.mark.parametrize("B,H,W", [(1, 384, 512), (2, 24, 32)])
def test_refine_matches_f16_bit_exact(backend, oracle, B, H, W, dot2):
    """Default fp16 path (every candidate's fp16 chain) and the DOT2 variant (bound-and-rescore:
    dot2 approximations, exact fp16 chains for the shortlist): both bit-exact."""
    mp = synth.make_match_pair(B=B, H=H, W=W, seed=11)
    p1 = torch.stack((mp.idx_init % W, mp.idx_init // W), -1).long()
    D11 = mp.D11.half()
    D21 = mp.D21.reshape(B, H * W, -1).half()
    out_g, out_o = _refine_both(backend, oracle, D11, D21, p1, variant=3 if dot2 else None)
    assert out_g.dtype == np.int64
    assert np.array_equal(out_g, out_o), f"{(out_g != out_o).any(-1).sum()} matches differ"


@pytest.mark.parametrize("variant", [1, 4, 5, 6])  # variants.LDS, LATTICE, BOX, PLANES
@pytest.mark.parametrize("scatter", [0, 3, 40, 10**6])
def test_refine_lds_tile_and_fallback(backend, oracle, scatter, variant):
    """The LDS-tiled and the lattice-bucket MFMA variants against the oracle and against the
    product candidate-gather kernel, bitwise (for the lattice kernel, 40 px scatter overflows the
    group boxes -> exact scoring of those groups).  ``scatter`` spreads the starting
    matches: 0/3 px keeps every tile's candidate box in LDS; 40 px makes the large-dilation
    boxes exceed the LDS budget (those levels gather from global memory); 10**6 puts most
    starts far outside the image (clipped windows, many empty)."""
    B, H, W = 2, 96, 128
    mp = synth.make_match_pair(B=B, H=H, W=W, seed=31)
    g = torch.Generator().manual_seed(scatter + 1)
    p1 = torch.stack((mp.idx_init % W, mp.idx_init // W), -1).long()
    if scatter:
        p1 = p1 + torch.randint(-scatter, scatter + 1, p1.shape, generator=g)
    D11 = mp.D11.half()
    D21 = mp.D21.reshape(B, H * W, -1).half()
    out_l, out_o = _refine_both(backend, oracle, D11, D21, p1, variant=variant)
    (out_gth,) = backend.refine_matches(D11.cuda(), D21.cuda(), p1.cuda(), 3, 5)
    assert np.array_equal(out_l, out_o), f"{(out_l != out_o).any(-1).sum()} matches differ"
    assert np.array_equal(out_l, out_gth.cpu().numpy())


@pytest.mark.parametrize("dtype,F", [(torch.float16, 24), (torch.float16, 5), (torch.float32, 24), (torch.float32, 3),
                                     (torch.float64, 24), (torch.float64, 7)])
def test_refine_matches_generic(backend, oracle, dtype, F):
    g = torch.Generator().manual_seed(F)
    B, H, W, N = 2, 13, 17, 40
    D11 = torch.randn((B, H, W, F), generator=g).to(dtype)
    D21 = torch.randn((B, N, F), generator=g).to(dtype)
    p1 = torch.stack((torch.randint(-5, W + 5, (B, N), generator=g),
                      torch.randint(-5, H + 5, (B, N), generator=g)), -1)
    for radius, dmax in ((3, 5), (1, 1), (0, 2), (2, 0)):
        out_g, out_o = _refine_both(backend, oracle, D11, D21, p1, radius, dmax)
        assert np.array_equal(out_g, out_o), (dtype, F, radius, dmax)


def test_refine_ties_and_zero_init(backend, oracle):
    # all-equal descriptors: ties everywhere -> strict '>' keeps the first candidate of the
    # first level; all-negative scores -> the match never moves (max starts at 0)
    B, H, W, F = 1, 20, 20, 24
    D11 = torch.full((B, H, W, F), 0.25, dtype=torch.float16)
    D21 = torch.full((B, 4, F), 0.25, dtype=torch.float16)
    p1 = torch.tensor([[[10, 10], [0, 0], [19, 5], [3, 17]]])
    out_g, out_o = _refine_both(backend, oracle, D11, D21, p1)
    assert np.array_equal(out_g, out_o)
    out_g2, out_o2 = _refine_both(backend, oracle, D11, -D21, p1)
    assert np.array_equal(out_g2, out_o2)
    assert np.array_equal(out_g2, p1.numpy())


def test_match_pipeline_against_golden(backend, oracle):
    """m3s.matching (GPU kernels) on the golden inputs.

    1. Identical-device inputs: the same glue on cuda, once with the HIP ops and once with
       the oracle as the ops (tensors moved to the host and back), must give identical
       indices and flags -- the kernels are bit-exact inside the pipeline.
    2. Against the reference-generated fixture (made by the reference glue on the CPU): the
       glue's own float ops (normalize, conv2d) run on the GPU here, whose conv/normalize
       kernels round differently from the CPU's, so a tiny fraction of p.long() truncation
       flips is possible; the glue itself is pinned bitwise on the CPU in
       tests/test_glue_golden.py.
    """
    import os
    import types

    import m3s.matching as mm

    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "glue_golden.npz"))
    t = lambda k: torch.from_numpy(gold[k]).cuda()

    ob = types.SimpleNamespace()

    def o_iter_proj(rays, pts, p_init, max_iter, lam, thr, contract="nvcc"):
        p, c = oracle.iter_proj(rays.cpu().numpy(), pts.cpu().numpy(), p_init.cpu().numpy(),
                                max_iter, lam, thr, contract=contract)
        return [torch.from_numpy(p).to(rays.device), torch.from_numpy(c).to(rays.device)]

    def o_refine(D11, D21, p1, radius, dmax):
        out = oracle.refine_matches(D11.cpu().numpy(), D21.cpu().numpy(), p1.cpu().numpy(), radius, dmax)
        return [torch.from_numpy(out).to(D11.device)]

    ob.iter_proj, ob.refine_matches = o_iter_proj, o_refine
    for tag, init in (("id", None), ("warm", t("idx_init"))):
        idx, valid = mm.match_iterative_proj(t("X11"), t("X21"), t("D11"), t("D21"), init, fused=False)
        real = mm.mast3r_slam_backends
        try:
            mm.mast3r_slam_backends = ob
            idx_o, valid_o = mm.match_iterative_proj(t("X11"), t("X21"), t("D11"), t("D21"), init,
                                                     fused=False)
        finally:
            mm.mast3r_slam_backends = real
        assert torch.equal(idx, idx_o) and torch.equal(valid, valid_o), tag
        agree = (idx.cpu().numpy() == gold[f"match_{tag}_idx"]).mean()
        vagree = (valid.cpu().numpy() == gold[f"match_{tag}_valid"]).mean()
        assert agree > 0.999 and vagree > 0.999, (tag, agree, vagree)


@pytest.mark.parametrize("contract", [None] + CONTRACTS)
def test_fused_pipeline_bitwise_equals_reference_fixture(backend, contract):
    """The fused op (csrc/match_glue.hip: prep + iter_proj + occlusion + refine + linear index)
    against the fixture made by running the REFERENCE's matching.py glue on the HOST, with the
    oracle as its two kernels (in each contraction convention; None = the default, the
    reference build's): identical indices and valid flags for the identity and the warm start.
    (The glue is bitwise the reference's host run; torch's GPU normalize / conv2d round
    differently -- bench.py reports how many matches that changes.)"""
    import os

    import m3s.matching as mm

    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "glue_golden.npz"))
    t = lambda k: torch.from_numpy(gold[k]).cuda()
    sfx = "" if contract is None else f"_{contract}"
    for tag, init in (("id", None), ("warm", t("idx_init"))):
        idx, valid = mm.match_iterative_proj(t("X11"), t("X21"), t("D11"), t("D21"), init, contract=contract)
        assert idx.dtype == torch.int64 and valid.dtype == torch.bool and valid.shape[-1] == 1
        assert np.array_equal(idx.cpu().numpy(), gold[f"match_{tag}{sfx}_idx"]), (
            tag, (idx.cpu().numpy() != gold[f"match_{tag}{sfx}_idx"]).sum())
        assert np.array_equal(valid.cpu().numpy(), gold[f"match_{tag}{sfx}_valid"]), tag


@pytest.mark.parametrize("B,H,W,radius,contract", [(1, 384, 512, 3, "nvcc"), (1, 384, 512, 3, "off"),
                                                    (2, 37, 53, 3, "nvcc_right"), (1, 24, 32, 0, "nvcc"),
                                                    (2, 16, 16, 2, "nvcc")])
def test_fused_pipeline_matches_oracle_pipeline(backend, oracle, B, H, W, radius, contract):
    """On synthetic pairs (full size, ragged tiles, radius 0 = no refine): the fused op equals
    the oracle's whole pipeline (its C restatement of the glue, pinned to the reference's glue
    by test_glue_golden.py, plus the oracle kernels) in the same contraction convention,
    identity and warm start."""
    import m3s.matching as mm
    from m3s.config import config as cfg0

    mp = synth.make_match_pair(B=B, H=H, W=W, seed=5 + H)
    c = dict(cfg0["matching"], radius=radius)
    for init in (None, mp.idx_init):
        idx, valid = mm.match_iterative_proj(mp.X11.cuda(), mp.X21.cuda(), mp.D11.cuda(), mp.D21.cuda(),
                                             None if init is None else init.cuda(), cfg={"matching": c},
                                             contract=contract)
        idx_o, valid_o = oracle.match_iterative_proj(
            mp.X11.numpy(), mp.X21.numpy(), mp.D11.numpy(), mp.D21.numpy(),
            None if init is None else init.numpy(), c["max_iter"], c["lambda_init"],
            c["convergence_thresh"], c["dist_thresh"], c["radius"], c["dilation_max"], contract=contract)
        assert np.array_equal(idx.cpu().numpy(), idx_o), (idx.cpu().numpy() != idx_o).sum()
        assert np.array_equal(valid.cpu().numpy(), valid_o)


@pytest.mark.parametrize("variant", [2, 4])  # variants.MFMA, variants.LATTICE
@pytest.mark.parametrize("warm", [False, True])
def test_refine_mfma_path_bit_exact(backend, oracle, warm, variant):
    """The MFMA correlation variant (approximate scores on
    v_mfma_f32_16x16x32_f16, exact c10::Half re-scoring of every candidate within the error
    bound of the best) gives the oracle's indices bit for bit at 512x384, and re-scores only a
    fraction of the candidates."""
    mp = synth.make_match_pair(B=1, H=384, W=512, seed=21)
    rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init if warm else None)
    p, _ = oracle.iter_proj(rays.numpy(), pts.numpy(), p_init.numpy(), 10, 1e-8, 1e-6)
    p1 = torch.from_numpy(p).long()
    D11 = mp.D11.half()
    D21 = mp.D21.view(1, -1, 24).half()
    from mast3r_slam_backends import variants
    variants.variant_stats(True)
    out_g, out_o = _refine_both(backend, oracle, D11, D21, p1, 3, 5, variant=variant)
    resc, total = variants.variant_stats(False)
    assert np.array_equal(out_g, out_o), f"{(out_g != out_o).any(-1).sum()} matches differ"
    assert 0 < resc < total, (resc, total)


@pytest.mark.parametrize("path", [2, 3, 4])  # variants.MFMA, variants.DOT2, variants.LATTICE
def test_refine_mfma_path_edge_cases(backend, oracle, path):
    """Ties everywhere, all-negative scores, out-of-image starts, huge values (bound beyond fp16
    range: every candidate re-scored) and NaN descriptors, all bit-exact on the MFMA and the dot2
    bound-and-rescore paths."""
    g = torch.Generator().manual_seed(4)
    B, H, W, F = 1, 40, 36, 24
    p1 = torch.stack((torch.randint(-5, W + 5, (B, H * W), generator=g),
                      torch.randint(-5, H + 5, (B, H * W), generator=g)), -1)
    cases = {
        "ties": (torch.full((B, H, W, F), 0.25), torch.full((B, H * W, F), 0.25)),
        "negative": (torch.full((B, H, W, F), 0.25), torch.full((B, H * W, F), -0.25)),
        "random": (torch.randn((B, H, W, F), generator=g), torch.randn((B, H * W, F), generator=g)),
        "huge": (torch.randn((B, H, W, F), generator=g) * 200, torch.randn((B, H * W, F), generator=g) * 200),
    }
    nan11 = torch.randn((B, H, W, F), generator=g)
    nan11[0, 7, 9, 3] = float("nan")
    cases["nan"] = (nan11, torch.randn((B, H * W, F), generator=g))
    for name, (D11, D21) in cases.items():
        out_g, out_o = _refine_both(backend, oracle, D11.half(), D21.half(), p1, 3, 5, variant=path)
        assert np.array_equal(out_g, out_o), name
