"""The oracle's c10::Half arithmetic (round-to-nearest-even, subnormals, overflow) against
numpy's IEEE float16, which the refine_matches parity rests on."""
import numpy as np


def test_f16_to_f32_all_bit_patterns(oracle):
    bits = np.arange(0, 1 << 16, dtype=np.uint32)
    ref = bits.astype(np.uint16).view(np.float16).astype(np.float32)
    got = np.array([oracle.f16_bits_to_f32(int(b)) for b in bits[::7]], np.float32)
    r = ref[::7]
    nan = np.isnan(r)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), r[~nan].view(np.uint32))


def test_f32_to_f16_rounding(oracle):
    rng = np.random.default_rng(0)
    # random floats over the half range, halfway cases, subnormals, overflow boundary
    vals = np.concatenate([
        rng.standard_normal(20000).astype(np.float32) * np.float32(10.0) ** rng.integers(-9, 5, 20000),
        (np.arange(1, 2048, dtype=np.float32) + 0.5) * np.float32(2.0 ** -24),  # subnormal ties
        np.array([65504, 65519.99, 65520, 65536, 1e9, -65520, 2.0 ** -25, 2.0 ** -26, 0.0, -0.0,
                  np.inf, -np.inf], np.float32),
    ]).astype(np.float32)
    # exact ties between adjacent normal halves
    h = np.arange(0x0400, 0x7bff, 37, dtype=np.uint16).view(np.float16).astype(np.float32)
    h2 = np.nextafter(h.astype(np.float16), np.float16(np.inf)).astype(np.float32)
    vals = np.concatenate([vals, (h + h2) / 2]).astype(np.float32)
    with np.errstate(over="ignore"):
        ref = vals.astype(np.float16).view(np.uint16)
    got = np.array([oracle.f32_to_f16_bits(float(v)) for v in vals], np.uint16)
    assert np.array_equal(got, ref)


def test_half_dot_is_sequential_per_op_rounding(oracle):
    """refine_matches scores: a 24-term dot product rounded to half after every * and +.
    Checked through the oracle kernel on a 1x1 image with a planted descriptor."""
    rng = np.random.default_rng(3)
    for _ in range(200):
        a = rng.standard_normal(24).astype(np.float16)
        b = rng.standard_normal(24).astype(np.float16)
        s = np.float16(0)
        for k in range(24):
            s = np.float16(s + np.float16(a[k] * b[k]))
        # one candidate image: the match moves iff the sequential half score > 0
        D11 = b.reshape(1, 1, 1, 24)
        D21 = a.reshape(1, 1, 24)
        p1 = np.array([[[0, 0]]], np.int64)
        out = oracle.refine_matches(D11, D21, p1, 1, 1)
        assert np.array_equal(out, p1)  # single in-bounds candidate is the start pixel
        # 2-pixel image: candidate (1,0) carries b, start pixel carries zeros
        D11b = np.zeros((1, 1, 2, 24), np.float16)
        D11b[0, 0, 1] = b
        out = oracle.refine_matches(D11b, D21, p1, 1, 1)
        assert (out[0, 0, 0] == 1) == bool(s > 0)
