"""Row f1's colour encodings (CommonData.cginc:479-509 packRGBE / unpackRGBE, :1576-1619
EncodeRGB / DecodeRGB) and HLSL pow, as pinned in the oracle restatement (the GPU side,
csrc/tt_encode.h, is checked against it bit for bit in test_gpu_parity.py). Known answers follow
from the formulas; the transcendental pins are checked against float64 math."""
import math

import numpy as np
import pytest

import oracle_ctypes as O


def f32(x):
    return float(np.float32(x))


def test_pack_rgbe_exponent_saturates():
    # floor(log2(5000)) + 20 = 32 clamps to 31: the reference's packRGBE saturates the exponent
    assert O.pack_rgbe([5000.0, 0.0, 0.0]) >> 27 == 31


def test_pack_rgbe_known_answers():
    assert O.pack_rgbe([0.0, 0.0, 0.0]) == 0
    assert O.pack_rgbe([-1.0, -2.0, float("nan")]) == 0  # max(0, v): negatives and NaN read as 0
    # max 1.0: exponent 0, scale 256 -> 256 per channel
    assert O.pack_rgbe([1.0, 1.0, 1.0]) == (20 << 27) | 256 | (256 << 9) | (256 << 18)
    # max 3.0: exponent floor(log2 3) = 1, scale 128: 3 -> 384, 0.5 -> 64, 1 -> 128
    assert O.pack_rgbe([3.0, 0.5, 1.0]) == (21 << 27) | 384 | (64 << 9) | (128 << 18)
    # just below a power of two: floor(log2) is exact (frexp), not the rounded log2
    x = f32(np.nextafter(np.float32(2.0), np.float32(0.0)))
    assert O.pack_rgbe([x, 0.0, 0.0]) >> 27 == 20  # exponent 0
    # round() is half-to-even: 0.5 * 256 / 2^... -> exact halves
    assert O.pack_rgbe([1.0, 1.5 / 256.0, 2.5 / 256.0]) & 0x7FFFFFF == 256 | (2 << 9) | (2 << 18)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_rgbe_round_trip(seed):
    rng = np.random.default_rng(seed)
    for _ in range(300):
        # the 5-bit exponent field holds floor(log2(max)) + 20 clamped to [0, 31] (:487), so the
        # round trip holds for max in [2^-20, 2^12)
        v = rng.uniform(0, 1, 3) * 10.0 ** rng.uniform(-4, 3.5)
        u = O.unpack_rgbe(O.pack_rgbe(v))
        m = v.max()
        assert np.all(np.abs(u - v) <= m / 256.0 * 0.51 + 1e-30), (v, u)


def test_encode_decode_rgb_round_trip():
    rng = np.random.default_rng(7)
    assert O.encode_rgb([0.0, 0.0, 0.0]) == 0
    assert np.array_equal(O.decode_rgb(0), np.zeros(3, np.float32))
    for _ in range(300):
        c = rng.uniform(0.05, 1.0, 3) * 10.0 ** rng.uniform(-2, 2)
        d = O.decode_rgb(O.encode_rgb(c))
        # LogLuv-style: 14-bit log luminance (1/409.6 octave), 9-bit chroma -> a few percent
        assert np.allclose(d, c, rtol=0.06, atol=0.02 * c.max()), (c, d)


def test_pow_pin_matches_float_semantics():
    """pow(x, y) = exp2(y * log2(x)) with float intermediates; log2 / exp2 correctly rounded except
    at rounding boundaries closer than the double series' error."""
    rng = np.random.default_rng(11)
    bad = 0
    xs = rng.uniform(0, 4, 2000).astype(np.float32)
    for x in xs:
        for y in (np.float32(2.2), np.float32(1.0) / np.float32(2.2)):
            lg = np.float32(math.log2(float(x))) if x > 0 else np.float32(-np.inf)
            want = np.float32(2.0 ** float(np.float32(y * lg))) if x > 0 else np.float32(0.0)
            got = np.float32(O.hlsl_pow(float(x), float(y)))
            bad += int(got != want)
    assert bad <= 2, f"{bad} of 4000 differ from correctly rounded log2 / exp2"
    assert O.hlsl_pow(0.0, 2.2) == 0.0
    assert O.hlsl_pow(2.0, 3.0) == 8.0 and O.hlsl_pow(2.0, -3.0) == 0.125
    assert math.isnan(O.hlsl_pow(-1.0, 2.2))
