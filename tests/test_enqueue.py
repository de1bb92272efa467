"""Row f2: the diffuse-bounce enqueue (kernel_shade's diffuse path + next-ray append,
RayTracingShader.compute:52-84, 99-124, 284, 293, 498-506) restated in the oracle with the
library's stable (source-order) compaction and the pinned sincos. CPU checks of the restatement;
the GPU comparison is tests/test_gpu_parity.py::test_bounce_enqueue_bit_exact."""
import math

import numpy as np
import pytest

import golden_io
import oracle_ctypes as O
import tthip

FAR = 1000.0


def test_sincos_pinned_accuracy():
    # the disc sample's angle range: [-pi/4, pi/4] (first branch) and [pi/4, 3pi/4] (second)
    phis = np.linspace(-0.25 * math.pi, 0.75 * math.pi, 20001, dtype=np.float32)
    worst = 0.0
    for phi in phis[::7]:
        s, c = O.sincos_pinned(float(phi))
        worst = max(worst, abs(s - math.sin(float(phi))), abs(c - math.cos(float(phi))))
    assert worst < 3e-7, worst  # a few float ulps of |sin|, |cos| <= 1
    s0, c0 = O.sincos_pinned(0.0)
    assert (s0, c0) == (0.0, 1.0)


def _traced_soup():
    g = golden_io.load("soup")
    sc, W, H = g["scene"], g["W"], g["H"]
    r = g["rays0"].copy()
    st, _ = O.trace(sc, r, W * H, 0, FAR, W, H)
    assert st == 0
    return sc, W, H, r


def test_oracle_enqueue_stable_and_geometric():
    sc, W, H, r = _traced_soup()
    nb = O.enqueue_bounce(sc, r, W * H, 0, FAR, W, H, frames=2, max_bounce=4)
    hit = (r["hits"][: W * H, 1] != 0xFFFFFFFF) & (r["hits"][: W * H, 2].view(np.float32) < FAR)
    assert 0 < nb <= int(hit.sum())
    out = r[W * H: W * H + nb]
    # stable compaction: survivors in source order, hit records carried over
    src_pix = r["PixelIndex"][: W * H][hit]
    sel = np.isin(src_pix, out["PixelIndex"])
    assert np.array_equal(src_pix[sel], out["PixelIndex"])
    assert np.all(np.diff(out["PixelIndex"].astype(np.int64)) > 0)
    assert np.array_equal(out["hits"], r["hits"][: W * H][hit][np.isin(src_pix, out["PixelIndex"])])
    d = out["direction"].astype(np.float64)
    assert np.allclose(np.linalg.norm(d, axis=1), 1.0, atol=1e-5)
    assert np.all(out["last_pdf"] > 0)
    # the new origin sits 1e-4 off the hit point along the unsmoothed normal, on the incoming side
    n6 = O.resolve_normals(sc, r, W * H, 0, FAR, W, H)[hit][np.isin(src_pix, out["PixelIndex"])]
    src = r[: W * H][hit][np.isin(src_pix, out["PixelIndex"])]
    t = src["hits"][:, 2].view(np.float32).astype(np.float64)
    pos = src["origin"].astype(np.float64) + src["direction"].astype(np.float64) * t[:, None]
    off = out["origin"].astype(np.float64) - pos
    assert np.all(np.linalg.norm(off, axis=1) < 2e-4)
    us = n6[:, 3:6].astype(np.float64)
    flip = np.sum(src["direction"] * us, axis=1) > 0
    us[flip] *= -1
    # the bounce leaves into the hemisphere of the (flipped) shading normal: mostly above the surface
    g = n6[:, 0:3].astype(np.float64)
    g[flip] *= -1
    assert np.mean(np.sum(d * g, axis=1) > 0) > 0.99


def test_oracle_enqueue_odd_bounce_reads_second_half():
    sc, W, H, r = _traced_soup()
    n1 = O.enqueue_bounce(sc, r, W * H, 0, FAR, W, H)
    st, _ = O.trace(sc, r, n1, 1, FAR, W, H)
    assert st == 0
    before = r[W * H:].copy()
    n2 = O.enqueue_bounce(sc, r, n1, 1, FAR, W, H)
    assert 0 < n2 <= n1
    assert np.array_equal(r[W * H:].view(np.uint8), before.view(np.uint8))  # source half untouched
    assert np.all(np.diff(r["PixelIndex"][:n2].astype(np.int64)) > 0)


def test_oracle_enqueue_empty_and_bad_args():
    sc, W, H, r = _traced_soup()
    assert O.enqueue_bounce(sc, r, 0, 0, FAR, W, H) == 0
    with pytest.raises(AssertionError):
        O.enqueue_bounce(sc, r, W * H + 1, 0, FAR, W, H)
