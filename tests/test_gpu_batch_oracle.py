"""Batched frames (tt_ctx_set_frame_pixels; bench.py's N = 1 headline traces 4 frames per launch) against the
ORACLE, frame by frame.

B frames are traced as one W x B*H screen: frame j's rays carry PixelIndex + j W H, the bounce enqueue draws
frame j's random numbers from the frame-local pixel at frames + j. Each frame must equal the oracle's frame
traced ALONE (oracle/tt_oracle.c through tests/oracle_ctypes.py: Generate at frames + j, the primary trace
with _PrimaryTriangleInfo, the enqueue at frames + j, the bounce-1 trace with its GlobalColors-gated
_PrimaryTriangleInfo), byte for byte: primary records, the compacted bounce-1 rays (frame j's survivors follow
frame j-1's, each frame in source order), their records and both info texel forms. A negative control shows
the test can fail: the oracle's enqueue keyed on the GLOBAL pixel (no frame_pixels) differs from frame 1 on.
"""
import numpy as np
import pytest

import oracle_ctypes as O
import ttconfigs as T
import tthip

from parity_util import CPU_THREADS, FAR

pytestmark = pytest.mark.gpu


def _run(sc, c2w, ip, W, H, B, F0, near):
    WH = W * H
    eng = tthip.Engine(0)
    try:
        eng.upload(sc)
        eng.set_frame_pixels(WH)
        alone = [O.generate(c2w, ip, W, H, near, FAR, jitter=1, frames=F0 + j, max_bounce=1) for j in range(B)]
        rb = np.zeros(2 * B * WH, tthip.RAY_DTYPE)
        for j in range(B):
            rb[j * WH:(j + 1) * WH] = alone[j][:WH]
            rb["PixelIndex"][j * WH:(j + 1) * WH] += np.uint32(j * WH)
        colors = np.zeros(WH, tthip.COL_DTYPE)
        colors["Data"][:, 3] = 1.0
        colors_b = np.tile(colors, B)
        info0 = np.full((B * WH, 4), 0xA5A5A5A5, np.uint32)
        info1 = np.full((B * WH, 4), 0xA5A5A5A5, np.uint32)
        eng.trace(rb, B * WH, 0, FAR, W, B * H, info=info0)
        primary = rb[:B * WH].copy()
        nb = eng.enqueue_bounce(rb, B * WH, 0, FAR, W, B * H, frames=F0, max_bounce=1)
        eng.trace(rb, nb, 1, FAR, W, B * H, info=info1, colors=colors_b)
    finally:
        eng.close()
    off = B * WH
    for j in range(B):
        o = alone[j]
        i0 = np.full((WH, 4), 0xA5A5A5A5, np.uint32)
        i1 = np.full((WH, 4), 0xA5A5A5A5, np.uint32)
        assert O.trace(sc, o, WH, 0, FAR, W, H, info=i0, nthreads=CPU_THREADS)[0] == 0
        nbj = O.enqueue_bounce(sc, o, WH, 0, FAR, W, H, frames=F0 + j, max_bounce=1)
        assert O.trace(sc, o, nbj, 1, FAR, W, H, info=i1, colors=colors, nthreads=CPU_THREADS)[0] == 0
        ref_p = o[:WH].copy()
        ref_p["PixelIndex"] += np.uint32(j * WH)
        assert np.array_equal(rb[j * WH:(j + 1) * WH].view(np.uint8), ref_p.view(np.uint8)), f"frame {j}: primary"
        assert np.array_equal(info0[j * WH:(j + 1) * WH], i0), f"frame {j}: _PrimaryTriangleInfo (bounce 0)"
        ref_b = o[WH:WH + nbj].copy()
        ref_b["PixelIndex"] += np.uint32(j * WH)
        assert off + nbj <= B * WH + nb, f"frame {j}: bounce count"
        assert np.array_equal(rb[off:off + nbj].view(np.uint8), ref_b.view(np.uint8)), f"frame {j}: bounce-1 rays/records"
        assert np.array_equal(info1[j * WH:(j + 1) * WH], i1), f"frame {j}: _PrimaryTriangleInfo (bounce 1)"
        off += nbj
    assert off == B * WH + nb
    # negative control: the enqueue keyed on the global pixel (the frame_pixels = 0 form) at F0 gives frame 0's
    # bounce rays but not frame 1's -- so a kernel that ignored frame_pixels fails the comparison above
    g = primary.copy()
    gb = np.zeros(2 * B * WH, tthip.RAY_DTYPE)
    gb[:B * WH] = g
    nbg = O.enqueue_bounce(sc, gb, B * WH, 0, FAR, W, B * H, frames=F0, max_bounce=1)
    assert nbg == nb  # survivors are the hits either way
    n0 = int((primary["hits"][:WH, 1] != 0xFFFFFFFF).sum())
    dirs_g = gb["direction"][B * WH:B * WH + nbg]
    # (rb's bounce rays were traced in place since; their directions are untouched by the trace)
    dirs = rb["direction"][B * WH:B * WH + nb]
    assert np.array_equal(dirs_g[:n0], dirs[:n0])
    assert not np.array_equal(dirs_g[n0:], dirs[n0:])


def test_batched_soup_two_frames_equal_the_oracle_frames():
    sc = tthip.single_object_scene(tthip.Mesh.soup(23, 30000, 1.0, 0.08))
    W, H = 256, 160
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.6), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, FAR)
    _run(sc, c2w, ip, W, H, 2, 3, 0.05)


def test_batched_c2_1080p_two_frames_equal_the_oracle_frames():
    """BASELINE.json C2 at 1920x1080, two frames per launch (the headline traces 4 this way)."""
    W, H = 1920, 1080
    c2w, ip = T.C2_VIEW.camera(W, H)
    _run(T.c2_sponza(), c2w, ip, W, H, 2, 0, T.NEAR)
