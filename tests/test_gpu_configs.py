"""GPU parity on the BASELINE.json configurations beyond C2's primary + bounce-1 case
("Synthetic inputs"; scenes from ``ttconfigs``):

  C3  C2 geometry at 1920x1080, primary + 3 diffuse bounces: every bounce's compacted rays (the
      GPU's stable look-back enqueue, itself bit-exact against the oracle's enqueue) traced
      bit-exact against the oracle, with the GlobalColors-gated _PrimaryTriangleInfo forms at
      bounces 1-3.
  C4  Bistro-shaped two-level instancing (600 unique BLAS, 2,400 instances, 4.8M unique tris) at
      1920x1080: full-frame primary and bounce-1 parity, BLAS-entry counts equal.
  C5  San-Miguel-shaped 10M tris at 3840x2160: determinism, full-frame oracle parity, and
      the 8-GPU 64x64 round-robin tile sharding reassembled byte-identical to
      the single-launch frame (hit records and _PrimaryTriangleInfo); the bench's C5 frame
      (MaxBounce 1, frames 0), whose one direction.x == +0 ray is the launch's longest chain.
"""
import numpy as np
import pytest

import oracle_ctypes as O
import ttconfigs as T
import ttdist
import tthip
from parity_util import CPU_THREADS, FAR, assert_same, trace_both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    return T.c2_sponza()


def test_c3_primary_plus_three_bounces(engine, c2):
    W, H = 1920, 1080  # the bench's C3 frame
    WH = W * H
    c2w, ip = T.C2_VIEW.camera(W, H)
    engine.upload(c2)
    rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=3, max_bounce=3)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = (np.arange(WH) % 5) - 1.0  # Data.w in {-1, 0, 1, 2, 3}: every gate form
    rg, rc, ig, ic, s, cnt = trace_both(engine, c2, rays, WH, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, WH)
    n = WH
    for bounce in (1, 2, 3):
        ref = rg.copy()
        nb = engine.enqueue_bounce(rg, n, bounce - 1, FAR, W, H, frames=3, max_bounce=3)
        assert 0 < nb <= n
        off = (bounce % 2) * WH
        assert O.enqueue_bounce(c2, ref, n, bounce - 1, FAR, W, H, frames=3, max_bounce=3) == nb
        assert np.array_equal(rg[off:off + nb].view(np.uint32), ref[off:off + nb].view(np.uint32))
        del ref
        assert np.allclose(np.linalg.norm(rg["direction"][off:off + nb], axis=1), 1.0, atol=1e-5)
        rg, rc, ig, ic, s, cnt = trace_both(engine, c2, rg, nb, bounce, W, H, colors=colors, upload=False)
        assert_same(rg, rc, ig, ic, off, nb)
        assert s.node_visits == int(cnt["node_visits"].sum()) and s.tri_tests == int(cnt["tri_tests"].sum())
        assert s.reps_exhausted == int((cnt["status"] == 1).sum())
        n = nb


@pytest.fixture(scope="module")
def c4():
    return T.c4_bistro()


def test_c4_bistro_1080p_full_parity(engine, c4):
    assert len(c4.meshdata) == 1 + 2400 and c4.meta["unique_blas"] == 600
    W, H = T.C4_VIEW.width, T.C4_VIEW.height
    WH = W * H
    c2w, ip = T.C4_VIEW.camera()
    engine.upload(c4)
    rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, T.NEAR, FAR, jitter=0)
    rg, rc, ig, ic, s, cnt = trace_both(engine, c4, rays, WH, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, WH)
    assert s.blas_entries == int(cnt["blas_entries"].sum()) > 2 * WH  # several instances per ray
    nb = engine.enqueue_bounce(rg, WH, 0, FAR, W, H)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    rg2, rc2, ig2, ic2, s2, cnt2 = trace_both(engine, c4, rg, nb, 1, W, H, colors=colors, upload=False)
    assert_same(rg2, rc2, ig2, ic2, WH, nb)
    assert s2.node_visits == int(cnt2["node_visits"].sum())


@pytest.fixture(scope="module")
def c5():
    return T.c5_san_miguel()


def test_c5_san_miguel_4k_full_parity_and_tile_sharded(engine, c5):
    sc = c5
    assert len(sc.tris) == T.C5_TRIS
    W, H = T.C5_VIEW.width, T.C5_VIEW.height
    WH = W * H
    c2w, ip = T.C5_VIEW.camera()
    engine.upload(sc)
    rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=1)
    a = rays.copy()
    info_a = np.zeros((WH, 4), np.uint32)
    engine.trace(a, WH, 0, FAR, W, H, info=info_a)
    b = rays.copy()
    engine.trace(b, WH, 0, FAR, W, H)
    assert np.array_equal(a, b), "two launches must give identical bytes"
    # the full 4K frame against the oracle (hit records and _PrimaryTriangleInfo)
    ref = rays.copy()
    info_ref = np.zeros((WH, 4), np.uint32)
    st, _ = O.trace(sc, ref, WH, 0, FAR, W, H, info=info_ref, nthreads=CPU_THREADS)
    assert st == 0
    assert np.array_equal(ref["hits"][:WH], a["hits"][:WH])
    assert np.array_equal(info_ref, info_a)
    # 8-GPU tile sharding, replayed rank by rank on this GPU: compact per-rank ray lists, traced
    # independently, reassembled on "rank 0" -> byte-identical to the single launch
    world = 8
    parts = []
    info_t = np.zeros((WH, 4), np.uint32)
    for r in range(world):
        pix = ttdist.tile_pixels(W, H, world, r)
        mine = np.zeros(2 * len(pix), tthip.RAY_DTYPE)
        mine[: len(pix)] = rays[pix]
        engine.trace(mine, len(pix), 0, FAR, W, H, info=info_t)
        parts.append(mine["hits"][: len(pix)].copy())
    full = ttdist.assemble_tiles(parts, W, H, world)
    assert np.array_equal(full, a["hits"][:WH])
    assert np.array_equal(info_t, info_a)


def test_c5_bench_frame_degenerate_ray(engine, c5):
    """bench.py's C5 frame (Generate with MaxBounce 1, frames 0) holds exactly one ray with an
    exactly-zero direction component (pixel 5,652,973: direction.x == +0, inf / NaN x slabs, 529
    node visits and 1,134 triangle tests -- profiles/r03/c5_tail/). That ray, every other ray within
    1e-6 of an axis, and a strided sample of the frame: traced on the GPU as one compacted list and by
    the oracle, byte-identical records and equal per-ray work."""
    W, H = T.C5_VIEW.width, T.C5_VIEW.height
    WH = W * H
    c2w, ip = T.C5_VIEW.camera()
    engine.upload(c5)
    rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=0, max_bounce=1)
    d = rays["direction"][:WH]
    zero = np.where((d == 0).any(axis=1))[0]
    assert zero.tolist() == [5652973] and d[5652973, 0] == 0 and not np.signbit(d[5652973, 0])
    near_axis = np.where((np.abs(d) < 1e-6).any(axis=1))[0]
    pick = np.unique(np.concatenate([near_axis, np.arange(0, WH, 101)]))
    n = len(pick)
    sub = np.zeros(2 * n, tthip.RAY_DTYPE)
    sub[:n] = rays[pick]
    rg, rc, ig, ic, s, cnt = trace_both(engine, c5, sub, n, 0, n, 1, info=False, upload=False)
    assert_same(rg, rc, ig, ic, 0, n)
    assert s.node_visits == int(cnt["node_visits"].sum()) and s.tri_tests == int(cnt["tri_tests"].sum())
    k = int(np.searchsorted(pick, 5652973))
    assert cnt["node_visits"][k] == 529 and cnt["tri_tests"][k] == 1134
