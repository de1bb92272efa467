"""Scheduling and output forms of the closest-hit launch that must not change what it computes.

TT_TRACE_ADAPTIVE_ORDER (csrc/tt_order.hip): a flagged launch records per-64-ray-chunk costs, the
next flagged launch of the same bounce index dequeues its chunks longest-first. Only which lane
traces which ray changes, so every flagged launch must be byte-identical to the unflagged one (which
the parity suites pin against the oracle). Every record's hit fields start as a sentinel, so a ray
the reordered dequeue skipped would show. Covered: the full-frame 8x8 tile swizzle and compacted
lists; ragged counts (the partial last chunk must stay last); counts below one chunk per segment; a
screen-size change (costs dropped); the material-check kernel form; _PrimaryTriangleInfo at bounce 0
and the GlobalColors-gated form at bounce 1; C2 at 1080p (primary + its compacted bounce-1 rays).

tt_trace_closest_hits: the compact hit-record stream the multi-GPU gather sends."""
import numpy as np
import pytest

import ttconfigs as T
import tthip
from parity_util import FAR

pytestmark = pytest.mark.gpu
ORD = tthip.TT_TRACE_ADAPTIVE_ORDER


def _sentinel(rays_t):
    """uint8 device view of RayData[]: every hits field set to 0xFFFFFFFF."""
    v = rays_t.view(-1, 48)
    v[:, 32:48] = 255
    return rays_t


def _run(engine, base, n, bounce, W, H, flags, colors=None):
    import torch

    t = _sentinel(base.clone())
    info = torch.zeros(W * H * 16, dtype=torch.uint8, device=base.device)
    engine.trace(t, n, bounce, FAR, W, H, info=info, colors=colors, device=True, flags=flags)
    torch.cuda.synchronize()
    return t, info


def _check_order_invariance(engine, base, n, bounce, W, H, extra=0, colors=None, repeats=3):
    import torch

    ref, ref_info = _run(engine, base, n, bounce, W, H, extra, colors)
    for k in range(repeats):  # k = 0 records costs (natural order), k >= 1 dequeue in the sorted order
        got, got_info = _run(engine, base, n, bounce, W, H, extra | ORD, colors)
        assert torch.equal(got, ref), (n, bounce, k)
        assert torch.equal(got_info, ref_info), (n, bounce, k)


def _soup_frame(engine, W, H, seed=41, frames=0):
    import torch

    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, 30000, 1.0, 0.1))
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.4), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, FAR)
    engine.upload(sc)
    base = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=torch.device("cuda:0"))
    engine.generate(base, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=frames, max_bounce=2, device=True)
    return base


def test_adaptive_order_full_frame_and_ragged(engine):
    W, H = 256, 160
    WH = W * H
    base = _soup_frame(engine, W, H)
    # full frame (8x8 tile swizzle), then compacted-list forms: ragged, tiny, one ray
    for n in (WH, WH - 1, 4097, 1000, 63, 1):
        _check_order_invariance(engine, base, n, 0, W, H)
    # the material-check kernel form (IgnoreBackfacing at bounce 0)
    _check_order_invariance(engine, base, WH, 0, W, H, extra=tthip.TT_TRACE_IGNORE_BACKFACING)
    _check_order_invariance(engine, base, WH - 5, 0, W, H, extra=tthip.TT_TRACE_IGNORE_BACKFACING)


def test_adaptive_order_screen_change_and_bounce(engine):
    import torch

    # a different screen size on the same context and bounce slot: the old costs are dropped
    for W, H in ((200, 120), (120, 96), (200, 120)):
        base = _soup_frame(engine, W, H, seed=43)
        _check_order_invariance(engine, base, W * H, 0, W, H, repeats=2)
    # bounce 1 on the compacted survivors of the traced primaries (the odd-bounce half of the buffer)
    W, H = 200, 120
    base = _soup_frame(engine, W, H, seed=43, frames=2)
    engine.trace(base, W * H, 0, FAR, W, H, device=True)
    nb = engine.enqueue_bounce(base, W * H, 0, FAR, W, H, frames=2, max_bounce=2, device=True)
    assert 0 < nb < W * H
    colors = np.zeros(W * H, tthip.COL_DTYPE)
    colors["Data"][:, 3] = (np.arange(W * H) % 3) - 1.0  # every Data.w gate form
    col_t = torch.from_numpy(colors.view(np.uint8)).to(base.device)
    _check_order_invariance(engine, base, nb, 1, W, H, colors=col_t)


def test_adaptive_order_c2_1080p_primary_and_bounce(engine):
    """The bench workload: C2 at 1920x1080, the primary launch and the compacted bounce-1 launch,
    each three times with the flag (the 2nd and 3rd in the sorted order), byte-identical."""
    import torch

    W, H = 1920, 1080
    WH = W * H
    sc = T.c2_sponza()
    engine.upload(sc)
    c2w, ip = T.C2_VIEW.camera(W, H)
    base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=torch.device("cuda:0"))
    engine.generate(base, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=0, max_bounce=1, device=True)
    _check_order_invariance(engine, base, WH, 0, W, H)
    engine.trace(base, WH, 0, FAR, W, H, device=True)
    nb = engine.enqueue_bounce(base, WH, 0, FAR, W, H, frames=0, max_bounce=1, device=True)
    colors = torch.zeros(WH * 64, dtype=torch.uint8, device=base.device)
    colors.view(torch.float32).view(WH, 16)[:, 15] = -1.0  # Data.w = -1: info written for every ray
    _check_order_invariance(engine, base, nb, 1, W, H, colors=colors)


def test_hit_stream_equals_ray_records(engine):
    """tt_trace_closest_hits: hits_out[i] is ray i's RayData.hits (full frame, ragged compacted list, an
    odd bounce's offset half, the adaptive-order kernel, the wide drain), and the rest of the outputs
    equal tt_trace_closest's; refusals for host / misaligned streams."""
    import torch

    W, H = 256, 160
    WH = W * H
    base = _soup_frame(engine, W, H, seed=47, frames=1)
    dev = base.device
    cases = [(WH, 0, 0), (WH - 7, 0, 0), (4097, 0, ORD), (WH, 0, ORD)]
    for n, bounce, flags in cases:
        ref, ref_info = _run(engine, base, n, bounce, W, H, 0)
        got = _sentinel(base.clone())
        info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
        hs = torch.full((n, 4), -1, dtype=torch.int32, device=dev)
        for _ in range(2 if flags else 1):
            engine.trace(got, n, bounce, FAR, W, H, info=info, device=True, flags=flags, hits_out=hs)
        torch.cuda.synchronize()
        assert torch.equal(got, ref) and torch.equal(info, ref_info), (n, flags)
        assert torch.equal(hs, got.view(-1, 48)[:n, 32:48].contiguous().view(torch.int32)), (n, flags)
    # bounce 1: the records live in the odd half (GlobalRays[W*H + i]); hits_out is indexed from 0
    engine.trace(base, WH, 0, FAR, W, H, device=True)
    nb = engine.enqueue_bounce(base, WH, 0, FAR, W, H, frames=1, max_bounce=2, device=True)
    got = _sentinel(base.clone())
    hs = torch.full((nb, 4), -1, dtype=torch.int32, device=dev)
    engine.trace(got, nb, 1, FAR, W, H, device=True, hits_out=hs)
    torch.cuda.synchronize()
    assert torch.equal(hs, got.view(-1, 48)[WH:WH + nb, 32:48].contiguous().view(torch.int32))
    # refusals: host pointers, a misaligned stream
    host_rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    hs = torch.zeros((WH + 1, 4), dtype=torch.int32, device=dev)
    p = tthip.TraceParams(n_rays=WH, bounce=0, far_plane=FAR, screen_width=W, screen_height=H, flags=0)
    assert engine.L.tt_trace_closest_hits(engine.h, tthip.C.byref(p), host_rays.ctypes.data, None, None,
                                          hs.data_ptr()) == tthip.TT_ERR_INVALID_ARG
    assert engine.trace(got, WH, 0, FAR, W, H, device=True, hits_out=hs.view(-1)[1:], check=False)[1] \
        == tthip.TT_ERR_INVALID_ARG


def test_hit_stream_keeps_the_records_of_rays_without_one(engine):
    """A ray that ends without a record -- the Reps < 1000 bound (IntersectionKernels.compute:155) or a
    stack overflow -- leaves RayData.hits as it was, and its hits_out entry is that same unchanged word
    (not whatever the stream buffer held: the stream starts as a sentinel unlike RayData.hits).
    Reps: the C2 1080p frame with UseReCur's unjittered camera, whose column x = W/2 has direction.z ==
    -0.0 and one Reps-exhausting ray (bench.py aux_recur_unjittered); overflow: the 17-level KAT."""
    import torch

    import kat_cases as K

    dev = torch.device("cuda:0")
    W, H = 1920, 1080
    WH = W * H
    engine.upload(T.c2_sponza())
    c2w, ip = T.C2_VIEW.camera(W, H)
    base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    engine.generate(base, c2w, ip, W, H, T.NEAR, FAR, jitter=0, frames=0, max_bounce=1, device=True)
    st = engine.trace(base.clone(), WH, 0, FAR, W, H, device=True, stats=True)
    assert st.reps_exhausted >= 1
    for flags in (0, ORD, ORD):  # natural order; adaptive (records costs), adaptive (sorted order)
        got = base.clone()
        hs = torch.full((WH, 4), 0x5A5A5A5A, dtype=torch.int32, device=dev)
        engine.trace(got, WH, 0, FAR, W, H, device=True, flags=flags, hits_out=hs)
        torch.cuda.synchronize()
        assert torch.equal(hs, got.view(-1, 48)[:WH, 32:48].contiguous().view(torch.int32)), flags
    # the exhausted ray's record is the one Generate wrote (the miss record), in both outputs
    unchanged = (got.view(-1, 48)[:WH, 32:48] == base.view(-1, 48)[:WH, 32:48]).all(1)
    assert int(unchanged.sum()) >= 1
    # stack overflow: one ray, 17 nested levels
    sc, rays = K.stack_overflow_scene(17)
    engine.upload(sc)
    r = torch.from_numpy(rays.view(np.uint8).copy()).to(dev)
    hs = torch.full((1, 4), 0x5A5A5A5A, dtype=torch.int32, device=dev)
    _, code = engine.trace(r, 1, 0, FAR, 1, 1, device=True, hits_out=hs, check=False)
    torch.cuda.synchronize()
    assert code == tthip.TT_ERR_STACK_OVERFLOW
    assert torch.equal(hs, r.view(-1, 48)[:1, 32:48].contiguous().view(torch.int32))
    assert torch.equal(r, torch.from_numpy(rays.view(np.uint8).copy()).to(dev))  # RayData untouched
