"""Two engine contexts on two streams of one GPU tracing the C2 1080p frame as two tile-interleaved
parts (bench.py's default layout), launches pipelined asynchronously (primary A,
primary B, bounce A, bounce B, several times over) so the contexts' kernels overlap. The parts'
primary hit records and _PrimaryTriangleInfo, reassembled in screen order, and their bounce-1 hit
records, matched by PixelIndex, must equal one context tracing the whole frame."""
import numpy as np
import pytest

import ttconfigs as T
import ttdist
import tthip
from parity_util import FAR

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["pool", "dedicated"])
def test_two_parts_on_two_streams_equal_one_launch(kind):
    """kind: torch pool streams, or streams on HW queues of their own (tt_stream_create, the layouts' kind)."""
    import torch

    W, H = 1920, 1080
    WH = W * H
    dev = torch.device("cuda:0")
    scene = T.c2_sponza()
    c2w, ip = T.C2_VIEW.camera(W, H)
    owned = [tthip.DedicatedStream(torch, dev) for _ in range(2)] if kind == "dedicated" else []
    streams = [d.stream for d in owned] if owned else [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    engines = [tthip.Engine(0, stream=s.cuda_stream) for s in streams]
    try:
        for e in engines:
            e.upload(scene)
        colors = np.zeros(WH, tthip.COL_DTYPE)
        colors["Data"][:, 3] = 1.0
        colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
        e0 = engines[0]
        with torch.cuda.stream(streams[0]):
            one = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            info1 = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        e0.generate(one, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        full = one[: WH * 48].clone()
        e0.trace(one, WH, 0, FAR, W, H, info=info1, device=True)
        nb1 = e0.enqueue_bounce(one, WH, 0, FAR, W, H, frames=0, max_bounce=1, device=True)
        e0.trace(one, nb1, 1, FAR, W, H, info=info1, colors=colors_t, device=True)
        torch.cuda.synchronize(dev)
        ref_prim = one.view(2 * WH, 48)[:WH, 32:48].cpu().numpy()
        ref_bnc = one.view(2 * WH, 48)[WH:WH + nb1].cpu().numpy()
        ref_info = info1.cpu().numpy()
        del one

        parts = []
        info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)  # shared: the parts' pixels are disjoint
        for s, pix_np in enumerate(ttdist.part_pixels(W, H, 1, 0, 2)):
            with torch.cuda.stream(streams[s]):
                rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            n = int(pix_np.shape[0])
            rays.view(2 * WH, 48)[:n] = full.view(WH, 48)[torch.from_numpy(pix_np).to(dev)]
            torch.cuda.synchronize(dev)
            engines[s].trace(rays, n, 0, FAR, W, H, info=info, device=True)
            nb = engines[s].enqueue_bounce(rays, n, 0, FAR, W, H, frames=0, max_bounce=1, device=True)
            parts.append((engines[s], rays, n, nb))
        torch.cuda.synchronize(dev)
        assert sum(p[3] for p in parts) == nb1
        for _ in range(3):  # pipelined, as bench.py's step
            for e, rays, n, nb in parts:
                e.trace(rays, n, 0, FAR, W, H, info=info, device=True, asynchronous=True)
            for e, rays, n, nb in parts:
                e.trace(rays, nb, 1, FAR, W, H, info=info, colors=colors_t, device=True, asynchronous=True)
        torch.cuda.synchronize(dev)

        own = np.concatenate([rays.view(2 * WH, 48)[:n, 32:48].cpu().numpy() for e, rays, n, nb in parts])
        frame = ttdist.assemble_parts([own.view(np.uint32).reshape(-1, 4)], [[p[2] for p in parts]], W, H, 1, 2)
        assert np.array_equal(frame, ref_prim.view(np.uint32).reshape(-1, 4))
        assert np.array_equal(info.cpu().numpy(), ref_info)
        # bounce-1: the parts compact their survivors in their own order; match records by PixelIndex
        got = np.concatenate([rays.view(2 * WH, 48)[WH:WH + nb].cpu().numpy() for e, rays, n, nb in parts])
        pix_of = lambda recs: recs[:, 12:16].copy().view(np.uint32)[:, 0]  # RayData.PixelIndex (bytes 12-15)
        og, orf = np.argsort(pix_of(got), kind="stable"), np.argsort(pix_of(ref_bnc), kind="stable")
        assert np.array_equal(got[og], ref_bnc[orf])
    finally:
        for e in engines:
            e.close()
        for d in owned:
            d.close()
            assert d.handle is None


def test_shared_scene_traces_identically_and_refuses_mutation(engine):
    """tt_ctx_share_scene: a context tracing another's scene buffers (no copy, its own stream) writes the
    same records as the owner (primary with info, bounce 1), sees the owner's in-place updates (a
    _MeshData rewrite + TLAS refit), and the guards hold: no scene mutation through the borrower, no
    re-upload or destroy of the lender while it lends, no sharing from a borrower."""
    import torch

    W, H = 320, 200
    WH = W * H
    dev = torch.device("cuda:0")
    sc = tthip.single_object_scene(tthip.Mesh.soup(51, 20000, 1.0, 0.1))
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.4), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, FAR)
    st_a, st_b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    lender = tthip.Engine(0, stream=st_a.cuda_stream)
    borrower = tthip.Engine(0, stream=st_b.cuda_stream)
    try:
        lender.upload(sc)
        borrower.share_scene(lender)
        base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        lender.generate(base, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=0, max_bounce=2, device=True)
        torch.cuda.synchronize(dev)

        def both(bounce, n, src):
            outs = []
            for e in (lender, borrower):
                r = src.clone()
                info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
                e.trace(r, n, bounce, FAR, W, H, info=info if bounce == 0 else None, device=True)
                outs.append((r, info))
            torch.cuda.synchronize(dev)
            assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), bounce
            return outs[0][0]

        traced = both(0, WH, base)
        nb = lender.enqueue_bounce(traced, WH, 0, FAR, W, H, frames=0, max_bounce=2, device=True)
        both(1, nb, traced)
        # an in-place update through the lender is what the borrower traces next
        md = sc.meshdata.copy()
        w2l = md["W2L"][0].astype(np.float64).reshape(4, 4).T
        shift = np.eye(4)
        shift[:3, 3] = [-0.05, 0.0, 0.02]
        md["W2L"][0] = tthip.unity_colmajor(w2l @ shift)
        lender.update_meshdata(0, md)
        torch.cuda.synchronize(dev)
        moved = both(0, WH, base)
        assert not torch.equal(moved, traced)  # the update changed the hits, on both contexts alike
        # guards
        assert borrower.L.tt_scene_update_meshdata(borrower.h, 0, 1, md.ctypes.data) == tthip.TT_ERR_INVALID_ARG
        assert lender.L.tt_scene_upload(lender.h, sc.nodes.ctypes.data, len(sc.nodes), sc.tris.ctypes.data,
                                        len(sc.tris), sc.tlas.ctypes.data, len(sc.tlas), sc.meshdata.ctypes.data,
                                        len(sc.meshdata), sc.materials.ctypes.data,
                                        len(sc.materials)) == tthip.TT_ERR_INVALID_ARG
        assert lender.L.tt_ctx_destroy(lender.h) == tthip.TT_ERR_INVALID_ARG  # still lending
        third = tthip.Engine(0)
        try:
            assert third.L.tt_ctx_share_scene(third.h, borrower.h) == tthip.TT_ERR_INVALID_ARG  # no chains
        finally:
            third.close()
    finally:
        lender.close()  # closes its borrower first
    assert borrower.h is None


def test_shared_scene_mutations_are_ordered_without_host_sync():
    """The per-frame pattern of the reference (AssetManager.cs:1821-1825: rewrite _MeshData, refit the
    TLAS, then dispatch the traces) across a lender and a borrower on two streams, with NO host
    synchronization between the calls, each stream kept busy by a queue of full-frame traces so an
    unordered call would overtake:
      * lender update_meshdata + tlas_refit, then a borrower trace -> the records of the moved scene;
      * a borrower trace, then lender update_meshdata + tlas_refit -> the records of the scene as it was
        when the trace was called.
    Expected records come from one synchronous context tracing both poses."""
    import torch

    from test_gpu_parity import refit_scene

    rng = np.random.default_rng(7)
    a = refit_scene(33)
    b = refit_scene(33, offsets=rng.normal(0, 1.5, (120, 3)))
    dev = torch.device("cuda:0")
    W, H = 160, 90
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    BW, BH = 1920, 1080  # the busy work: full-frame traces of the same scene
    bc2w, bip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, BW, BH, 0.3, FAR)
    boxes = {k: torch.from_numpy(np.ascontiguousarray(s.meta["mesh_aabbs"], np.float32)).to(dev)
             for k, s in (("a", a), ("b", b))}
    md = {"a": a.meshdata, "b": b.meshdata}

    ref = tthip.Engine(0)
    try:
        ref.upload(a)
        rays0 = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
        big = torch.zeros(2 * BW * BH * 48, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        ref.generate(rays0, c2w, ip, W, H, 0.3, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        ref.generate(big, bc2w, bip, BW, BH, 0.3, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        exp = {}
        for k in ("a", "b"):
            ref.update_meshdata(0, md[k])
            ref.tlas_refit(a.tlas_nodes, boxes[k], device=True)
            r = rays0.clone()
            torch.cuda.synchronize(dev)
            ref.trace(r, W * H, 0, FAR, W, H, device=True)
            exp[k] = r.view(-1, 48)[: W * H, 32:48].clone()
        assert not torch.equal(exp["a"], exp["b"])  # the move changes the hits
    finally:
        ref.close()

    # streams on HW queues of their own: two pool streams may share one queue, which would run the calls in
    # submission order whatever the library's events say, and let the test pass without them
    owned = [tthip.DedicatedStream(torch, dev) for _ in range(2)]
    lender = tthip.Engine(0, stream=owned[0].stream.cuda_stream)
    borrower = tthip.Engine(0, stream=owned[1].stream.cuda_stream)

    def busy(e, k=12):
        for _ in range(k):
            e.trace(big, BW * BH, 0, FAR, BW, BH, device=True, asynchronous=True)

    def pose(k, asynchronous):
        lender.update_meshdata(0, md[k])
        lender.tlas_refit(a.tlas_nodes, boxes[k], device=True, asynchronous=asynchronous)

    try:
        lender.upload(a)
        borrower.share_scene(lender)
        for rep in range(2):
            # lender mutates (behind its busy queue), then the borrower traces at once
            pose("a", False)
            r = rays0.clone()
            torch.cuda.synchronize(dev)
            busy(lender)
            pose("b", True)
            borrower.trace(r, W * H, 0, FAR, W, H, device=True, asynchronous=True)
            torch.cuda.synchronize(dev)
            assert torch.equal(r.view(-1, 48)[: W * H, 32:48], exp["b"]), ("lender -> borrower", rep)
            # the borrower traces (behind its busy queue), then the lender mutates at once
            r2 = rays0.clone()
            torch.cuda.synchronize(dev)
            busy(borrower)
            borrower.trace(r2, W * H, 0, FAR, W, H, device=True, asynchronous=True)
            pose("a", True)
            torch.cuda.synchronize(dev)
            assert torch.equal(r2.view(-1, 48)[: W * H, 32:48], exp["b"]), ("borrower -> lender", rep)
            r3 = rays0.clone()
            torch.cuda.synchronize(dev)
            borrower.trace(r3, W * H, 0, FAR, W, H, device=True)
            assert torch.equal(r3.view(-1, 48)[: W * H, 32:48], exp["a"]), ("after both", rep)
    finally:
        lender.close()
        for d in owned:
            d.close()
    assert borrower.h is None


def test_shared_scene_sections_from_two_threads():
    """The lender and a borrower driven from two host threads at once: the lender flips
    the pose (update_meshdata + a device tlas_refit, asynchronous) while the borrower issues asynchronous
    traces, none waiting on the host. The library holds the lender's mutex across each read / write
    section, so every borrower trace sees the scene between two whole calls: its records equal those of
    one of the four states the lender passes through ((_MeshData, TLAS boxes) of pose a / b: a+a, b+a after
    the records' rewrite, b+b after the refit, a+b, ...) exactly.
    The borrower records no event per launch (tt_api.hip SceneRead); the lender records one on the
    borrower's stream per mutation."""
    import threading

    import torch

    from test_gpu_parity import refit_scene

    rng = np.random.default_rng(11)
    a = refit_scene(34)
    b = refit_scene(34, offsets=rng.normal(0, 1.5, (120, 3)))
    dev = torch.device("cuda:0")
    W, H = 160, 90
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    boxes = {k: torch.from_numpy(np.ascontiguousarray(s.meta["mesh_aabbs"], np.float32)).to(dev)
             for k, s in (("a", a), ("b", b))}
    md = {"a": a.meshdata, "b": b.meshdata}
    ref = tthip.Engine(0)
    try:
        ref.upload(a)
        rays0 = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        ref.generate(rays0, c2w, ip, W, H, 0.3, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        exp = {}
        for km in ("a", "b"):
            for kb in ("a", "b"):
                ref.update_meshdata(0, md[km])
                ref.tlas_refit(a.tlas_nodes, boxes[kb], device=True)
                r = rays0.clone()
                torch.cuda.synchronize(dev)
                ref.trace(r, W * H, 0, FAR, W, H, device=True)
                exp[km + kb] = r.view(-1, 48)[: W * H, 32:48].clone()
        assert not torch.equal(exp["aa"], exp["bb"])
    finally:
        ref.close()
    owned = [tthip.DedicatedStream(torch, dev) for _ in range(2)]
    lender = tthip.Engine(0, stream=owned[0].stream.cuda_stream)
    borrower = tthip.Engine(0, stream=owned[1].stream.cuda_stream)
    n_traces = 40
    outs = [rays0.clone() for _ in range(n_traces)]
    errors = []
    try:
        lender.upload(a)
        lender.update_meshdata(0, md["a"])
        lender.tlas_refit(a.tlas_nodes, boxes["a"], device=True)
        borrower.share_scene(lender)
        torch.cuda.synchronize(dev)

        def mutate():
            try:
                for i in range(n_traces):
                    k = "b" if i % 2 == 0 else "a"
                    lender.update_meshdata(0, md[k])
                    lender.tlas_refit(a.tlas_nodes, boxes[k], device=True, asynchronous=True)
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(e)

        def trace():
            try:
                for r in outs:
                    borrower.trace(r, W * H, 0, FAR, W, H, device=True, asynchronous=True)
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        th = [threading.Thread(target=mutate), threading.Thread(target=trace)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize(dev)
        assert not errors, errors
        for i, r in enumerate(outs):
            got = r.view(-1, 48)[: W * H, 32:48]
            assert any(torch.equal(got, v) for v in exp.values()), f"trace {i} saw a torn scene"
    finally:
        lender.close()
        for d in owned:
            d.close()


def test_timing_switch():
    """tt_ctx_set_timing: off, asynchronous traces add no timing entry (no HIP-event markers); synchronous
    traces still report their kernel time; on again, asynchronous traces are timed."""
    import torch

    dev = torch.device("cuda:0")
    sc = tthip.single_object_scene(tthip.Mesh.soup(5, 4000, 1.0, 0.1))
    W, H = 128, 64
    c2w, ip = tthip.unity_camera((0.2, 0.3, 3.0), (-0.05, -0.1, -1.0), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    e = tthip.Engine(0)
    try:
        e.upload(sc)
        rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
        e.generate(rays, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        torch.cuda.synchronize(dev)
        e.timing_reset()
        e.set_timing(False)
        for _ in range(3):
            e.trace(rays, W * H, 0, FAR, W, H, device=True, asynchronous=True)
        assert len(e.timing_read()) == 0
        s = e.trace(rays, W * H, 0, FAR, W, H, device=True, stats=True)
        assert s.kernel_ms > 0 and len(e.timing_read()) == 1
        e.set_timing(True)
        e.timing_reset()
        for _ in range(3):
            e.trace(rays, W * H, 0, FAR, W, H, device=True, asynchronous=True)
        ms = e.timing_read()
        assert len(ms) == 3 and (ms > 0).all()
    finally:
        e.close()


@pytest.mark.parametrize("stride,cycle", [(0, 1), (1, 1), (1, 2)])
def test_frame_slots_equal_one_launch(stride, cycle):
    """bench.py's N = 1 layout (ttlayout.FrameLayout: the whole frame as one launch per bounce, 3 frames in
    flight on contexts that borrow one scene, streams on dedicated HW queues), several frames issued
    back to back: every slot's primary hit records and _PrimaryTriangleInfo equal one context tracing
    the frame its slot traces -- the same sample in every slot (stride 0), or slot f's own jittered sample
    f (stride 1, the bench's layout since round 5), or with cycle 2 the two samples each slot alternates
    between (bench.py --cycle at N > 1: every buffer of the cycle checked) -- and its bounce-1 records equal
    that context's bounce-1 launch."""
    import torch

    import ttlayout

    W, H = 1920, 1080
    WH = W * H
    dev = torch.device("cuda:0")
    scene = T.c2_sponza()
    c2w, ip = T.C2_VIEW.camera(W, H)
    base = tthip.Engine(0, stream=tthip.dedicated_stream(torch, dev, -1).cuda_stream)
    try:
        base.upload(scene)
        colors = np.zeros(WH, tthip.COL_DTYPE)
        colors["Data"][:, 3] = 1.0
        colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
        refs = {}
        for k in sorted({stride * (f + 3 * r) for f in range(3) for r in range(cycle)}):
            one = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            info1 = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            base.generate(one, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=k, max_bounce=1, device=True)
            base.trace(one, WH, 0, FAR, W, H, info=info1, device=True)
            torch.cuda.synchronize(dev)
            info0 = info1.cpu().numpy()  # the bounce-0 form
            info1.zero_()
            nb1 = base.enqueue_bounce(one, WH, 0, FAR, W, H, frames=k, max_bounce=1, device=True)
            base.trace(one, nb1, 1, FAR, W, H, info=info1, colors=colors_t, device=True)
            torch.cuda.synchronize(dev)
            refs[k] = (nb1, one.view(2 * WH, 48)[:WH, 32:48].cpu().numpy(),
                       one.view(2 * WH, 48)[WH:WH + nb1, 32:48].cpu().numpy(), info0, info1.cpu().numpy())
            del one
        make_full = ttlayout.full_frame_maker(torch, base, dev, W, H, c2w, ip, T.NEAR, FAR)
        lay = ttlayout.FrameLayout(torch, tthip, base, dev, W, H, FAR, [[(0, np.arange(WH, dtype=np.int64))]],
                                   make_full, slots=3, bounce=True, info=True, colors=colors_t, slot_stride=stride,
                                   cycle=cycle)
        try:
            for _ in range(6 * cycle + 1):  # asynchronous, three frames in flight; every cycle buffer traced
                lay.step()
            torch.cuda.synchronize(dev)
            for f, row in enumerate(lay.slots):
                p = row[0]
                r_last = lay.cycle_of(max(k for k in range(lay.k) if k % 3 == f))
                for r in range(cycle):
                    nb1, ref_prim, ref_bnc, ref_info0, ref_info1 = refs[lay.sample_of(f, 0, r)]
                    assert p.n == WH and p.nb_r[r] == nb1
                    prim = p.rays_r[r].view(-1, 48)[:WH, 32:48].cpu().numpy()
                    assert np.array_equal(prim, ref_prim), f"slot {f} cycle {r}: primary records"
                    bnc = p.rays_r[r].view(-1, 48)[WH:WH + nb1, 32:48].cpu().numpy()
                    assert np.array_equal(bnc, ref_bnc), f"slot {f} cycle {r}: bounce-1 records"
                    if r == r_last:
                        assert np.array_equal(lay.info0[f].cpu().numpy(), ref_info0), f"slot {f}: bounce-0 info"
                        # the bounce-1 form is written at the frame's bounce-1 pixels only (the slot's other
                        # cycle sample wrote others before): compare there
                        pix = p.rays_r[r].view(-1, 48)[WH:WH + nb1, 12:16].cpu().numpy().copy().view(np.uint32)[:, 0]
                        got1 = lay.info1[f].cpu().numpy().reshape(-1, 16)[pix]
                        assert np.array_equal(got1, ref_info1.reshape(-1, 16)[pix]), f"slot {f}: bounce-1 info"
                        if cycle == 1:
                            assert np.array_equal(lay.info1[f].cpu().numpy(), ref_info1), f"slot {f}: bounce-1 info"
            if stride:
                assert len({lay.rays_of_slot(f) for f in range(3)}) > 1  # the jitter changes the bounce counts
        finally:
            lay.close()
    finally:
        base.close()


@pytest.mark.parametrize("cycle", [1, 2])
def test_batched_frames_equal_frames_traced_alone(cycle):
    """bench.py at N > 1 (--batch, here 2): a rank's tiles as 2 parts x 3 frame slots, every launch tracing two
    frames of those tiles on a 2H-tall screen (frame j's PixelIndex + j W H, tt_ctx_set_frame_pixels(W H)).
    For every slot, cycle position and frame: the primary hit records, the bounce-1 rays (origin, direction,
    pdf -- drawn from the frame-local pixel at the frame's own sample) and their hit records, and the bounce-0
    _PrimaryTriangleInfo texels equal one context tracing the whole frame at that sample alone."""
    import torch

    import ttdist
    import ttlayout

    W, H, B, F, P = 640, 384, 2, 3, 2
    WH = W * H
    dev = torch.device("cuda:0")
    scene = T.c2_sponza()
    c2w, ip = T.C2_VIEW.camera(W, H)
    base = tthip.Engine(0, stream=tthip.dedicated_stream(torch, dev, -1).cuda_stream)
    try:
        base.upload(scene)
        colors = np.zeros(WH, tthip.COL_DTYPE)
        colors["Data"][:, 3] = 1.0
        colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
        refs = {}
        for k in range(F * cycle * B):  # every sample the layout traces: j + B (f + F r)
            one = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            info0 = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
            base.generate(one, c2w, ip, W, H, T.NEAR, FAR, jitter=1, frames=k, max_bounce=1, device=True)
            base.trace(one, WH, 0, FAR, W, H, info=info0, device=True)
            nb1 = base.enqueue_bounce(one, WH, 0, FAR, W, H, frames=k, max_bounce=1, device=True)
            base.trace(one, nb1, 1, FAR, W, H, colors=colors_t, device=True)
            torch.cuda.synchronize(dev)
            a = one.view(2 * WH, 48).cpu().numpy()
            bnc = a[WH:WH + nb1]
            refs[k] = (a[:WH, 32:48], {int(px): row for px, row in zip(bnc[:, 12:16].copy().view(np.uint32)[:, 0], bnc)},
                       info0.cpu().numpy().reshape(WH, 16))
            del one
        pix_parts = ttdist.part_pixels(W, H, 2, 0, P)
        plan = [[(b, pix) for b in range(B)] for pix in pix_parts]
        make_full = ttlayout.full_frame_maker(torch, base, dev, W, H, c2w, ip, T.NEAR, FAR)
        lay = ttlayout.FrameLayout(torch, tthip, base, dev, W, H, FAR, plan, make_full, slots=F, bounce=True,
                                   info=True, colors=colors_t, slot_stride=B, cycle=cycle, batch=B)
        try:
            for _ in range(2 * F * cycle + 1):
                lay.step()
            torch.cuda.synchronize(dev)
            for f, row in enumerate(lay.slots):
                r_last = lay.cycle_of(max(k for k in range(lay.k) if k % F == f))
                for r in range(cycle):
                    for p, pix in zip(row, pix_parts):
                        m = len(pix)
                        a = p.rays_r[r].view(-1, 48).cpu().numpy()
                        bnc = a[WH * B:WH * B + p.nb_r[r]]
                        bpi = bnc[:, 12:16].copy().view(np.uint32)[:, 0]
                        assert p.n == B * m and int(bpi.max()) < B * WH
                        for j in range(B):
                            s = lay.sample_of(f, j, r)
                            ref_prim, ref_bnc, ref_info0 = refs[s]
                            where = f"slot {f} cycle {r} frame {j} (sample {s})"
                            assert np.array_equal(a[j * m:(j + 1) * m, 32:48], ref_prim[pix]), where + ": primary records"
                            mine = bnc[(bpi >= j * WH) & (bpi < (j + 1) * WH)]
                            want = [ref_bnc[int(px)] for px in pix if int(px) in ref_bnc]
                            assert len(mine) == len(want), where + ": bounce-1 ray count"
                            mine = mine[np.argsort(mine[:, 12:16].copy().view(np.uint32)[:, 0], kind="stable")]
                            want = np.stack(want) if want else np.zeros((0, 48), np.uint8)
                            want = want[np.argsort(want[:, 12:16].copy().view(np.uint32)[:, 0], kind="stable")]
                            assert np.array_equal(mine[:, 12:16].copy().view(np.uint32)[:, 0],
                                                  want[:, 12:16].copy().view(np.uint32)[:, 0] + j * WH), where
                            assert np.array_equal(mine[:, :12], want[:, :12]), where + ": bounce-1 origins"
                            assert np.array_equal(mine[:, 16:48], want[:, 16:48]), where + ": bounce-1 rays / records"
                            if r == r_last:
                                got = lay.info0[f].cpu().numpy().reshape(B * WH, 16)[j * WH + pix]
                                assert np.array_equal(got, ref_info0[pix]), where + ": bounce-0 info"
        finally:
            lay.close()
    finally:
        base.close()


def test_enqueue_counter_blocks_survive_empty_and_indirect_calls():
    """The bounce enqueue uses two counter blocks in turn, each launch zeroing the other for the next one
    (tt_api.hip enqueue_call). Real, empty (0 rays), indirect (device count) and real calls in a mixed sequence
    on one context must each return the count and the records of a fresh context's single enqueue."""
    import torch

    dev = torch.device("cuda:0")
    sc = tthip.single_object_scene(tthip.Mesh.soup(9, 8000, 1.0, 0.1))
    W, H = 160, 96
    WH = W * H
    c2w, ip = tthip.unity_camera((0.2, 0.3, 3.0), (-0.05, -0.1, -1.0), (0, 1, 0), 55.0, W, H, 0.05, FAR)

    def primary(e, frame):
        r = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        e.generate(r, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=frame, max_bounce=2, device=True)
        e.trace(r, WH, 0, FAR, W, H, device=True)
        return r

    ref = tthip.Engine(0)
    want = {}
    try:
        ref.upload(sc)
        for frame in (0, 1, 2):
            r = primary(ref, frame)
            nb = ref.enqueue_bounce(r, WH, 0, FAR, W, H, frames=frame, max_bounce=2, device=True)
            want[frame] = (nb, r.view(-1, 48)[WH:WH + nb].cpu().numpy())
    finally:
        ref.close()
    e = tthip.Engine(0)
    try:
        e.upload(sc)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        seq = [("real", 0), ("empty", None), ("real", 1), ("empty", None), ("empty", None), ("indirect", 2),
               ("real", 0), ("indirect", 1), ("real", 2)]
        for kind, frame in seq:
            if kind == "empty":
                r = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
                assert e.enqueue_bounce(r, 0, 0, FAR, W, H, frames=0, max_bounce=2, device=True) == 0
                continue
            r = primary(e, frame)
            if kind == "real":
                nb = e.enqueue_bounce(r, WH, 0, FAR, W, H, frames=frame, max_bounce=2, device=True)
            else:
                e.enqueue_bounce_indirect(r, None, WH, cnt, 0, FAR, W, H, frames=frame, max_bounce=2)
                torch.cuda.synchronize(dev)
                nb = int(cnt.item())
            assert nb == want[frame][0], (kind, frame)
            assert np.array_equal(r.view(-1, 48)[WH:WH + nb].cpu().numpy(), want[frame][1]), (kind, frame)
    finally:
        e.close()
