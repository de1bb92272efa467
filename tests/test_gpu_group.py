"""The multi-GPU group behind the C ABI (tt_group_*, csrc/tt_group.hip) against the oracle and
the single-device path.

A group traces a frame tile-sharded over its members and gathers the primary hit records to rank 0 in screen
order; each member continues its own rays with bounce 1. On this one-GPU pool a group has either one RCCL member
(ncclCommInitAll over device 0, or ncclCommInitRank at world 1: the RCCL gather then is rank 0's send to itself)
or several members sharing device 0 with the copy gather (TT_GROUP_COPY_GATHER): the shard, trace, gather and
scatter code is the one a node of 8 MI355X runs.

Bar: the gathered frame is bit-identical to the oracle's Generate + trace of the whole frame (and to the
engine's own tt_generate_primary + tt_trace_closest); every member's bounce-1 rays and records are bit-identical
to the oracle's enqueue + trace over that member's own ray list (tt_group_tile_pixels order).
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ctypes as O
import tthip

from parity_util import CPU_THREADS, FAR

pytestmark = pytest.mark.gpu

NEAR = 0.05


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch


def _hip():
    # torch's own HIP runtime (same soname): copies of raw device pointers the group hands out
    L = C.CDLL("libamdhip64.so.7")
    L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    return L


def device_rays(ptr: int, n: int) -> np.ndarray:
    out = np.zeros(n, tthip.RAY_DTYPE)
    if n:
        assert _hip().hipMemcpy(out.ctypes.data, ptr, 48 * n, 2) == 0  # hipMemcpyDeviceToHost
    return out


@pytest.fixture(scope="module")
def soup():
    return tthip.single_object_scene(tthip.Mesh.soup(11, 40000, 1.0, 0.07))


def soup_camera(W, H):
    return tthip.unity_camera((0.3, 0.2, 2.6), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, NEAR, FAR)


def oracle_frame(sc, c2w, ip, W, H, frames, max_bounce=1, info=None):
    """The oracle's whole frame: Generate (jittered at `frames`) and the primary trace (with _PrimaryTriangleInfo
    into `info` when given); returns the rays."""
    rays = O.generate(c2w, ip, W, H, NEAR, FAR, jitter=1, frames=frames, max_bounce=max_bounce)
    assert O.trace(sc, rays, W * H, 0, FAR, W, H, info=info, nthreads=CPU_THREADS)[0] == 0
    return rays


def oracle_member(sc, full, pix, W, H, frames, max_bounce=1):
    """The oracle's view of one member: its primary rays (the frame's rays at its pixels, in its order, hits
    included), the enqueue of their bounce-1 rays at [W*H, + nb) and the bounce-1 trace. Returns (rays, nb)."""
    n = len(pix)
    r = np.zeros(W * H + n, tthip.RAY_DTYPE)
    r[:n] = full[pix.astype(np.int64)]
    nb = O.enqueue_bounce(sc, r, n, 0, FAR, W, H, frames=frames, max_bounce=max_bounce)
    assert O.trace(sc, r, nb, 1, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
    return r, nb


def check_members(g, sc, full, W, H, frames, world):
    for m in range(g.local_members()):
        n, nb, ptr = g.frame_rays(m)
        pix = tthip.group_tile_pixels(W, H, world, m)
        assert n == len(pix)
        got = device_rays(ptr, W * H + n)
        ref, nb_ref = oracle_member(sc, full, pix, W, H, frames)
        assert nb == nb_ref, (m, nb, nb_ref)
        assert np.array_equal(got[:n].view(np.uint8), ref[:n].view(np.uint8)), f"member {m}: primary rays"
        assert np.array_equal(got[W * H:W * H + nb].view(np.uint8), ref[W * H:W * H + nb].view(np.uint8)), \
            f"member {m}: bounce-1 rays / records"


def test_copy_gather_three_members_equal_the_oracle_frame(soup):
    """3 members on device 0 (copy gather), a screen that is no multiple of the tile: the gathered frame (hit
    records and _PrimaryTriangleInfo, TT_GROUP_INFO) and every member's bounce chain against the oracle."""
    torch = _torch()
    W, H, frames = 328, 200, 5
    c2w, ip = soup_camera(W, H)
    g = tthip.Group(W, H, devices=[0, 0, 0], bounce=True, copy=True, info=True)
    try:
        g.upload(soup)
        hits = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        info = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        g.trace_frame(hits, c2w, ip, NEAR, FAR, jitter=1, frames=frames, max_bounce=1, info_out=info)
        info_ref = np.full((W * H, 4), 0xA5A5A5A5, np.uint32)
        full = oracle_frame(soup, c2w, ip, W, H, frames, info=info_ref)
        got = hits.cpu().numpy().view(np.uint32)
        assert int((full["hits"][:W * H, 1] != 0xFFFFFFFF).sum()) > W * H // 4
        assert np.array_equal(got, full["hits"][:W * H]), "gathered screen-order records"
        assert np.array_equal(info.cpu().numpy().view(np.uint32), info_ref), "gathered _PrimaryTriangleInfo"
        check_members(g, soup, full, W, H, frames, 3)
    finally:
        g.close()


@pytest.mark.parametrize("gather", [False, True], ids=["direct", "forced_gather"])
def test_one_member_rccl_group_equals_the_single_launch(engine, soup, gather, monkeypatch):
    """A one-device RCCL group (ncclCommInitAll over device 0): the frame equals tt_generate_primary +
    tt_trace_closest on one context, and the member's bounce chain the engine's -- traced straight into hits_out
    (a one-rank group's path), and through the gather (rank 0's send to itself) + scatter with
    TT_GROUP_FORCE_GATHER."""
    torch = _torch()
    if gather:
        monkeypatch.setenv("TT_GROUP_FORCE_GATHER", "1")
    W, H, frames = 320, 192, 2
    c2w, ip = soup_camera(W, H)
    g = tthip.Group(W, H, devices=[0], bounce=True)
    try:
        g.upload(soup)
        hits = torch.zeros((W * H, 4), dtype=torch.int32, device="cuda:0")
        g.trace_frame(hits, c2w, ip, NEAR, FAR, jitter=1, frames=frames, max_bounce=1)
        engine.upload(soup)
        rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
        engine.generate(rays, c2w, ip, W, H, NEAR, FAR, jitter=1, frames=frames, max_bounce=1)
        engine.trace(rays, W * H, 0, FAR, W, H)
        assert np.array_equal(hits.cpu().numpy().view(np.uint32), rays["hits"][:W * H])
        nb = engine.enqueue_bounce(rays, W * H, 0, FAR, W, H, frames=frames, max_bounce=1)
        engine.trace(rays, nb, 1, FAR, W, H)
        n, nb_g, ptr = g.frame_rays(0)
        assert (n, nb_g) == (W * H, nb)
        got = device_rays(ptr, W * H + n)
        assert np.array_equal(got[:W * H + nb].view(np.uint8), rays[:W * H + nb].view(np.uint8))
        full = oracle_frame(soup, c2w, ip, W, H, frames)
        check_members(g, soup, full, W, H, frames, 1)
    finally:
        g.close()


@pytest.mark.parametrize("gather", [False, True], ids=["direct", "forced_gather"])
def test_rank_mode_world_one(soup, gather, monkeypatch):
    """tt_group_unique_id + tt_group_create_rank (the one-process-per-GPU shape bench.py uses) at world 1."""
    torch = _torch()
    if gather:
        monkeypatch.setenv("TT_GROUP_FORCE_GATHER", "1")
    W, H, frames = 256, 128, 0
    c2w, ip = soup_camera(W, H)
    g = tthip.Group(W, H, rank=0, world=1, uid=tthip.group_unique_id(), device=0)
    try:
        g.upload(soup)
        hits = torch.zeros((W * H, 4), dtype=torch.int32, device="cuda:0")
        g.trace_frame(hits, c2w, ip, NEAR, FAR, jitter=1, frames=frames)
        full = oracle_frame(soup, c2w, ip, W, H, frames)
        assert np.array_equal(hits.cpu().numpy().view(np.uint32), full["hits"][:W * H])
        assert g.frame_rays(0)[1] == 0  # no TT_GROUP_BOUNCE
    finally:
        g.close()


def test_asynchronous_frames_over_slots(soup):
    """Seven asynchronous frames over 3 slots and 2 members (each frame its own jitter and output buffer): after
    one tt_group_sync every frame's records equal the oracle's frame."""
    torch = _torch()
    W, H = 192, 128
    c2w, ip = soup_camera(W, H)
    g = tthip.Group(W, H, devices=[0, 0], slots=3, bounce=True, copy=True)
    try:
        g.upload(soup)
        outs = [torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0") for _ in range(7)]
        for k, o in enumerate(outs):
            g.trace_frame(o, c2w, ip, NEAR, FAR, jitter=1, frames=k, asynchronous=True)
        g.sync()
        for k, o in enumerate(outs):
            full = oracle_frame(soup, c2w, ip, W, H, k)
            assert np.array_equal(o.cpu().numpy().view(np.uint32), full["hits"][:W * H]), k
        check_members(g, soup, oracle_frame(soup, c2w, ip, W, H, 6), W, H, 6, 2)  # the latest frame's chains
    finally:
        g.close()


def test_sponza_1080p_eight_members_copy_gather(sponza_scene):
    """C2's scene at 1920x1080 dealt over 8 members (as on an 8-GPU node, here all on device 0): the gathered frame
    equals the oracle's, and two members' bounce chains (the first and last rank) too."""
    torch = _torch()
    W, H, frames = 1920, 1080, 1
    c2w, ip = tthip.unity_camera((-10, 2, 0), (1, 0, 0), (0, 1, 0), 60, W, H, 0.3, FAR)
    g = tthip.Group(W, H, devices=[0] * 8, bounce=True, copy=True, info=True)
    try:
        g.upload(sponza_scene)
        hits = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        info = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        cam = dict(jitter=1, frames=frames, max_bounce=1)
        g.trace_frame(hits, c2w, ip, 0.3, FAR, info_out=info, **cam)
        full = O.generate(c2w, ip, W, H, 0.3, FAR, **cam)
        info_ref = np.zeros((W * H, 4), np.uint32)
        assert O.trace(sponza_scene, full, W * H, 0, FAR, W, H, info=info_ref, nthreads=CPU_THREADS)[0] == 0
        assert np.array_equal(hits.cpu().numpy().view(np.uint32), full["hits"][:W * H])
        assert np.array_equal(info.cpu().numpy().view(np.uint32), info_ref)
        for m in (0, 7):
            n, nb, ptr = g.frame_rays(m)
            pix = tthip.group_tile_pixels(W, H, 8, m)
            got = device_rays(ptr, W * H + n)
            r = np.zeros(W * H + n, tthip.RAY_DTYPE)
            r[:n] = full[pix.astype(np.int64)]
            nb_ref = O.enqueue_bounce(sponza_scene, r, n, 0, FAR, W, H, frames=frames, max_bounce=1)
            assert O.trace(sponza_scene, r, nb_ref, 1, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
            assert nb == nb_ref and nb > 0.9 * n
            assert np.array_equal(got[:n].view(np.uint8), r[:n].view(np.uint8))
            assert np.array_equal(got[W * H:W * H + nb].view(np.uint8), r[W * H:W * H + nb].view(np.uint8))
    finally:
        g.close()


@pytest.fixture(scope="module")
def sponza_scene():
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.sponza()), None, np.zeros(7, tthip.MAT_DTYPE))
    return am.build()


def test_group_refusals(soup):
    torch = _torch()
    L = tthip._group_lib()
    cfg = tthip.GroupConfig(width=64, height=64)
    h = C.c_void_p()
    devs = np.zeros(2, np.int32)
    # RCCL takes one rank per device: two members on device 0 need the copy gather
    assert L.tt_group_create(devs.ctypes.data, 2, C.byref(cfg), C.byref(h)) == tthip.TT_ERR_INVALID_ARG
    bad = tthip.GroupConfig(width=64, height=64, tile=12)
    assert L.tt_group_create(devs.ctypes.data, 1, C.byref(bad), C.byref(h)) == tthip.TT_ERR_INVALID_ARG
    g = tthip.Group(64, 64, devices=[0, 0], copy=True)
    try:
        c2w, ip = soup_camera(64, 64)
        hits = torch.zeros((64 * 64, 4), dtype=torch.int32, device="cuda:0")
        with pytest.raises(tthip.TTError) as e:  # no scene yet
            g.trace_frame(hits, c2w, ip, NEAR, FAR)
        assert e.value.status == tthip.TT_ERR_NO_SCENE
        g.upload(soup)
        host = np.zeros((64 * 64, 4), np.uint32)
        with pytest.raises(tthip.TTError) as e:  # a host hits_out needs a synchronous frame
            g.trace_frame(host, c2w, ip, NEAR, FAR, asynchronous=True)
        assert e.value.status == tthip.TT_ERR_INVALID_ARG
        g.trace_frame(host, c2w, ip, NEAR, FAR, jitter=1, frames=2)  # staged on device 0, copied back
        assert np.array_equal(host, oracle_frame(soup, c2w, ip, 64, 64, 2)["hits"][:64 * 64])
    finally:
        g.close()
    # TT_GROUP_INFO into host arrays (staged) and its refusals: info_out missing, or not hits_out's kind of memory
    g = tthip.Group(64, 64, devices=[0, 0], copy=True, info=True)
    try:
        g.upload(soup)
        host, hinfo = np.zeros((64 * 64, 4), np.uint32), np.zeros((64 * 64, 4), np.uint32)
        with pytest.raises(tthip.TTError):
            g.trace_frame(host, c2w, ip, NEAR, FAR)
        with pytest.raises(tthip.TTError):
            g.trace_frame(host, c2w, ip, NEAR, FAR, info_out=torch.zeros((64 * 64, 4), dtype=torch.int32, device="cuda:0"))
        g.trace_frame(host, c2w, ip, NEAR, FAR, jitter=1, frames=3, info_out=hinfo)
        iref = np.zeros((64 * 64, 4), np.uint32)
        assert np.array_equal(host, oracle_frame(soup, c2w, ip, 64, 64, 3, info=iref)["hits"][:64 * 64])
        assert np.array_equal(hinfo, iref)
        cam = tthip.Camera()
        cam.width, cam.height, cam.far_plane = 32, 64, FAR  # not the group's screen
        assert L.tt_group_trace_frame(g.h, C.byref(cam), hits.data_ptr(), None, 0) == tthip.TT_ERR_INVALID_ARG
        dinfo = torch.zeros((64 * 64, 4), dtype=torch.int32, device="cuda:0")
        g.trace_frame(hits, c2w, ip, NEAR, FAR, info_out=dinfo)  # still usable after refusals
    finally:
        g.close()


def test_per_frame_scene_updates_reach_every_member():
    """A dynamic two-level scene through the group: frame 0, then every instance moved (tt_group_scene_update_meshdata
    + tt_group_tlas_refit, AssetManager.cs:1767-1826 on every device) and frame 1 issued with no synchronisation in
    between (2 slots, 3 members, copy gather): each frame's gathered records equal the oracle's on the scene as it
    was when the frame was issued (the refit TLAS read back from a member, the moved _MeshData)."""
    torch = _torch()
    from test_gpu_parity import instanced_scene

    sc = instanced_scene(17, n_props=4, n_inst=40)
    W, H = 160, 96
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, NEAR, FAR)
    g = tthip.Group(W, H, devices=[0, 0, 0], slots=2, copy=True)
    try:
        g.upload(sc)
        o0 = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        o1 = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
        g.trace_frame(o0, c2w, ip, NEAR, FAR, jitter=1, frames=0, asynchronous=True)
        rng = np.random.default_rng(17)
        md = sc.meshdata.copy()
        box = np.ascontiguousarray(sc.meta["mesh_aabbs"], np.float32).copy()
        for i in range(1, len(md)):
            d = rng.normal(0, 2.0, 3)
            w2l = md["W2L"][i].astype(np.float64).reshape(4, 4).T
            sh = np.eye(4)
            sh[:3, 3] = -d
            md["W2L"][i] = tthip.unity_colmajor(w2l @ sh)
            box[i, 0:3] += d.astype(np.float32)
            box[i, 3:6] += d.astype(np.float32)
        g.update_meshdata(0, md)
        g.tlas_refit(sc.tlas_nodes, box, asynchronous=True)
        g.trace_frame(o1, c2w, ip, NEAR, FAR, jitter=1, frames=1, asynchronous=True)
        g.sync()
        L = tthip.hip_lib()
        nodes = sc.nodes.copy()
        tl = np.zeros(sc.tlas_nodes, tthip.NODE_DTYPE)
        assert L.tt_scene_read_nodes(g.member_ctx(2), 0, sc.tlas_nodes, tl.ctypes.data) == tthip.TT_OK
        nodes[: sc.tlas_nodes] = tl
        moved = tthip.Scene(nodes, sc.tris, sc.tlas, md, sc.materials, tlas_nodes=sc.tlas_nodes)
        f0 = oracle_frame(sc, c2w, ip, W, H, 0)
        f1 = oracle_frame(moved, c2w, ip, W, H, 1)
        assert np.array_equal(o0.cpu().numpy().view(np.uint32), f0["hits"][:W * H]), "frame 0: the scene before"
        assert np.array_equal(o1.cpu().numpy().view(np.uint32), f1["hits"][:W * H]), "frame 1: the moved scene"
        still = oracle_frame(sc, c2w, ip, W, H, 1)  # frame 1's rays on the scene before the move
        assert not np.array_equal(still["hits"][:W * H], f1["hits"][:W * H])  # the move is visible
    finally:
        g.close()


def test_group_create_destroy_releases_everything(soup):
    """Groups made and destroyed repeatedly (copy and RCCL forms, several slot counts) leave no library stream
    behind (each member's slot streams and its communication stream are tt_stream_create streams) and a group
    made afterwards still traces correctly."""
    torch = _torch()
    L = tthip.hip_lib()
    base = L.tt_stream_live_count()
    for k, (members, slots, copy) in enumerate([(1, 1, False), (2, 2, True), (3, 3, True), (1, 4, False)]):
        g = tthip.Group(64, 64, devices=[0] * members, slots=slots, copy=copy)
        assert L.tt_stream_live_count() == base + members * (slots + 1)  # slot streams + the communication stream
        if k == 3:
            g.upload(soup)
        g.close()
        assert L.tt_stream_live_count() == base
    c2w, ip = soup_camera(64, 64)
    g = tthip.Group(64, 64, devices=[0, 0], copy=True)
    try:
        g.upload(soup)
        out = torch.zeros((64 * 64, 4), dtype=torch.int32, device="cuda:0")
        g.trace_frame(out, c2w, ip, NEAR, FAR, jitter=1, frames=4)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle_frame(soup, c2w, ip, 64, 64, 4)["hits"][:64 * 64])
    finally:
        g.close()


def test_batched_group_frames_equal_the_oracle_frames(soup):
    """tt_group_config.batch = 3: each call traces frames f .. f + 2 of one camera as one 3-frames-tall screen (3
    members, copy gather, bounce 1 and _PrimaryTriangleInfo). Frame b's gathered records and info texels (at
    [b W H, (b + 1) W H)) equal the oracle's frame f + b traced alone; every member's primary rays are its pixels'
    rays of each frame (PixelIndex + b W H) and its bounce-1 rays and records are the oracle's per-frame enqueue +
    trace over its own rays at f + b, frame after frame (the enqueue keyed on the frame-local pixel)."""
    torch = _torch()
    W, H, B, f0, members = 200, 136, 3, 7, 3
    WH = W * H
    c2w, ip = soup_camera(W, H)
    g = tthip.Group(W, H, devices=[0] * members, bounce=True, copy=True, info=True, batch=B, slots=2)
    try:
        g.upload(soup)
        hits = torch.full((B * WH, 4), -1, dtype=torch.int32, device="cuda:0")
        info = torch.full((B * WH, 4), -1, dtype=torch.int32, device="cuda:0")
        g.trace_frame(hits, c2w, ip, NEAR, FAR, jitter=1, frames=f0, max_bounce=1, info_out=info)
        got_h, got_i = hits.cpu().numpy().view(np.uint32), info.cpu().numpy().view(np.uint32)
        fulls = []
        for b in range(B):
            iref = np.full((WH, 4), 0xA5A5A5A5, np.uint32)
            full = oracle_frame(soup, c2w, ip, W, H, f0 + b, info=iref)
            fulls.append(full)
            assert np.array_equal(got_h[b * WH:(b + 1) * WH], full["hits"][:WH]), f"frame {b}: records"
            assert np.array_equal(got_i[b * WH:(b + 1) * WH], iref), f"frame {b}: _PrimaryTriangleInfo"
        for m in range(members):
            n_all, nb, ptr = g.frame_rays(m)
            pix = tthip.group_tile_pixels(W, H, members, m).astype(np.int64)
            n = len(pix)
            assert n_all == B * n
            got = device_rays(ptr, B * WH + B * n)
            off = B * WH
            for b in range(B):
                ref_p = fulls[b][pix].copy()
                ref_p["PixelIndex"] += np.uint32(b * WH)
                assert np.array_equal(got[b * n:(b + 1) * n].view(np.uint8), ref_p.view(np.uint8)), (m, b, "primary")
                ref, nb_b = oracle_member(soup, fulls[b], pix, W, H, f0 + b)
                ref_b = ref[WH:WH + nb_b].copy()
                ref_b["PixelIndex"] += np.uint32(b * WH)
                assert np.array_equal(got[off:off + nb_b].view(np.uint8), ref_b.view(np.uint8)), (m, b, "bounce 1")
                off += nb_b
            assert off == B * WH + nb
    finally:
        g.close()


def test_one_rank_direct_path_batched_info_host_outputs(soup, monkeypatch):
    """A one-rank group traces straight into the caller's outputs: two frames per call with _PrimaryTriangleInfo,
    into host arrays (the staging path) and into device tensors, equal to the same group forced through the
    gather + scatter and to the oracle's frames."""
    torch = _torch()
    W, H, B, f0 = 200, 120, 2, 3
    c2w, ip = soup_camera(W, H)
    outs = {}
    for mode in ("direct", "gather"):
        if mode == "gather":
            monkeypatch.setenv("TT_GROUP_FORCE_GATHER", "1")
        g = tthip.Group(W, H, devices=[0], bounce=True, info=True, batch=B)
        try:
            g.upload(soup)
            hh = np.full((B * W * H, 4), 0xA5A5A5A5, np.uint32)
            hi = np.full((B * W * H, 4), 0xA5A5A5A5, np.uint32)
            g.trace_frame(hh, c2w, ip, NEAR, FAR, jitter=1, frames=f0, max_bounce=1, info_out=hi)
            dh = torch.full((B * W * H, 4), -1, dtype=torch.int32, device="cuda:0")
            di = torch.full((B * W * H, 4), -1, dtype=torch.int32, device="cuda:0")
            g.trace_frame(dh, c2w, ip, NEAR, FAR, jitter=1, frames=f0, max_bounce=1, info_out=di)
            assert np.array_equal(dh.cpu().numpy().view(np.uint32), hh)
            assert np.array_equal(di.cpu().numpy().view(np.uint32), hi)
            outs[mode] = (hh, hi)
        finally:
            g.close()
    assert np.array_equal(outs["direct"][0], outs["gather"][0]) and np.array_equal(outs["direct"][1], outs["gather"][1])
    for b in range(B):
        info_ref = np.full((W * H, 4), 0xA5A5A5A5, np.uint32)
        full = oracle_frame(soup, c2w, ip, W, H, f0 + b, info=info_ref)
        assert np.array_equal(outs["direct"][0][b * W * H:(b + 1) * W * H], full["hits"][:W * H]), b
        assert np.array_equal(outs["direct"][1][b * W * H:(b + 1) * W * H], info_ref), b
