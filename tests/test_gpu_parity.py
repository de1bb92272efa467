"""GPU parity: the gfx950 engine, called through the C ABI, against the CPU oracle.

The bar is bit-exact hit records (mesh_id, triangle_id, asuint(t), packed u/v) and
_PrimaryTriangleInfo for every ray; normals within 1e-5. Sizes run from single hand-built rays
(known answers) to the full BASELINE.json C2 configuration (Sponza-shaped, 1920x1080 primary
plus bounce 1), where the oracle is multithreaded.
"""
import os

import numpy as np
import pytest

import golden_io
import handbuilt as hb
import kat_cases as K
import oracle_ctypes as O
import tthip

from parity_util import CPU_THREADS, FAR, assert_same, bounce_rays, same_floats, trace_both

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ numerics contract
def test_fast_reciprocal_is_correctly_rounded_for_every_input(engine):
    """rcp() is pinned to the correctly rounded 1.0f/x; the kernels compute it as v_rcp_f32 + one FMA
    Newton step for normal inputs with a full-division fallback. Exhaustive over all 2^32 inputs."""
    assert engine.selftest_rcp() == 0


# ------------------------------------------------------------------ known answers
@pytest.mark.parametrize("case", K.ALL_CASES, ids=lambda c: c.__name__)
def test_kat_on_gpu(engine, case):
    name, sc, rays, n, expected = case()
    engine.upload(sc)
    r = rays.copy()
    engine.trace(r, n, 0, FAR, n, 1)
    assert r["hits"][:n].tolist() == [list(map(int, e)) for e in expected], name


def test_kat_stack_overflow_on_gpu(engine):
    sc, rays = K.stack_overflow_scene(17)
    engine.upload(sc)
    s, st = engine.trace(rays.copy(), 1, 0, FAR, 1, 1, check=False)
    assert st == tthip.TT_ERR_STACK_OVERFLOW and s.stack_overflows == 1
    sc, rays = K.stack_overflow_scene(16)
    engine.upload(sc)
    r = rays.copy()
    engine.trace(r, 1, 0, FAR, 1, 1)
    assert r["hits"][0, 1] == 0


def test_kat_invisible_on_gpu(engine):
    sc, rays, exp0, exp1 = K.case_invisible_bounce0()
    engine.upload(sc)
    r0 = rays.copy()
    engine.trace(r0, 1, 0, FAR, 1, 1)
    assert r0["hits"][0].tolist() == exp0
    r1 = rays.copy()
    r1[1] = r1[0]
    engine.trace(r1, 1, 1, FAR, 1, 1)
    assert r1["hits"][1].tolist() == exp1


def test_cutout_without_atlas_is_refused():
    sc, rays, _, _ = K.case_invisible_bounce0()
    sc.materials[0]["MatType"] = tthip.MAT_CUTOUT_INDEX
    fresh = tthip.Engine(0)  # no alpha atlas uploaded on this context
    fresh.upload(sc)
    s, st = fresh.trace(rays.copy(), 1, 0, FAR, 1, 1, check=False)
    assert st == tthip.TT_ERR_UNSUPPORTED


def test_cutout_wrap_and_no_texture_on_gpu(engine):
    wrap, none, rays, exp_wrap, exp_none = K.case_cutout_wrap_and_no_texture()
    for sc, exp in ((wrap, exp_wrap), (none, exp_none)):
        engine.upload(sc)
        r = rays.copy()
        engine.trace(r, 1, 0, FAR, 1, 1)
        assert r["hits"][0].tolist() == exp


def test_malformed_scene_is_refused(engine):
    sc = tthip.single_object_scene(tthip.Mesh.soup(3, 200, 1.0, 0.1))
    sc.nodes[2]["base_child"] = 10 ** 6
    with pytest.raises(tthip.TTError) as e:
        engine.upload(sc)
    assert e.value.status == tthip.TT_ERR_INVALID_ARG


def test_nan_far_plane_is_refused(engine):
    """FarPlane seeds best.t, the node test's t_max, which the kernel's clamp assumes is not a NaN:
    tt_trace_closest refuses a NaN far plane (an infinite one is traced)."""
    sc = tthip.single_object_scene(tthip.Mesh.soup(3, 200, 1.0, 0.1))
    engine.upload(sc)
    rays = np.zeros(2 * 64, tthip.RAY_DTYPE)
    rays["direction"][:, 2] = 1.0
    with pytest.raises(tthip.TTError) as e:
        engine.trace(rays, 64, 0, float("nan"), 8, 8)
    assert e.value.status == tthip.TT_ERR_INVALID_ARG
    engine.trace(rays, 64, 0, float("inf"), 8, 8)


# ------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", golden_io.NAMES)
def test_golden_on_gpu(engine, name):
    g = golden_io.load(name)
    sc, W, H = g["scene"], g["W"], g["H"]
    engine.upload(sc)
    r0 = g["rays0"].copy()
    info0 = np.zeros((W * H, 4), np.uint32)
    s = engine.trace(r0, W * H, 0, g["far"], W, H, info=info0, stats=True)
    assert np.array_equal(r0["hits"][: W * H], g["hits0"])
    assert np.array_equal(info0, g["info0"])
    c0 = g["counts0"].view(O.COUNTS_DTYPE)
    assert s.node_visits == int(c0["node_visits"].sum()) and s.tri_tests == int(c0["tri_tests"].sum())
    assert s.blas_entries == int(c0["blas_entries"].sum()) and s.accepts == int(c0["accepts"].sum())
    r1 = g["rays1"].copy()
    info1 = np.zeros((W * H, 4), np.uint32)
    engine.trace(r1, g["n1"], 1, g["far"], W, H, info=info1, colors=g["colors"])
    assert np.array_equal(r1["hits"][W * H:W * H + g["n1"]], g["hits1"])
    assert np.array_equal(info1, g["info1"])


def test_golden_device_pointers(engine):
    import torch

    g = golden_io.load("instanced")
    sc, W, H = g["scene"], g["W"], g["H"]
    engine.upload(sc)
    dev = torch.device("cuda:0")
    rt = torch.from_numpy(g["rays0"].view(np.uint8).copy()).to(dev)
    it = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    engine.trace(rt, W * H, 0, g["far"], W, H, info=it, device=True)
    r = rt.cpu().numpy().view(tthip.RAY_DTYPE)
    assert np.array_equal(r["hits"][: W * H], g["hits0"])
    assert np.array_equal(it.cpu().numpy().view(np.uint32).reshape(-1, 4), g["info0"])


def test_back_to_back_async_launches(engine):
    """A chain of asynchronous traces of different sizes on one stream (with a synchronous launch
    and a stats launch in the chain) must give every ray the record a lone launch gives: each
    launch starts from a clean control block (dequeue tickets, error counters)."""
    import torch

    sc = tthip.single_object_scene(tthip.Mesh.soup(7, 30000, 1.0, 0.08))
    W, H = 320, 200
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.6), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    engine.upload(sc)
    ref = rays.copy()
    engine.trace(ref, W * H, 0, FAR, W, H)
    dev = torch.device("cuda:0")
    sizes = [W * H, 777, W * H, W * H - 5, 64, W * H, 1, W * H]
    bufs = [torch.from_numpy(rays.view(np.uint8).copy()).to(dev) for _ in sizes]
    torch.cuda.synchronize()
    for k, (b, n) in enumerate(zip(bufs, sizes)):
        if k == 3:
            engine.trace(b, n, 0, FAR, W, H, device=True)  # synchronous, in the middle of the chain
        elif k == 5:
            engine.trace(b, n, 0, FAR, W, H, device=True, stats=True)
        else:
            engine.trace(b, n, 0, FAR, W, H, device=True, asynchronous=True)
    torch.cuda.synchronize()
    hits = int((ref["hits"][: W * H, 1] != 0xFFFFFFFF).sum())
    assert hits > W * H // 4
    for b, n in zip(bufs, sizes):
        got = b.cpu().numpy().view(tthip.RAY_DTYPE)
        assert np.array_equal(got["hits"][:n], ref["hits"][:n]), n


# ------------------------------------------------------------------ random scenes
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_random_soup_random_camera(engine, seed):
    rng = np.random.default_rng(seed)
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, int(rng.integers(500, 40000)), 1.0,
                                                   float(rng.uniform(0.02, 0.2))))
    W, H = int(rng.integers(17, 200)), int(rng.integers(9, 120))  # ragged, not multiples of 64
    pos = rng.uniform(-2.5, 2.5, 3)
    c2w, ip = tthip.unity_camera(pos, -pos + rng.normal(0, 0.3, 3), (0, 1, 0), float(rng.uniform(30, 100)), W, H,
                                 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, W * H)
    assert s.node_visits == int(cnt["node_visits"].sum())


def instanced_scene(seed, n_props=12, n_inst=200):
    rng = np.random.default_rng(seed)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(seed, 3000, 20.0, 0.5)), tthip.trs_matrix((0, 0, 0)),
                  np.zeros(2, tthip.MAT_DTYPE))
    props = [am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(seed * 100 + k, int(rng.integers(50, 4000)))),
                                    np.zeros(2, tthip.MAT_DTYPE)) for k in range(n_props)]
    for i in range(n_inst):
        am.add_instance(props[i % n_props], tthip.trs_matrix(rng.uniform(-40, 40, 3) * [1, 0.1, 1],
                                                             float(rng.uniform(0, 360)), float(rng.uniform(0.3, 2))))
    return am.build()


@pytest.mark.parametrize("seed", [5, 6])
def test_instanced_two_level(engine, seed):
    sc = instanced_scene(seed)
    W, H = 160, 90
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, W * H)
    assert s.blas_entries == int(cnt["blas_entries"].sum()) > W * H


def test_update_meshdata_and_nodes(engine):
    """Per-frame transform update (AssetManager.cs:1825) and TLAS node rewrite (:1760)."""
    sc = instanced_scene(9, n_props=3, n_inst=20)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    engine.upload(sc)
    md = sc.meshdata.copy()
    md["W2L"][1:] = tthip.unity_colmajor(np.linalg.inv(tthip.trs_matrix((1.0, 0, 0), 5.0, 1.1)))
    engine.update_meshdata(0, md)
    sc2 = tthip.Scene(sc.nodes, sc.tris, sc.tlas, md, sc.materials)
    rg, rc, ig, ic, _, _ = trace_both(engine, sc2, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)
    nodes = sc.nodes.copy()
    nodes[0]["p"] = nodes[0]["p"] - 1.0  # a (conservatively wrong) refit of the TLAS root
    engine.update_nodes(0, nodes[:1])
    sc3 = tthip.Scene(nodes, sc.tris, sc.tlas, md, sc.materials)
    rg, rc, ig, ic, _, _ = trace_both(engine, sc3, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)
    bad = nodes[:1].copy()
    bad[0]["base_child"] = 10 ** 7
    with pytest.raises(tthip.TTError):
        engine.update_nodes(0, bad)


def test_incremental_async_updates(engine):
    """The per-frame update paths are incremental and asynchronous (no host sync): a sub-range of
    _MeshData records (the caller's buffer overwritten right after the call: the library staged
    it), back-to-back updates (pinned staging slots reused), a record re-pointed at another
    validated BLAS, a rejected record (out-of-range BLAS: nothing changes), a BLAS-node rewrite
    (full validation) -- every state traced against the oracle on the same buffers."""
    sc = instanced_scene(11, n_props=4, n_inst=30)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    engine.upload(sc)
    md = sc.meshdata.copy()
    rng = np.random.default_rng(11)
    for step in range(3):  # three updates back to back, no trace or sync between them
        buf = md.copy()
        for i in range(5, 17):
            buf["W2L"][i] = tthip.unity_colmajor(np.linalg.inv(tthip.trs_matrix(
                rng.uniform(-30, 30, 3) * [1, 0.1, 1], float(rng.uniform(0, 360)), float(rng.uniform(0.5, 1.5)))))
        engine.update_meshdata(5, buf[5:17])
        md[5:17] = buf[5:17]
        buf["W2L"][:] = np.nan  # the caller reuses its buffer at once
    sc2 = tthip.Scene(sc.nodes, sc.tris, sc.tlas, md, sc.materials)
    rg, rc, ig, ic, _, _ = trace_both(engine, sc2, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)
    # re-point instance 3 at the BLAS of instance 4 (validated at upload)
    if (md["NodeOffset"][3], md["TriOffset"][3]) == (md["NodeOffset"][4], md["TriOffset"][4]):
        j = next(k for k in range(5, len(md)) if md["NodeOffset"][k] != md["NodeOffset"][3])
    else:
        j = 4
    rec = md[3:4].copy()
    for f in ("NodeOffset", "TriOffset", "mesh_data_bvh_offsets"):
        rec[f] = md[f][j]
    engine.update_meshdata(3, rec)
    md[3:4] = rec
    # a record naming an out-of-range BLAS root is refused and changes nothing
    bad = md[6:7].copy()
    bad["mesh_data_bvh_offsets"] = len(sc.nodes) + 5
    bad["W2L"][:] = 0.0
    with pytest.raises(tthip.TTError):
        engine.update_meshdata(6, bad)
    sc3 = tthip.Scene(sc.nodes, sc.tris, sc.tlas, md, sc.materials)
    rg, rc, ig, ic, _, _ = trace_both(engine, sc3, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)
    # a BLAS node (outside the TLAS) rewritten: the root of instance 5's BLAS grown conservatively
    nodes = sc.nodes.copy()
    r5 = int(md["mesh_data_bvh_offsets"][5]) & 0x7FFFFFFF
    nodes[r5]["p"] = nodes[r5]["p"] - 0.25
    engine.update_nodes(r5, nodes[r5:r5 + 1])
    sc4 = tthip.Scene(nodes, sc.tris, sc.tlas, md, sc.materials)
    rg, rc, ig, ic, _, _ = trace_both(engine, sc4, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)


def test_info_forms_at_later_bounce(engine):
    g = golden_io.load("soup")
    sc, W, H = g["scene"], g["W"], g["H"]
    for flags in (0, tthip.TT_TRACE_USE_RESTIRGI, tthip.TT_TRACE_USE_ASVGF,
                  tthip.TT_TRACE_USE_RESTIRGI | tthip.TT_TRACE_USE_ASVGF):
        for bounce in (1, 2, 3):
            rays = g["rays1"].copy()
            if bounce % 2 == 0:  # even bounces read the first half of the ping-pong buffer
                rays[: W * H] = rays[W * H:]
            off = W * H if bounce % 2 else 0
            colors = g["colors"].copy()
            colors["Data"][:, 3] = np.where(np.arange(W * H) % 2 == 0, float(bounce), -1.0)
            rg, rc, ig, ic, _, _ = trace_both(engine, sc, rays, g["n1"], bounce, W, H, colors=colors, flags=flags)
            assert_same(rg, rc, ig, ic, off, g["n1"])


@pytest.mark.parametrize("n", [0, 1, 63, 65, 257, 4097])
def test_ragged_ray_counts(engine, n):
    g = golden_io.load("soup")
    sc, W, H = g["scene"], g["W"], g["H"]
    rng = np.random.default_rng(n)
    rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    m = min(n, W * H)
    src = g["rays0"][rng.permutation(W * H)[:m]]
    rays[:m] = src
    rg, rc, ig, ic, s, _ = trace_both(engine, sc, rays, m, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, m)
    assert s.rays == m


def test_normals_within_1e5(engine):
    sc = instanced_scene(11, n_props=4, n_inst=30)
    W, H = 128, 72
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    engine.upload(sc)
    engine.trace(rays, W * H, 0, FAR, W, H)
    ng = engine.resolve_normals(rays, W * H, 0, FAR, W, H)
    nc = O.resolve_normals(sc, rays, W * H, 0, FAR, W, H)
    hit = rays["hits"][: W * H, 1] != 0xFFFFFFFF
    assert hit.sum() > 100
    assert np.abs(ng - nc).max() <= 1e-5
    assert np.allclose(np.linalg.norm(ng[hit, :3], axis=1), 1.0, atol=1e-5)


def test_raygen_matches_restatement(engine):
    sc = tthip.single_object_scene(tthip.Mesh.cornell())
    engine.upload(sc)
    W, H = 320, 200
    c2w, ip = tthip.unity_camera((0.1, 0.2, 3.4), (0, 0, -1), (0, 1, 0), 40, W, H, 0.3, FAR)
    for jitter in (0, 1):
        rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
        engine.generate(rays, c2w, ip, W, H, 0.3, FAR, jitter=jitter, frames=3, max_bounce=5)
        ref = O.generate(c2w, ip, W, H, 0.3, FAR, jitter=jitter, frames=3, max_bounce=5)
        assert np.array_equal(rays[: W * H].view(np.uint32), ref[: W * H].view(np.uint32))


def test_bounce_enqueue_compaction(engine):
    g = golden_io.load("soup")
    sc, W, H = g["scene"], g["W"], g["H"]
    engine.upload(sc)
    r = g["rays0"].copy()
    engine.trace(r, W * H, 0, FAR, W, H)
    ref = r.copy()
    nb = engine.enqueue_bounce(r, W * H, 0, FAR, W, H)
    hit = r["hits"][: W * H, 1] != 0xFFFFFFFF
    assert nb == hit.sum()
    out = r[W * H:W * H + nb]
    # stable compaction: bit-identical to the oracle's source-order restatement
    assert O.enqueue_bounce(sc, ref, W * H, 0, FAR, W, H) == nb
    assert np.array_equal(out.view(np.uint32), ref[W * H:W * H + nb].view(np.uint32))
    assert np.allclose(np.linalg.norm(out["direction"], axis=1), 1.0, atol=1e-5)
    # the compacted bounce rays trace identically on both sides
    rg, rc, ig, ic, _, _ = trace_both(engine, sc, r, nb, 1, W, H, info=False)
    assert_same(rg, rc, ig, ic, W * H, nb)


@pytest.mark.parametrize("n", [0, 1, 63, 1023, 4095, 4096, 4097, 70001])
def test_bounce_enqueue_ragged_and_odd_bounce(engine, n):
    """Tile edges of the look-back scan (4096 rays per tile, 64-tile look-back window) and the odd-bounce
    direction (second half -> first half), bit-exact against the oracle."""
    W, H = 400, 300
    sc = tthip.single_object_scene(tthip.Mesh.soup(7, 3000))
    engine.upload(sc)
    c2w, ip = tthip.unity_camera((0.2, 0.1, 3.0), (0, 0, -1), (0, 1, 0), 50, W, H, 0.3, FAR)
    r = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    engine.generate(r, c2w, ip, W, H, 0.3, FAR, jitter=1, frames=5, max_bounce=4)
    engine.trace(r, W * H, 0, FAR, W, H)
    nb = engine.enqueue_bounce(r, W * H, 0, FAR, W, H, frames=5, max_bounce=4)
    engine.trace(r, nb, 1, FAR, W, H)
    m = min(n, nb)
    ref = r.copy()
    n2 = engine.enqueue_bounce(r, m, 1, FAR, W, H, frames=5, max_bounce=4)
    assert O.enqueue_bounce(sc, ref, m, 1, FAR, W, H, frames=5, max_bounce=4) == n2
    assert np.array_equal(r[:n2].view(np.uint32), ref[:n2].view(np.uint32))
    assert np.array_equal(r[W * H:].view(np.uint32), ref[W * H:].view(np.uint32))


# ------------------------------------------------------------------ BASELINE.json C2 at full size
@pytest.fixture(scope="module")
def sponza():
    blas = tthip.Blas(tthip.Mesh.sponza())
    am = tthip.AssetManager()
    am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
    return am.build()


def test_sponza_1080p_primary_and_bounce_full_parity(engine, sponza):
    W, H = 1920, 1080
    c2w, ip = tthip.unity_camera((-10, 2, 0), (1, 0, 0), (0, 1, 0), 60, W, H, 0.3, FAR)
    engine.upload(sponza)
    rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, 0.3, FAR, jitter=0)  # no jitter: the centre ray is axis-parallel
    rg, rc, ig, ic, s, cnt = trace_both(engine, sponza, rays, W * H, 0, W, H, upload=False)
    assert_same(rg, rc, ig, ic, 0, W * H)
    assert s.reps_exhausted == int((cnt["status"] == 1).sum())
    ro = rg.copy()
    nb = engine.enqueue_bounce(rg, W * H, 0, FAR, W, H)
    assert nb > 0.9 * W * H
    # 2,025 look-back tiles: the compacted bounce rays are bit-identical to the oracle's
    assert O.enqueue_bounce(sponza, ro, W * H, 0, FAR, W, H) == nb
    assert np.array_equal(rg[W * H:W * H + nb].view(np.uint32), ro[W * H:W * H + nb].view(np.uint32))
    del ro
    colors = np.zeros(W * H, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    rg2, rc2, ig2, ic2, s2, cnt2 = trace_both(engine, sponza, rg, nb, 1, W, H, colors=colors, upload=False)
    assert_same(rg2, rc2, ig2, ic2, W * H, nb)
    assert s2.node_visits == int(cnt2["node_visits"].sum())


@pytest.mark.parametrize("frames", [0, 1, 2])
def test_sponza_1080p_jittered_frames_through_the_timed_kernels(engine, sponza, frames):
    """bench.py's exact workload and kernels: the reference's default jittered Generate (frames_accumulated =
    frames, one per frame slot), the primary launch through tt_trace_kernel<false,false,1> and the bounce-1
    launch through <false,false,2> -- the non-stats instantiations the bench times (trace_both runs the STATS
    ones) -- with every hit record and _PrimaryTriangleInfo texel poisoned first, so a record the kernels
    fail to write cannot pass as the oracle's."""
    W, H = 1920, 1080
    WH = W * H
    c2w, ip = tthip.unity_camera((-10, 2, 0), (1, 0, 0), (0, 1, 0), 60, W, H, 0.3, FAR)
    engine.upload(sponza)
    rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, 0.3, FAR, jitter=1, frames=frames, max_bounce=1)
    engine.trace(rays, WH, 0, FAR, W, H)
    nb = engine.enqueue_bounce(rays, WH, 0, FAR, W, H, frames=frames, max_bounce=1)
    assert nb > 0.9 * WH
    rays["hits"][:WH] = 0xA5A5A5A5
    rays["hits"][WH:WH + nb] = 0xA5A5A5A5
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    rg, rc = rays.copy(), rays.copy()
    ig0, ic0, ig1, ic1 = (np.full((WH, 4), 0xA5A5A5A5, np.uint32) for _ in range(4))
    s0 = engine.trace(rg, WH, 0, FAR, W, H, info=ig0)  # stats=False: the non-stats kernel
    s1 = engine.trace(rg, nb, 1, FAR, W, H, info=ig1, colors=colors)
    assert s0.node_visits == 0 and s1.node_visits == 0  # no counters: not the STATS instantiation
    assert O.trace(sponza, rc, WH, 0, FAR, W, H, info=ic0, nthreads=CPU_THREADS)[0] == 0
    assert O.trace(sponza, rc, nb, 1, FAR, W, H, info=ic1, colors=colors, nthreads=CPU_THREADS)[0] == 0
    assert_same(rg, rc, ig0, ic0, 0, WH)
    assert_same(rg, rc, ig1, ic1, WH, nb)
    # a record neither side writes (the Reps bound) keeps the poison on both; nearly every ray gets one
    assert int(np.all(rg["hits"][:WH] == 0xA5A5A5A5, axis=1).sum()) < 16


def test_sponza_4k_properties(engine, sponza):
    """At C5's ray count (3840x2160): determinism (two launches give identical bytes) and a
    strided 1/64 sample against the oracle."""
    W, H = 3840, 2160
    c2w, ip = tthip.unity_camera((-12, 6, 3), (1, -0.2, -0.1), (0, 1, 0), 75, W, H, 0.3, FAR)
    engine.upload(sponza)
    rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, 0.3, FAR, jitter=1, frames=7)
    a = rays.copy()
    engine.trace(a, W * H, 0, FAR, W, H)
    b = rays.copy()
    engine.trace(b, W * H, 0, FAR, W, H)
    assert np.array_equal(a, b)
    idx = np.arange(0, W * H, 64)
    sample = np.zeros(2 * len(idx), tthip.RAY_DTYPE)
    sample[: len(idx)] = rays[idx]
    st, _ = O.trace(sponza, sample, len(idx), 0, FAR, len(idx), 1, nthreads=CPU_THREADS)
    assert st == 0
    assert np.array_equal(sample["hits"][: len(idx)], a["hits"][idx])


# ------------------------------------------------------------------ any-hit (kernel_shadow, §8 f1)
def shadow_both(engine, sc, srays, bounce, W, H, upload=True):
    if upload:
        engine.upload(sc)
    n = len(srays)
    out = []
    for side in ("gpu", "cpu"):
        r = srays.copy()
        vis = np.full((n, 4), 7.0, np.float32)
        col = np.zeros(W * H, tthip.COL_DTYPE)
        col["Direct"] = 0.5
        nee = np.full((W * H, 4), 9.0, np.float32)
        if side == "gpu":
            s = engine.trace_shadow(r, n, bounce, W, H, visibility=vis, colors=col, nee_pos=nee, stats=True)
            out.append((r, vis, col, nee, s))
        else:
            st, cnt = O.shadow(sc, r, n, bounce, W, H, visibility=vis, colors=col, nee_pos=nee, counts=True,
                               nthreads=CPU_THREADS)
            assert st == 0
            out.append((r, vis, col, nee, cnt))
    (rg, vg, cg, ng, s), (rc, vc, cc, nc, cnt) = out
    b = lambda x: np.ascontiguousarray(x).view(np.uint8)  # noqa: E731  (NaN-safe comparison)
    assert np.array_equal(b(rg), b(rc)), f"{int((b(rg) != b(rc)).sum())} shadow ray bytes differ"
    assert same_floats(vg, vc), "visibility differs"
    assert same_floats(np.ascontiguousarray(cg).view(np.float32), np.ascontiguousarray(cc).view(np.float32)), \
        "GlobalColors differ"
    assert same_floats(ng, nc), "NEEPosA differs"
    assert s.node_visits == int(cnt["node_visits"].sum()) and s.tri_tests == int(cnt["tri_tests"].sum())
    assert s.hits == int((cnt["status"] == 4).sum())
    return rg, vg, s, cnt


@pytest.mark.parametrize("case", K.SHADOW_CASES, ids=lambda c: c.__name__)
def test_shadow_kat_on_gpu(engine, case):
    name, sc, rays, expected = case()
    n = len(rays)
    rg, vg, s, cnt = shadow_both(engine, sc, rays, 0, n, 1)
    assert cnt["status"].tolist() == expected, name
    assert [0 if v[3] == 1.0 else 4 for v in vg] == expected


def test_shadow_reps_and_glass_on_gpu(engine):
    _, sc, _, _, _ = K.case_reps_exhausted()
    rays = hb.shadow_rays([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)], [2.0])
    engine.upload(sc)
    vis = np.zeros((1, 4), np.float32)
    s = engine.trace_shadow(rays, 1, 0, 1, 1, visibility=vis, stats=True)
    assert rays["t"][0] == 2.0 and vis[0].tolist() == [0, 0, 0, -1] and s.reps_exhausted == 1
    _, sc, rays, _ = K.shadow_case_single_triangle()
    sc.materials[0]["specTrans"] = 1.0
    engine.upload(sc)
    s, st = engine.trace_shadow(rays, len(rays), 0, len(rays), 1, check=False)
    assert st == tthip.TT_ERR_UNSUPPORTED


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_shadow_random_soup(engine, seed):
    rng = np.random.default_rng(seed)
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, int(rng.integers(2000, 40000)), 1.0,
                                                   float(rng.uniform(0.02, 0.2))))
    W, H = int(rng.integers(40, 200)), int(rng.integers(20, 120))
    pos = rng.uniform(-2.5, 2.5, 3)
    c2w, ip = tthip.unity_camera(pos, -pos, (0, 1, 0), 60.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    engine.upload(sc)
    engine.trace(rays, W * H, 0, FAR, W, H)
    sr = hb.nee_rays_from_hits(rays, W * H, pos * 1.2 + rng.normal(0, 0.3, 3), seed)  # light near the eye
    assert len(sr) > 0
    _, vg, s, cnt = shadow_both(engine, sc, sr, 0, W, H, upload=False)
    assert 0 < s.hits < len(sr)  # some occluded, some not


@pytest.mark.parametrize("seed", [15])
def test_shadow_instanced_bounce1(engine, seed):
    sc = instanced_scene(seed)
    W, H = 160, 90
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    engine.upload(sc)
    engine.trace(rays, W * H, 0, FAR, W, H)
    sr = hb.nee_rays_from_hits(rays, W * H, (5.0, 30.0, 10.0), seed)
    for bounce in (0, 1):
        _, _, s, cnt = shadow_both(engine, sc, sr, bounce, W, H, upload=False)
        assert s.blas_entries > len(sr)


def test_shadow_sponza_1080p_full_parity(engine, sponza):
    W, H = 1920, 1080
    c2w, ip = tthip.unity_camera((-10, 2, 0), (1, 0, 0), (0, 1, 0), 60, W, H, 0.3, FAR)
    engine.upload(sponza)
    rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    engine.generate(rays, c2w, ip, W, H, 0.3, FAR, jitter=1)
    engine.trace(rays, W * H, 0, FAR, W, H)
    sr = hb.nee_rays_from_hits(rays, W * H, (0.0, 9.0, 0.5), 3)
    assert len(sr) > 0.9 * W * H
    _, _, s, cnt = shadow_both(engine, sponza, sr, 0, W, H, upload=False)
    assert 0 < s.hits < len(sr)


def test_shadow_device_pointers(engine):
    import torch
    _, sc, rays, expected = K.shadow_case_flags()
    engine.upload(sc)
    n = len(rays)
    dev = torch.device("cuda:0")
    rt = torch.from_numpy(rays.view(np.uint8).copy()).to(dev)
    vt = torch.zeros((n, 4), dtype=torch.float32, device=dev)
    engine.trace_shadow(rt, n, 0, n, 1, visibility=vt, device=True)
    torch.cuda.synchronize()
    back = rt.cpu().numpy().view(tthip.SHADOW_DTYPE)
    assert [0 if v == 1.0 else 4 for v in vt[:, 3].cpu().tolist()] == expected
    assert [int(t == 0.0) * 4 for t in back["t"]] == expected


# ------------------------------------------------------------------ Cutout alpha test (§8 f3)
def cutout_soup(seed):
    """Random soup where every other triangle uses a Cutout material with a random atlas rectangle,
    random UVs (including negative / > 1 to exercise AlignUV's wrap) and a noisy 64x32 alpha atlas."""
    rng = np.random.default_rng(seed)
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, 6000, 1.0, 0.15))
    n = len(sc.tris)
    sc.tris["tex0"] = rng.uniform(-1.5, 1.5, (n, 2))
    sc.tris["texedge1"] = rng.uniform(-1.5, 1.5, (n, 2))
    sc.tris["texedge2"] = rng.uniform(-1.5, 1.5, (n, 2))
    sc.tris["MatDat"] = np.arange(n) % 3
    mats = np.zeros(3, tthip.MAT_DTYPE)
    for m in (1, 2):
        mats[m]["MatType"] = tthip.MAT_CUTOUT_INDEX
        mats[m]["AlphaCutoff"] = rng.uniform(0.2, 0.8)
        mats[m]["AlbedoTexScale"] = [rng.uniform(0.5, 2), rng.uniform(0.5, 2), rng.uniform(-1, 1), rng.uniform(-1, 1)]
        lo = rng.integers(0, 8000, 2)
        hi = lo + rng.integers(1000, 8000, 2)
        mats[m]["AlphaTex"] = [int(hi[0]) | (int(hi[1]) << 15), int(lo[0]) | (int(lo[1]) << 15)]
    sc.materials = mats
    sc.alpha_atlas = rng.integers(0, 256, (32, 64)).astype(np.uint8)
    return sc


@pytest.mark.parametrize("seed", [21, 22])
def test_cutout_random_soup_closest_and_shadow(engine, seed):
    sc = cutout_soup(seed)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, W * H)
    # the alpha test must actually reject some candidates: closest hits differ from an opaque trace
    opaque = rays.copy()
    sc_opaque = cutout_soup(seed)
    sc_opaque.materials["MatType"] = 0
    st, _ = O.trace(sc_opaque, opaque, W * H, 0, FAR, W, H, nthreads=CPU_THREADS)
    assert st == 0 and (opaque["hits"][: W * H] != rg["hits"][: W * H]).any(1).sum() > 50
    sr = hb.nee_rays_from_hits(rg, W * H, (0.5, 2.0, 2.5), seed)
    shadow_both(engine, sc, sr, 0, W, H, upload=False)


# ------------------------------------------------------------------ stained-glass shadows (§8 f1)
def test_shadow_glass_kat_on_gpu(engine):
    name, sc, rays, expected, thr = K.shadow_case_glass()
    n = len(rays)
    rg, vg, s, cnt = shadow_both(engine, sc, rays, 0, n, 1)
    assert cnt["status"].tolist() == expected
    for i, e in enumerate(expected):
        if e == 0:
            assert vg[i, :3].tobytes() == thr[i].astype(np.float32).tobytes(), i


def test_shadow_glass_without_texture_atlas_is_refused():
    _, sc, rays, _, _ = K.shadow_case_glass()
    sc.texture_atlas = None
    e = tthip.Engine(0)
    try:
        e.upload(sc)
        with pytest.raises(tthip.TTError) as ex:
            e.trace_shadow(rays.copy(), len(rays), 0, len(rays), 1)
        assert ex.value.status == tthip.TT_ERR_UNSUPPORTED
    finally:
        e.close()


def glass_soup(seed):
    """Random soup with opaque, glass (textured / untextured), glass + Cutout and Cutout materials,
    random UVs (wrapping), a noisy alpha atlas and a random RGBA half texture atlas."""
    rng = np.random.default_rng(seed)
    sc = cutout_soup(seed)
    n = len(sc.tris)
    sc.tris["MatDat"] = rng.integers(0, 5, n)
    mats = np.zeros(5, tthip.MAT_DTYPE)
    for m in (1, 2, 3):
        mats[m]["specTrans"] = 1.0
        mats[m]["surfaceColor"] = rng.uniform(0.2, 1.0, 3)
        mats[m]["AlbedoTexScale"] = [rng.uniform(0.5, 2), rng.uniform(0.5, 2), rng.uniform(-1, 1), rng.uniform(-1, 1)]
        lo = rng.integers(0, 8000, 2)
        hi = lo + rng.integers(1000, 8000, 2)
        mats[m]["AlbedoTex"] = [int(hi[0]) | (int(hi[1]) << 15), int(lo[0]) | (int(lo[1]) << 15)] if m != 2 else [0, 0]
    for m in (3, 4):
        mats[m]["MatType"] = tthip.MAT_CUTOUT_INDEX
        mats[m]["AlphaCutoff"] = rng.uniform(0.2, 0.8)
        lo = rng.integers(0, 8000, 2)
        hi = lo + rng.integers(1000, 8000, 2)
        mats[m]["AlphaTex"] = [int(hi[0]) | (int(hi[1]) << 15), int(lo[0]) | (int(lo[1]) << 15)]
    mats[4]["AlbedoTexScale"] = [1.0, 1.0, 0.0, 0.0]
    sc.materials = mats
    sc.texture_atlas = rng.uniform(0.0, 4.0, (24, 40, 4)).astype(np.float16)
    return sc


@pytest.mark.parametrize("seed", [41, 42])
def test_glass_random_soup_shadow(engine, seed):
    """Throughput = product of the glass tints in traversal order, bit for bit against the oracle,
    including the cooperative drain phase (the tints of a group's triangles multiplied in order)."""
    sc = glass_soup(seed)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, W * H)
    sr = hb.nee_rays_from_hits(rg, W * H, (0.5, 2.0, 2.5), seed)
    _, vg, _, sc_cnt = shadow_both(engine, sc, sr, 0, W, H, upload=False)
    reached = sc_cnt["status"] == 0
    tinted = reached & (vg[:, :3] != 1.0).any(1)
    assert tinted.sum() > 100, "glass must tint a good share of the unoccluded rays"


# ------------------------------------------------------------------ TLAS refit (§8 f4)
def refit_scene(seed, offsets=None, n_inst=120):
    rng = np.random.default_rng(seed)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(seed, 3000, 20.0, 0.5)), tthip.trs_matrix((0, 0, 0)),
                  np.zeros(1, tthip.MAT_DTYPE))
    props = [am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(seed * 10 + k, 600)), np.zeros(1, tthip.MAT_DTYPE))
             for k in range(6)]
    for i in range(n_inst):
        pos = rng.uniform(-40, 40, 3) * [1, 0.2, 1]
        if offsets is not None:
            pos = pos + offsets[i]
        am.add_instance(props[i % 6], tthip.trs_matrix(pos, float(rng.uniform(0, 360)), float(rng.uniform(0.5, 2))))
    return am.build()


@pytest.mark.parametrize("seed", [31, 32])
def test_tlas_refit_matches_oracle(engine, seed):
    sc = refit_scene(seed)
    rng = np.random.default_rng(seed)
    boxes = sc.meta["mesh_aabbs"].copy()
    boxes += rng.normal(0, 2.0, (len(boxes), 1)).astype(np.float32)  # move every instance
    boxes[3, 3:] = boxes[3, :3]                                        # a degenerate (flat) box
    engine.upload(sc)
    engine.tlas_refit(sc.tlas_nodes, boxes)
    got = engine.scene_nodes(0, len(sc.nodes))
    st, want = O.tlas_refit(sc, boxes)
    assert st == 0
    assert np.array_equal(got, want), f"{int((got != want).sum())} nodes differ"
    # device-pointer, asynchronous form, repeated (the plan is cached), same bytes
    import torch
    bt = torch.from_numpy(boxes).to(torch.device("cuda:0"))
    engine.tlas_refit(sc.tlas_nodes, bt, device=True, asynchronous=True)
    engine.sync()
    assert np.array_equal(engine.scene_nodes(0, len(sc.nodes)), want)


def test_tlas_refit_moved_instances_then_trace(engine):
    """Per-frame path of the reference: instances move (new _MeshData W2L + new mesh AABBs), the
    TLAS is refit on the GPU (topology kept), then traced. Bit-exact vs the oracle on the same
    refit nodes, and the same closest hits as a TLAS freshly built for the moved scene."""
    rng = np.random.default_rng(7)
    a = refit_scene(33)
    b = refit_scene(33, offsets=rng.normal(0, 1.5, (120, 3)))
    engine.upload(a)
    engine.update_meshdata(0, b.meshdata)
    engine.tlas_refit(a.tlas_nodes, b.meta["mesh_aabbs"])
    W, H = 160, 90
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    rg = rays.copy()
    engine.trace(rg, W * H, 0, FAR, W, H)
    st, nodes = O.tlas_refit(tthip.Scene(a.nodes, a.tris, a.tlas, b.meshdata, a.materials, tlas_nodes=a.tlas_nodes),
                             b.meta["mesh_aabbs"])
    assert st == 0
    refit = tthip.Scene(nodes, a.tris, a.tlas, b.meshdata, a.materials, tlas_nodes=a.tlas_nodes)
    rc = rays.copy()
    assert O.trace(refit, rc, W * H, 0, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
    assert np.array_equal(rg["hits"], rc["hits"])
    rf = rays.copy()
    assert O.trace(b, rf, W * H, 0, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
    same = (rf["hits"][: W * H, :3] == rg["hits"][: W * H, :3]).all(1)
    assert same.mean() > 0.999  # ties between coincident instances may resolve differently


# ------------------------------------------------------------------ BLAS refit (§8 f4, deforming meshes)
@pytest.mark.parametrize("n_tris", [2000, 60000])
def test_blas_refit_matches_oracle_and_traces(engine, n_tris):
    from test_blas_refit import deform, two_mesh_scene, vertex_buffer

    sc, mesh, blas = two_mesh_scene(seed=13, n=n_tris)
    pos, nrm, idx = mesh.arrays()
    leaf = blas.leaf_order()
    engine.upload(sc)
    W, H = 128, 96
    c2w, ip = tthip.unity_camera((1.0, 3.0, 14.0), (0, -0.15, -1), (0, 1, 0), 60, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    for t, xf in ((0.3, np.eye(4)), (1.9, tthip.trs_matrix((0.2, -0.1, 0.3), 17.0, 1.0))):
        V = vertex_buffer(deform(pos, t), nrm)
        engine.blas_refit(1, V, idx, leaf, xf)
        st, nodes, tris = O.blas_refit(sc, 1, V, idx, leaf, xf)
        assert st == 0
        assert np.array_equal(engine.scene_nodes(0, len(nodes)), nodes), "refit nodes differ"
        assert np.array_equal(engine.scene_tris(0, len(tris)), tris), "re-derived triangles differ"
        sc2 = tthip.Scene(nodes, tris, sc.tlas, sc.meshdata, sc.materials, tlas_nodes=sc.tlas_nodes)
        rg, rc, ig, ic, _, _ = trace_both(engine, sc2, rays, W * H, 0, W, H, upload=False)
        assert_same(rg, rc, ig, ic, 0, W * H)


def test_blas_refit_device_pointers_and_errors(engine):
    import torch

    from test_blas_refit import deform, two_mesh_scene, vertex_buffer

    sc, mesh, blas = two_mesh_scene(seed=21, n=3000)
    pos, nrm, idx = mesh.arrays()
    leaf = blas.leaf_order()
    engine.upload(sc)
    V = vertex_buffer(deform(pos, 0.8), nrm)
    dev = torch.device("cuda", 0)
    Vd, Id, Ld = (torch.from_numpy(a).to(dev) for a in (V, idx, leaf))
    engine.blas_refit(1, Vd, Id, Ld, device=True)
    torch.cuda.synchronize()
    st, nodes, tris = O.blas_refit(sc, 1, V, idx, leaf)
    assert st == 0
    assert np.array_equal(engine.scene_nodes(0, len(nodes)), nodes)
    assert np.array_equal(engine.scene_tris(0, len(tris)), tris)
    with pytest.raises(tthip.TTError):
        engine.blas_refit(7, V, idx, leaf)  # no such mesh
    bad = idx.copy()
    bad[5] = len(pos) + 3
    with pytest.raises(tthip.TTError):
        engine.blas_refit(1, V, bad, leaf)  # index out of range (host arrays are validated)


# ------------------------------------------------------------------ degenerate ray inputs
def degenerate_rays(n, seed):
    """Normal rays mixed with the numerically hostile ones a renderer can hand over: zero, signed-zero,
    denormal, NaN and infinite direction components, NaN / infinite origins."""
    rng = np.random.default_rng(seed)
    rays = np.zeros(2 * n, tthip.RAY_DTYPE)
    o = rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    specials = np.array([0.0, -0.0, 1e-40, -1e-40, np.nan, np.inf, -np.inf, 1e-30, 1e30], np.float32)
    k = rng.integers(0, 4, n)  # 0: normal, 1: special direction component, 2: special origin, 3: both
    for i in range(n):
        if k[i] in (1, 3):
            d[i, rng.integers(0, 3)] = specials[rng.integers(0, len(specials))]
            if rng.random() < 0.2:
                d[i] = 0.0
        if k[i] in (2, 3):
            o[i, rng.integers(0, 3)] = specials[rng.integers(4, len(specials))]
    rays["origin"][:n] = o
    rays["direction"][:n] = d
    rays["PixelIndex"][:n] = np.arange(n)
    return rays


@pytest.mark.parametrize("seed", [3, 4])
def test_degenerate_rays_closest_and_shadow(engine, seed):
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, 4000, 1.0, 0.15))
    n = 4096
    rays = degenerate_rays(n, seed)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, n, 0, n, 1, upload=True)
    assert_same(rg, rc, ig, ic, 0, n)
    assert s.node_visits == int(cnt["node_visits"].sum())
    sh = np.zeros(n, tthip.SHADOW_DTYPE)
    sh["origin"] = rays["origin"][:n]
    sh["direction"] = rays["direction"][:n]
    sh["t"] = np.where(np.arange(n) % 3 == 0, np.float32(np.inf), np.float32(2.5))
    sh["illumination"] = 1.0
    sh["PixelIndex"] = np.arange(n)
    shadow_both(engine, sc, sh, 0, n, 1, upload=False)


def test_degenerate_rays_later_bounce_info(engine):
    """Bounce 1 with every pixel's GlobalColors.Data.w = -1: the _PrimaryTriangleInfo position /
    direction form is written for all rays, including the NaN ones (NaN payloads may differ)."""
    sc = tthip.single_object_scene(tthip.Mesh.soup(8, 3000, 1.0, 0.15))
    n = 2048
    base = degenerate_rays(n, 8)
    rays = np.zeros(2 * n, tthip.RAY_DTYPE)
    rays[n:] = base[:n]  # odd bounces read the second half
    colors = np.zeros(n, tthip.COL_DTYPE)
    colors["Data"][:, 3] = -1.0
    engine.upload(sc)
    rg, rc = rays.copy(), rays.copy()
    ig, ic = np.zeros((n, 4), np.uint32), np.zeros((n, 4), np.uint32)
    engine.trace(rg, n, 1, FAR, n, 1, info=ig, colors=colors)
    st, _ = O.trace(sc, rc, n, 1, FAR, n, 1, info=ic, colors=colors, nthreads=CPU_THREADS)
    assert st == 0
    assert np.array_equal(rg.view(np.uint8), rc.view(np.uint8))
    assert same_floats(ig.view(np.float32), ic.view(np.float32))


# ------------------------------------------------------------------ coincident / degenerate geometry
def duplicate_soup(seed, n_base=1500):
    """A soup where every triangle exists 1-3 times at identical positions (exact t ties between
    triangles in different leaves: the first found in the reference's order must win), plus
    zero-area, collinear and far-away triangles."""
    rng = np.random.default_rng(seed)
    base = rng.uniform(-1, 1, (n_base, 1, 3)) + rng.normal(scale=0.08, size=(n_base, 3, 3))
    reps = rng.integers(1, 4, n_base)
    tris = np.repeat(base, reps, axis=0)
    extra = [np.repeat(rng.uniform(-1, 1, (1, 3)), 3, axis=0) for _ in range(40)]            # points
    extra += [np.outer(rng.uniform(0, 1, 3), rng.normal(size=3)) for _ in range(40)]         # collinear
    extra += [rng.uniform(-1, 1, (1, 3)) * 1e5 + rng.normal(size=(3, 3)) for _ in range(10)]  # far away
    tris = np.concatenate([tris, np.stack(extra)]).astype(np.float32)
    tris = tris[rng.permutation(len(tris))]
    pos = tris.reshape(-1, 3)
    idx = np.arange(len(pos), dtype=np.int32)
    return tthip.single_object_scene(tthip.Mesh.from_arrays(pos, idx))


@pytest.mark.parametrize("seed", [31, 32])
def test_coincident_triangles_tie_break(engine, seed):
    sc = duplicate_soup(seed)
    W, H = 200, 150
    c2w, ip = tthip.unity_camera((0.1, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 60, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H)
    assert_same(rg, rc, ig, ic, 0, W * H)
    assert s.accepts == int(cnt["accepts"].sum())


# ------------------------------------------------ trace variants IgnoreGlassMain / IgnoreBackfacing
@pytest.mark.parametrize("seed", [61, 62])
@pytest.mark.parametrize("flags", [tthip.TT_TRACE_IGNORE_GLASS, tthip.TT_TRACE_IGNORE_BACKFACING,
                                   tthip.TT_TRACE_IGNORE_GLASS | tthip.TT_TRACE_IGNORE_BACKFACING])
def test_trace_variant_flags_random_soup(engine, seed, flags):
    """IntersectionKernels.compute:42-47 as launch flags, bit for bit against the oracle on a soup
    with glass, glass + Cutout, Cutout and opaque materials (some MatDat out of range), primary
    rays with _PrimaryTriangleInfo and bounce-1 rays (IgnoreBackfacing applies at bounce 0 only)."""
    sc = glass_soup(seed)
    rng = np.random.default_rng(seed)
    sc.tris["MatDat"] = np.where(rng.random(len(sc.tris)) < 0.05, 9, sc.tris["MatDat"])  # out of range
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    rg, rc, ig, ic, s, cnt = trace_both(engine, sc, rays, W * H, 0, W, H, flags=flags)
    assert_same(rg, rc, ig, ic, 0, W * H)
    plain = rays.copy()
    O.trace(sc, plain, W * H, 0, FAR, W, H)
    changed = int((plain["hits"][: W * H] != rc["hits"][: W * H]).any(1).sum())
    assert changed > 50, "the variant must change a good share of the primary hits"
    r1, n1 = bounce_rays(sc, rc, W, H, seed)
    if n1:
        colors = np.zeros(W * H, tthip.COL_DTYPE)
        colors["Data"][:, 3] = 1.0
        rg1, rc1, ig1, ic1, _, _ = trace_both(engine, sc, r1, n1, 1, W, H, colors=colors, flags=flags, upload=False)
        assert_same(rg1, rc1, ig1, ic1, W * H, n1)


# ------------------------------------------- row f1: the full kernel_shadow output contract
@pytest.mark.parametrize("bounce", [0, 1])
@pytest.mark.parametrize("flags", [tthip.TT_SHADOW_RADIANCE_CACHE, tthip.TT_SHADOW_RADIANCE_CACHE | tthip.TT_TRACE_USE_RESTIRGI,
                                   0, tthip.TT_TRACE_USE_RESTIRGI])
def test_shadow_accumulations_match_oracle(engine, bounce, flags):
    """IntersectionKernels.compute:457-485 with and without the RadianceCache define: CacheBuffer
    CurrentIlluminance (EncodeRGB / DecodeRGB), Indirect, PrimaryNEERay (packRGBE of pow terms),
    Direct, NEEPosA -- bit for bit against the oracle, glass-tinted throughputs included. Random
    initial colours, packed words (PrimaryNEERay, LuminanceIncomming, CurrentIlluminance) and
    Data.w in {-1, bounce, other}; t < 0 on a quarter of the rays (the sign picks the target)."""
    seed = 70 + bounce * 4 + flags % 7
    sc = glass_soup(seed)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    O.trace(sc, rays, W * H, 0, FAR, W, H)
    rng = np.random.default_rng(seed)
    sr = hb.nee_rays_from_hits(rays, W * H, (0.5, 2.0, 2.5), seed)
    sr["illumination"] *= rng.uniform(0.1, 30.0, (len(sr), 1)).astype(np.float32)
    lum = (rng.integers(14, 26, len(sr)).astype(np.uint32) << 27) | rng.integers(0, 1 << 27, len(sr)).astype(np.uint32)
    sr["LuminanceIncomming"] = lum.view(np.float32)
    col = np.zeros(W * H, tthip.COL_DTYPE)
    col["Direct"] = rng.uniform(0, 2, (W * H, 3))
    col["Indirect"] = rng.uniform(0, 2, (W * H, 3))
    col["PrimaryNEERay"] = (rng.integers(12, 24, W * H).astype(np.uint32) << 27) | \
        rng.integers(0, 1 << 27, W * H).astype(np.uint32)
    col["Data"][:, 3] = rng.choice(np.array([-1.0, float(bounce), 5.0], np.float32), W * H)
    cache = np.zeros(W * H, tthip.CACHE_DTYPE)
    cache["CurrentIlluminance"] = rng.integers(0, 1 << 32, W * H, dtype=np.uint64).astype(np.uint32)
    cache["CurrentIlluminance"][::7] = 0
    engine.upload(sc)
    n = len(sr)
    out = []
    for side in ("gpu", "cpu"):
        r, c, ch = sr.copy(), col.copy(), cache.copy()
        vis = np.full((n, 4), 7.0, np.float32)
        nee = np.full((W * H, 4), 9.0, np.float32)
        if side == "gpu":
            engine.trace_shadow(r, n, bounce, W, H, visibility=vis, colors=c, nee_pos=nee, cache=ch, flags=flags)
        else:
            st, _ = O.shadow(sc, r, n, bounce, W, H, visibility=vis, colors=c, nee_pos=nee, cache=ch, flags=flags,
                             nthreads=CPU_THREADS)
            assert st == 0
        out.append((r, c, ch, vis, nee))
    (rg, cg, hg, vg, ng), (rc, cc, hc, vc, nc) = out
    b = lambda x: np.ascontiguousarray(x).view(np.uint8)  # noqa: E731
    assert np.array_equal(b(rg), b(rc)), "shadow ray bytes differ"
    assert same_floats(vg, vc), "visibility differs"
    assert same_floats(ng, nc), "NEEPosA differs"
    for f in ("Direct", "Indirect", "Data"):
        assert same_floats(cg[f], cc[f]), f"GlobalColors.{f} differs"
    assert np.array_equal(cg["PrimaryNEERay"], cc["PrimaryNEERay"]), \
        f"{int((cg['PrimaryNEERay'] != cc['PrimaryNEERay']).sum())} PrimaryNEERay words differ"
    assert np.array_equal(hg["CurrentIlluminance"], hc["CurrentIlluminance"]), \
        f"{int((hg['CurrentIlluminance'] != hc['CurrentIlluminance']).sum())} CurrentIlluminance words differ"
    reached = vc[:, 3] == 1.0
    assert reached.sum() > 200
    if flags & tthip.TT_SHADOW_RADIANCE_CACHE:
        assert (hc["CurrentIlluminance"] != cache["CurrentIlluminance"]).sum() > 100
    if not (bounce != 0 and (flags & tthip.TT_SHADOW_RADIANCE_CACHE) and (flags & tthip.TT_TRACE_USE_RESTIRGI)):
        # (with RadianceCache + ReSTIR GI every t < 0 ray of a later bounce goes to Indirect, :477)
        assert (cc["PrimaryNEERay"] != col["PrimaryNEERay"]).sum() > 20


@pytest.mark.parametrize("bounce", [0, 1])
def test_legacy_shadow_entry_contract(engine, bounce):
    """tt_trace_shadow keeps its original contract (include/truetrace_hip.h): visibility, the t = 0
    write-back, Direct += at bounce 0 and NEEPosA -- and none of tt_trace_shadow_ex's Indirect /
    PrimaryNEERay accumulations, so a caller doing those itself does not double-count. Against the
    oracle, with t < 0 on a quarter of the rays and Data.w == bounce (the rays tt_trace_shadow_ex
    would accumulate into Indirect / PrimaryNEERay)."""
    seed = 90 + bounce
    sc = glass_soup(seed)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    O.trace(sc, rays, W * H, 0, FAR, W, H)
    rng = np.random.default_rng(seed)
    sr = hb.nee_rays_from_hits(rays, W * H, (0.5, 2.0, 2.5), seed)
    assert (sr["t"] < 0).sum() > 100
    col = np.zeros(W * H, tthip.COL_DTYPE)
    col["Direct"] = rng.uniform(0, 2, (W * H, 3))
    col["Indirect"] = rng.uniform(0, 2, (W * H, 3))
    col["PrimaryNEERay"] = (rng.integers(12, 24, W * H).astype(np.uint32) << 27) | \
        rng.integers(0, 1 << 27, W * H).astype(np.uint32)
    col["Data"][:, 3] = float(bounce)
    engine.upload(sc)
    n = len(sr)
    rg, cg = sr.copy(), col.copy()
    vg = np.full((n, 4), 7.0, np.float32)
    ng = np.full((W * H, 4), 9.0, np.float32)
    engine.trace_shadow(rg, n, bounce, W, H, visibility=vg, colors=cg, nee_pos=ng, legacy=True)
    rc, cc = sr.copy(), col.copy()
    vc = np.full((n, 4), 7.0, np.float32)
    nc = np.full((W * H, 4), 9.0, np.float32)
    st, _ = O.shadow(sc, rc, n, bounce, W, H, visibility=vc, colors=cc, nee_pos=nc, nthreads=CPU_THREADS)
    assert st == 0
    b = lambda x: np.ascontiguousarray(x).view(np.uint8)  # noqa: E731
    assert np.array_equal(b(rg), b(rc)), "shadow ray bytes differ"
    assert same_floats(vg, vc), "visibility differs"
    assert same_floats(ng, nc), "NEEPosA differs"
    assert same_floats(cg["Direct"], cc["Direct"]), "GlobalColors.Direct differs"
    # the accumulations tt_trace_shadow leaves to the caller: untouched
    assert np.array_equal(b(cg["Indirect"]), b(col["Indirect"]))
    assert np.array_equal(cg["PrimaryNEERay"], col["PrimaryNEERay"])
    # ... which the full contract (the oracle) does change on this input
    changed = (cc["PrimaryNEERay"] != col["PrimaryNEERay"]).sum() + (cc["Indirect"] != col["Indirect"]).any(1).sum()
    assert changed > 20


@pytest.mark.parametrize("seed", [81, 82])
def test_visibility_check_mode(engine, seed):
    """VisabilityCheckCompute (CommonData.cginc:710-819): the distance as given, visibility only,
    nothing else written -- against the oracle's literal restatement."""
    sc = glass_soup(seed)
    W, H = 96, 64
    c2w, ip = tthip.unity_camera((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    O.trace(sc, rays, W * H, 0, FAR, W, H)
    sr = hb.nee_rays_from_hits(rays, W * H, (0.5, 2.0, 2.5), seed)
    engine.upload(sc)
    n = len(sr)
    vg = np.full((n, 4), 7.0, np.float32)
    vc = vg.copy()
    rg, rc = sr.copy(), sr.copy()
    col = np.zeros(W * H, tthip.COL_DTYPE)
    cg, cc = col.copy(), col.copy()
    engine.trace_shadow(rg, n, 0, W, H, visibility=vg, colors=cg, flags=tthip.TT_SHADOW_VISIBILITY_CHECK)
    st, _ = O.shadow(sc, rc, n, 0, W, H, visibility=vc, colors=cc, flags=tthip.TT_SHADOW_VISIBILITY_CHECK,
                     nthreads=CPU_THREADS)
    assert st == 0
    assert np.array_equal(vg, vc), f"{int((vg != vc).any(1).sum())} visibilities differ"
    assert set(np.unique(vg[:, 0])) <= {0.0, 1.0} and (vg[:, 0] == 0).sum() > 50 and (vg[:, 0] == 1).sum() > 50
    b = lambda x: np.ascontiguousarray(x).view(np.uint8)  # noqa: E731
    assert np.array_equal(b(rg), b(sr)) and np.array_equal(b(cg), b(col)), "visibility mode writes nothing else"
    # negative distance: nothing can be hit (tmax < 0), every ray is visible, as in the reference
    neg = sr.copy()
    neg["t"] = -np.abs(neg["t"])
    v2 = np.zeros((n, 4), np.float32)
    engine.trace_shadow(neg, n, 0, W, H, visibility=v2, flags=tthip.TT_SHADOW_VISIBILITY_CHECK)
    assert (v2[:, 0] == 1.0).all()


def test_async_chain_stack_overflow_is_reported(engine):
    """an overflow inside a TT_TRACE_ASYNC chain must not be lost when a later launch
    zeroes the control block it was counted in: tt_async_overflows reports every launch's."""
    import torch

    sc, rays = K.stack_overflow_scene(17)
    engine.upload(sc)
    engine.async_overflows()  # clear what earlier tests on the shared context left
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(rays.view(np.uint8).copy()).to(dev)
    for _ in range(3):  # three async launches: each overflows one ray; later launches zero the blocks
        engine.trace(buf, 1, 0, FAR, 1, 1, device=True, asynchronous=True)
    assert engine.async_overflows() == 3
    assert engine.async_overflows() == 0  # reset by the read


# ------------------------------------------------------------------ indirect dispatch (§8 f2, TransferKernel)
def test_indirect_bounce_chain_matches_host_counts(engine):
    """Primary + 3 bounces with device-resident counts (the reference's BufferSizes[].tracerays +
    TransferKernel + DispatchIndirect): trace_indirect -> enqueue_bounce_indirect -> ... issued back to
    back on the context stream with no host round trip, bit-identical to the host-count chain
    (rays, hit records, _PrimaryTriangleInfo, every bounce's survivor count); the full-frame tile order
    at bounce 0 is chosen on the device (count == W*H)."""
    import torch

    sc = tthip.single_object_scene(tthip.Mesh.soup(31, 25000, 1.0, 0.1))
    W, H = 256, 160
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.4), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, FAR)
    engine.upload(sc)
    dev = torch.device("cuda:0")
    WH = W * H
    base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    engine.generate(base, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=3, max_bounce=4, device=True)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 2.0  # _PrimaryTriangleInfo written at bounce 2
    col_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    # host-count reference chain
    ref = base.clone()
    info_ref = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
    counts = [WH]
    for b in range(3):
        engine.trace(ref, counts[-1], b, FAR, W, H, info=info_ref, colors=col_t if b else None, device=True)
        counts.append(engine.enqueue_bounce(ref, counts[-1], b, FAR, W, H, frames=3, max_bounce=4, device=True))
    engine.trace(ref, counts[-1], 3, FAR, W, H, device=True)
    # device-count chain: nothing read back until the end
    got = base.clone()
    info_got = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
    n_dev = torch.zeros(5, dtype=torch.int32, device=dev)
    n_dev[0] = WH
    torch.cuda.synchronize()
    for b in range(3):
        engine.trace_indirect(got, n_dev[b:], WH, b, FAR, W, H, info=info_got, colors=col_t if b else None)
        engine.enqueue_bounce_indirect(got, n_dev[b:], WH, n_dev[b + 1:], b, FAR, W, H, frames=3, max_bounce=4)
    engine.trace_indirect(got, n_dev[3:], WH, 3, FAR, W, H)
    torch.cuda.synchronize()
    assert n_dev[:4].tolist() == counts
    assert counts[1] > WH // 3 and counts[3] > 0
    assert torch.equal(got, ref)
    assert torch.equal(info_got, info_ref)


def test_indirect_counts_clamp_zero_and_refusals(engine):
    import torch

    sc = tthip.single_object_scene(tthip.Mesh.soup(32, 8000, 1.0, 0.1))
    W, H = 120, 90
    c2w, ip = tthip.unity_camera((0.2, 0.1, 2.8), (0, 0, -1), (0, 1, 0), 55.0, W, H, 0.05, FAR)
    engine.upload(sc)
    dev = torch.device("cuda:0")
    WH = W * H
    base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    engine.generate(base, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=0, max_bounce=2, device=True)
    for count, capacity in ((0, WH), (777, WH), (WH + 1000, 5000), (4097, 4097)):
        ref = base.clone()
        engine.trace(ref, min(count, capacity), 0, FAR, W, H, device=True)
        got = base.clone()
        n = torch.tensor([count], dtype=torch.int32, device=dev)
        engine.trace_indirect(got, n, capacity, 0, FAR, W, H)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (count, capacity)
        # enqueue: traced count from the device (clamped), survivors to the device
        ref_n = engine.enqueue_bounce(ref, min(count, capacity), 0, FAR, W, H, frames=0, max_bounce=2, device=True)
        nn = torch.zeros(1, dtype=torch.int32, device=dev)
        engine.enqueue_bounce_indirect(got, n, capacity, nn, 0, FAR, W, H, frames=0, max_bounce=2)
        torch.cuda.synchronize()
        assert int(nn.item()) == ref_n and torch.equal(got, ref), (count, capacity)
    # host pointers, host count buffers and stats are refused
    host_rays = np.zeros(2 * WH, tthip.RAY_DTYPE)
    n = torch.tensor([10], dtype=torch.int32, device=dev)
    p = tthip.TraceParams(n_rays=WH, bounce=0, far_plane=FAR, screen_width=W, screen_height=H, flags=0)
    assert engine.L.tt_trace_closest_indirect(engine.h, tthip.C.byref(p), n.data_ptr(), host_rays.ctypes.data,
                                              None, None) == tthip.TT_ERR_INVALID_ARG
    hn = np.array([10], np.uint32)
    assert engine.trace_indirect(base, hn, WH, 0, FAR, W, H, check=False) == tthip.TT_ERR_INVALID_ARG
    assert engine.trace_indirect(base, n, WH, 0, FAR, W, H, flags=tthip.TT_TRACE_STATS,
                                 check=False) == tthip.TT_ERR_INVALID_ARG
    assert engine.trace_indirect(base, None, WH, 0, FAR, W, H, check=False) == tthip.TT_ERR_INVALID_ARG


def test_indirect_shadow_matches_host_count(engine):
    import torch

    seed = 33
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, 12000, 1.0, 0.1))
    W, H = 140, 100
    pos = np.array([1.5, 1.0, 2.0])
    c2w, ip = tthip.unity_camera(pos, -pos, (0, 1, 0), 60.0, W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    engine.upload(sc)
    engine.trace(rays, W * H, 0, FAR, W, H)
    sr = hb.nee_rays_from_hits(rays, W * H, pos * 1.2, seed)
    ns = len(sr)
    assert ns > 100
    dev = torch.device("cuda:0")
    colors = np.zeros(W * H, tthip.COL_DTYPE)
    for count in (ns, ns // 3, 0):
        outs = []
        for indirect in (False, True):
            rt = torch.from_numpy(sr.view(np.uint8).copy()).to(dev)
            vt = torch.zeros((ns, 4), dtype=torch.float32, device=dev)
            ct = torch.from_numpy(colors.view(np.uint8).copy()).to(dev)
            if indirect:
                engine.trace_shadow_indirect(rt, torch.tensor([count], dtype=torch.int32, device=dev), ns, 0, W, H,
                                             visibility=vt, colors=ct)
            elif count:
                engine.trace_shadow(rt, count, 0, W, H, visibility=vt, colors=ct, device=True)
            torch.cuda.synchronize()
            outs.append((rt.cpu(), vt.cpu(), ct.cpu()))
        assert all(torch.equal(a, b) for a, b in zip(*outs)), count
