"""Oracle vs analytic known answers (parity pin for the CPU restatement; no GPU)."""
import numpy as np
import pytest

import handbuilt as hb
import kat_cases as K
import oracle_ctypes as O
import tthip


@pytest.mark.parametrize("case", K.ALL_CASES, ids=lambda c: c.__name__)
def test_kat_hits(case):
    name, sc, rays, n, expected = case()
    st, cnt = O.trace(sc, rays, n, 0, 1000.0, n, 1, counts=True)
    assert st == tthip.TT_OK
    got = rays["hits"][:n].tolist()
    assert got == [list(map(int, e)) for e in expected], name


def test_kat_culling_counts():
    _, sc, rays, n, _ = K.case_octant_order_and_culling()
    st, cnt = O.trace(sc, rays, n, 0, 1000.0, n, 1, counts=True)
    assert st == 0
    # TLAS node + root + first child visited + second child visited (its leaf is culled)
    assert cnt["node_visits"].tolist() == [4, 4]
    assert cnt["tri_tests"].tolist() == [1, 1]
    assert cnt["blas_entries"].tolist() == [1, 1]


def test_kat_reps_counts():
    _, sc, rays, n, _ = K.case_reps_exhausted()
    st, cnt = O.trace(sc, rays, n, 0, 1000.0, n, 1, counts=True)
    assert st == 0 and cnt["status"][0] == 1 and cnt["node_visits"][0] == 1000
    _, sc, rays, n, _ = K.case_chain_within_bound()
    st, cnt = O.trace(sc, rays, n, 0, 1000.0, n, 1, counts=True)
    assert st == 0 and cnt["status"][0] == 0 and cnt["node_visits"][0] == 1000


def test_kat_stack_overflow():
    # one push per level: 16 levels fill uint2 stack[16] exactly, the 17th push overflows
    sc, rays = K.stack_overflow_scene(17)
    st, cnt = O.trace(sc, rays, 1, 0, 1000.0, 1, 1, counts=True)
    assert st == tthip.TT_ERR_STACK_OVERFLOW and cnt["status"][0] == 2
    sc, rays = K.stack_overflow_scene(16)
    st, cnt = O.trace(sc, rays, 1, 0, 1000.0, 1, 1, counts=True)
    assert st == 0 and cnt["max_stack"][0] == 16 and cnt["status"][0] == 0


def test_kat_invisible_only_at_bounce0():
    sc, rays, exp0, exp1 = K.case_invisible_bounce0()
    r0 = rays.copy()
    assert O.trace(sc, r0, 1, 0, 1000.0, 1, 1)[0] == 0
    assert r0["hits"][0].tolist() == exp0
    r1 = rays.copy()
    r1[1] = r1[0]  # odd bounces read GlobalRays[W*H + i] (IntersectionKernels.compute:82)
    assert O.trace(sc, r1, 1, 1, 1000.0, 1, 1)[0] == 0
    assert r1["hits"][1].tolist() == exp1


def test_cutout_without_atlas_unsupported():
    sc, rays, _, _ = K.case_invisible_bounce0()
    sc.materials[0]["MatType"] = tthip.MAT_CUTOUT_INDEX
    assert O.trace(sc, rays, 1, 0, 1000.0, 1, 1)[0] == tthip.TT_ERR_UNSUPPORTED


def test_cutout_wrap_and_no_texture():
    wrap, none, rays, exp_wrap, exp_none = K.case_cutout_wrap_and_no_texture()
    r = rays.copy()
    assert O.trace(wrap, r, 1, 0, 1000.0, 1, 1)[0] == 0 and r["hits"][0].tolist() == exp_wrap
    r = rays.copy()
    assert O.trace(none, r, 1, 0, 1000.0, 1, 1)[0] == 0 and r["hits"][0].tolist() == exp_none


def test_primary_info_bounce0_and_miss():
    _, sc, rays, n, expected = K.case_single_triangle()
    info = np.zeros((n, 4), np.uint32)
    assert O.trace(sc, rays, n, 0, 1000.0, n, 1, info=info)[0] == 0
    # hit: (mesh_id, tri - TriOffset, asuint(u), asuint(v)) at full precision (:233)
    assert info[0].tolist() == [0, 0, int(np.float32(0.25).view(np.uint32)), int(np.float32(0.25).view(np.uint32))]
    # miss: mesh 0, -1 - MeshData[0].TriOffset, u = v = 0
    assert info[2].tolist() == [0, 0xFFFFFFFF, 0, 0]


def test_primary_info_later_bounce_forms():
    _, sc, rays, n, _ = K.case_single_triangle()
    r = rays.copy()
    r[n:2 * n] = rays[:n]
    colors = np.zeros(n, tthip.COL_DTYPE)
    colors["Data"][:, 3] = [1.0, -1.0, 1.0, 2.0]  # ray 3: Data.w = 2 != CurBounce -> no write
    for flags in (0, tthip.TT_TRACE_USE_RESTIRGI, tthip.TT_TRACE_USE_ASVGF):
        info = np.full((n, 4), 0xABCDEF, np.uint32)
        rr = r.copy()
        assert O.trace(sc, rr, n, 1, 1000.0, n, 1, info=info, colors=colors, flags=flags)[0] == 0
        d = rays["direction"][:n].view(np.uint32)
        if flags == tthip.TT_TRACE_USE_RESTIRGI:
            assert info[0, :3].tolist() == [0, 0, (16383 | (16383 << 16))]
        else:
            assert info[0, :3].tolist() == d[0].tolist()
        assert info[0, 3] == 0
        # miss (ray 2): ASVGF -> direction; otherwise direction * FarPlane + origin
        if flags == tthip.TT_TRACE_USE_ASVGF:
            assert info[2, :3].tolist() == d[2].tolist()
        else:
            pos = (rays["direction"][2] * np.float32(1000.0) + rays["origin"][2]).astype(np.float32)
            assert info[2, :3].tolist() == pos.view(np.uint32).tolist()
        assert info[2, 3] == 1
        assert info[3].tolist() == [0xABCDEF] * 4


def test_zero_rays_and_bad_args():
    _, sc, rays, n, _ = K.case_single_triangle()
    before = rays.copy()
    assert O.trace(sc, rays, 0, 0, 1000.0, n, 1)[0] == 0
    assert np.array_equal(before, rays)
    assert O.trace(sc, rays, 1, 0, 1000.0, 0, 1)[0] == tthip.TT_ERR_INVALID_ARG


def test_out_of_range_material_reads_as_zero():
    """D3D returns zeros for an out-of-range StructuredBuffer read: a triangle whose
    MaterialOffset + MatDat is past _Materials behaves as an unflagged material."""
    sc, rays, exp0, exp1 = K.case_invisible_bounce0()
    sc.tris["MatDat"][1] = 5  # past the 2-entry material buffer: not invisible any more
    r = rays.copy()
    assert O.trace(sc, r, 1, 0, 1000.0, 1, 1)[0] == 0
    assert r["hits"][0].tolist() == exp1


# ------------------------------------------------------------------- any-hit (kernel_shadow)
@pytest.mark.parametrize("case", K.SHADOW_CASES, ids=lambda c: c.__name__)
def test_shadow_kat(case):
    name, sc, rays, expected = case()
    n = len(rays)
    t_in = rays["t"].copy()
    vis = np.full((n, 4), 7.0, np.float32)
    colors = np.zeros(n, tthip.COL_DTYPE)
    nee = np.full((n, 4), 9.0, np.float32)
    st, cnt = O.shadow(sc, rays, n, 0, n, 1, visibility=vis, colors=colors, nee_pos=nee, counts=True)
    assert st == tthip.TT_OK, name
    assert cnt["status"].tolist() == expected, name
    for i, e in enumerate(expected):
        if e == 4:  # occluded: t = 0 in place (IntersectionKernels.compute:449-454), nothing else
            assert rays["t"][i] == 0.0 and vis[i].tolist() == [0, 0, 0, 0]
            assert colors["Direct"][i].tolist() == [0, 0, 0] and nee[i].tolist() == [9, 9, 9, 9]
        else:       # reached |t|: NEEPosA, Direct only for t >= 0 (:461-470)
            assert rays["t"][i] == t_in[i] and vis[i].tolist() == [1, 1, 1, 1]
            o, d = rays["origin"][i], rays["direction"][i]
            assert nee[i].tolist() == (o + d * np.float32(abs(t_in[i]))).tolist() + [0.0]
            want = [1.0, 2.0, 4.0] if t_in[i] >= 0 else [0.0, 0.0, 0.0]
            assert colors["Direct"][i].tolist() == want


def test_shadow_bounce1_no_color_outputs():
    _, sc, rays, expected = K.shadow_case_single_triangle()
    n = len(rays)
    colors = np.zeros(n, tthip.COL_DTYPE)
    nee = np.full((n, 4), 9.0, np.float32)
    st, cnt = O.shadow(sc, rays, n, 1, n, 1, colors=colors, nee_pos=nee, counts=True)
    assert st == 0 and cnt["status"].tolist() == expected
    assert not colors["Direct"].any() and (nee == 9.0).all()


def test_shadow_reps_exhausted_writes_nothing():
    _, sc, _, _, _ = K.case_reps_exhausted()
    rays = hb.shadow_rays([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)], [2.0])
    vis = np.zeros((1, 4), np.float32)
    st, cnt = O.shadow(sc, rays, 1, 0, 1, 1, visibility=vis, counts=True)
    assert st == 0 and cnt["status"][0] == 1 and rays["t"][0] == 2.0 and vis[0].tolist() == [0, 0, 0, -1]


def test_shadow_glass_unsupported():
    _, sc, rays, _ = K.shadow_case_single_triangle()
    sc.materials[0]["specTrans"] = 1.0
    st, _ = O.shadow(sc, rays, len(rays), 0, len(rays), 1)
    assert st == tthip.TT_ERR_UNSUPPORTED


# ------------------------------------------------------------------ TLAS refit (§8 f4)
def _decode_slot_boxes(node):
    """World boxes of the 8 child slots of an 80-B node: p + q * 2^(e-127) per axis."""
    e = [(int(node["e_imask"]) >> (8 * a)) & 0xff for a in range(3)]
    scale = [np.float32(2.0) ** (ea - 127) for ea in e]
    q = {}
    for name in ("qlo_x", "qhi_x", "qlo_y", "qhi_y", "qlo_z", "qhi_z"):
        w = node[name]
        q[name] = [(int(w[k >> 2]) >> (8 * (k & 3))) & 0xff for k in range(8)]
    lo = np.array([[node["p"][0] + q["qlo_x"][k] * scale[0], node["p"][1] + q["qlo_y"][k] * scale[1],
                    node["p"][2] + q["qlo_z"][k] * scale[2]] for k in range(8)])
    hi = np.array([[node["p"][0] + q["qhi_x"][k] * scale[0], node["p"][1] + q["qhi_y"][k] * scale[1],
                    node["p"][2] + q["qhi_z"][k] * scale[2]] for k in range(8)])
    return lo, hi


def _refit_scene(seed, n_inst=60):
    rng = np.random.default_rng(seed)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(seed, 800, 10.0, 0.5)), tthip.trs_matrix((0, 0, 0)),
                  np.zeros(1, tthip.MAT_DTYPE))
    props = [am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(seed * 10 + k, 300)), np.zeros(1, tthip.MAT_DTYPE))
             for k in range(4)]
    for i in range(n_inst):
        am.add_instance(props[i % 4], tthip.trs_matrix(rng.uniform(-30, 30, 3), float(rng.uniform(0, 360)),
                                                       float(rng.uniform(0.5, 2))))
    return am.build()


def test_refit_bounds_every_instance():
    """After the refit (AssetManager.RefitTLAS) every TLAS slot box contains the AABBs of all the
    instances below it (the quantization rounds outward), and BLAS nodes are untouched."""
    sc = _refit_scene(3)
    boxes = sc.meta["mesh_aabbs"].copy()
    boxes[:, :3] += 1.5  # moved: every instance shifted by +1.5 in x, y, z
    boxes[:, 3:] += 1.5
    st, nodes = O.tlas_refit(sc, boxes)
    assert st == 0
    assert np.array_equal(nodes[sc.tlas_nodes:], sc.nodes[sc.tlas_nodes:])

    def meta_of(node):
        return [(int(node["meta"][k >> 2]) >> (8 * (k & 3))) & 0xff for k in range(8)]

    def instances_below(n):
        node, out = nodes[n], []
        for m in meta_of(node):
            if m and (m & 0x1f) >= 24:
                out += instances_below(int(node["base_child"]) + (m & 0x1f) - 24)
            elif m:
                first, cnt = m & 0x1f, bin(m >> 5).count("1")
                out += [int(sc.tlas[t]) for t in range(int(node["base_tri"]) + first, int(node["base_tri"]) + first + cnt)]
        return out

    checked = 0
    for n in range(sc.tlas_nodes):
        node = nodes[n]
        lo, hi = _decode_slot_boxes(node)
        for k, m in enumerate(meta_of(node)):
            if m == 0:
                continue
            if (m & 0x1f) >= 24:
                ids = instances_below(int(node["base_child"]) + (m & 0x1f) - 24)
            else:
                first, cnt = m & 0x1f, bin(m >> 5).count("1")
                ids = [int(sc.tlas[t]) for t in range(int(node["base_tri"]) + first, int(node["base_tri"]) + first + cnt)]
            for i in ids:
                assert (boxes[i, 3:] >= lo[k]).all() and (boxes[i, :3] <= hi[k]).all(), (n, k, i)
                checked += 1
    assert checked >= len(boxes)


def test_refit_traces_like_a_fresh_build():
    """Refit TLAS (reference topology, new boxes) finds the same closest hits as tracing with the
    TLAS built for the same boxes; both are the oracle."""
    sc = _refit_scene(4)
    st, nodes = O.tlas_refit(sc, sc.meta["mesh_aabbs"])
    assert st == 0
    refit = tthip.Scene(nodes, sc.tris, sc.tlas, sc.meshdata, sc.materials, tlas_nodes=sc.tlas_nodes)
    W, H = 64, 48
    c2w, ip = tthip.unity_camera((0, 10, 50), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, 1000.0)
    a = O.generate(c2w, ip, W, H, 0.3, 1000.0)
    b = a.copy()
    assert O.trace(sc, a, W * H, 0, 1000.0, W, H, nthreads=8)[0] == 0
    assert O.trace(refit, b, W * H, 0, 1000.0, W, H, nthreads=8)[0] == 0
    assert np.array_equal(a["hits"][: W * H, :3], b["hits"][: W * H, :3])
    assert (a["hits"][: W * H, 1] != 0xFFFFFFFF).sum() > W * H // 4


def test_degenerate_rays_are_deterministic_on_the_oracle():
    """Zero / NaN / infinite / denormal ray components: the oracle finishes every ray (hit, miss or
    Reps exhaustion), single- and multi-threaded runs agree bit for bit."""
    from test_gpu_parity import degenerate_rays

    sc = tthip.single_object_scene(tthip.Mesh.soup(3, 2000, 1.0, 0.15))
    n = 2048
    rays = degenerate_rays(n, 5)
    a, b = rays.copy(), rays.copy()
    st1, c1 = O.trace(sc, a, n, 0, 1000.0, n, 1, counts=True, nthreads=1)
    st2, c2 = O.trace(sc, b, n, 0, 1000.0, n, 1, counts=True, nthreads=4)
    assert st1 == st2 == 0
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)) and np.array_equal(c1, c2)
    assert set(np.unique(c1["status"]).tolist()) <= {0, 1}


def test_shadow_glass_tint_kat():
    """Stained-glass shadows (CommonData.cginc:613-625): known throughputs, visibility xyz and
    GlobalColors.Direct = 0.5 + illumination * throughput, bit for bit."""
    name, sc, rays, expected, thr = K.shadow_case_glass()
    n = len(rays)
    rays["illumination"] = (0.75, 1.5, 3.0)
    rays["PixelIndex"] = np.arange(n)
    vis = np.full((n, 4), 7.0, np.float32)
    colors = np.zeros(n, tthip.COL_DTYPE)
    colors["Direct"] = 0.5
    st, cnt = O.shadow(sc, rays, n, 0, n, 1, visibility=vis, colors=colors, counts=True)
    assert st == tthip.TT_OK
    assert cnt["status"].tolist() == expected
    for i, e in enumerate(expected):
        if e == 0:
            assert vis[i].tobytes() == np.append(thr[i], np.float32(1.0)).astype(np.float32).tobytes(), i
            want = np.float32(0.5) + np.asarray((0.75, 1.5, 3.0), np.float32) * thr[i]
            assert colors["Direct"][i].astype(np.float32).tobytes() == want.astype(np.float32).tobytes(), i
    assert not np.array_equal(thr[0], np.ones(3, np.float32))


def test_shadow_glass_needs_texture_atlas():
    _, sc, rays, _, _ = K.shadow_case_glass()
    sc.texture_atlas = None
    st, _ = O.shadow(sc, rays, len(rays), 0, len(rays), 1)
    assert st == tthip.TT_ERR_UNSUPPORTED
