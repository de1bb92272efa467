"""Builder restatement (BVH2Builder / BVH8Builder / Aggregate / ParentObject / AssetManager):
structural invariants of the buffers the trace kernel consumes, and the host-side validator."""
import ctypes as C

import numpy as np
import pytest

import handbuilt as hb
import kat_cases as K
import tthip


def decode_nodes(nodes):
    """Per node: list of (slot, kind, ...) decoded from the 80-byte layout."""
    out = []
    for n in nodes:
        meta = [(int(n["meta"][k >> 2]) >> ((k & 3) * 8)) & 0xFF for k in range(8)]
        e = [int(n["e_imask"]) & 0xFF, (int(n["e_imask"]) >> 8) & 0xFF, (int(n["e_imask"]) >> 16) & 0xFF]
        imask = int(n["e_imask"]) >> 24

        def q(arr, k):
            return (int(arr[k >> 2]) >> ((k & 3) * 8)) & 0xFF

        kids = []
        for k in range(8):
            m = meta[k]
            lo = [q(n["qlo_x"], k), q(n["qlo_y"], k), q(n["qlo_z"], k)]
            hi = [q(n["qhi_x"], k), q(n["qhi_y"], k), q(n["qhi_z"], k)]
            if (m & 0x18) == 0x18:
                kids.append(("inner", k, m & 0x1F, lo, hi))
            elif m >> 5:
                kids.append(("leaf", k, m, lo, hi))
        out.append((n["p"].astype(np.float64), e, imask, int(n["base_child"]), int(n["base_tri"]), kids))
    return out


def check_blas(nodes, tris, padded_aabbs=None):
    dec = decode_nodes(nodes)
    seen = np.zeros(len(tris), np.int32)
    for p, e, imask, bc, bt, kids in dec:
        scale = np.array([2.0 ** (x - 127) for x in e])
        n_inner = sum(1 for k in kids if k[0] == "inner")
        assert imask == (1 << n_inner) - 1
        ntri = 0
        inner_seen = []
        for kind, slot, m, lo, hi in kids:
            bmin, bmax = p + np.array(lo) * scale, p + np.array(hi) * scale
            if kind == "inner":
                inner_seen.append(m - 24)
            else:
                cnt = bin(m >> 5).count("1")
                assert (m >> 5) in (1, 3, 7) and cnt <= 3
                off = m & 0x1F
                ntri += cnt
                for j in range(cnt):
                    t = bt + off + j
                    seen[t] += 1
                    tr = tris[t]
                    v = np.stack([tr["pos0"], tr["pos0"] + tr["posedge1"], tr["pos0"] + tr["posedge2"]]).astype(np.float64)
                    # quantized child box is conservative for the triangle (floor/ceil quantization)
                    assert (v.min(0) >= bmin - 1e-4 * (1 + np.abs(bmin))).all()
                    assert (v.max(0) <= bmax + 1e-4 * (1 + np.abs(bmax))).all()
        assert ntri <= 24
        assert sorted(inner_seen) == list(range(n_inner))
    assert (seen == 1).all(), "every triangle referenced by exactly one leaf"


def test_cornell_blas():
    b = tthip.Blas(tthip.Mesh.cornell())
    nodes, tris = b.arrays()
    assert b.n_tris == 12
    check_blas(nodes, tris)


@pytest.mark.parametrize("seed,n", [(1, 100), (2, 3000), (3, 20000)])
def test_soup_blas(seed, n):
    b = tthip.Blas(tthip.Mesh.soup(seed, n, 1.0, 0.05))
    nodes, tris = b.arrays()
    assert b.n_tris == n
    check_blas(nodes, tris)


def test_builder_deterministic():
    a = tthip.Blas(tthip.Mesh.soup(5, 5000, 2.0, 0.1)).arrays()
    b = tthip.Blas(tthip.Mesh.soup(5, 5000, 2.0, 0.1)).arrays()
    assert a[0].tobytes() == b[0].tobytes() and a[1].tobytes() == b[1].tobytes()


def test_winding_and_edges():
    # ParentObject.cs:1002-1004: V1 = idx[i], V2 = idx[i+2], V3 = idx[i+1]; edges V2-V1, V3-V1
    pos = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0]], np.float32)
    m = tthip.Mesh.from_arrays(pos, np.array([0, 1, 2], np.int32))
    _, tris = tthip.Blas(m).arrays()
    assert tris[0]["pos0"].tolist() == [0, 0, 0]
    assert tris[0]["posedge1"].tolist() == [0, 2, 0]
    assert tris[0]["posedge2"].tolist() == [1, 0, 0]


def test_pack_octahedral_known_values():
    L = tthip.scene_lib()
    assert L.tt_pack_octahedral(0.0, 0.0, 1.0) == 32767 | (32767 << 16)
    assert L.tt_pack_octahedral(0.0, 0.0, -1.0) == 65535 | (65535 << 16)
    assert L.tt_pack_octahedral(1.0, 0.0, 0.0) == 65535 | (32767 << 16)
    assert L.tt_pack_octahedral(-1.0, 0.0, 0.0) == 0 | (32767 << 16)


def test_dotnet_sort_is_a_sort():
    rng = np.random.default_rng(0)
    for n in (1, 2, 3, 10, 16, 17, 100, 5000):
        keys = rng.integers(0, 7, n).astype(np.float32)  # many ties
        items = np.arange(n, dtype=np.int32)
        tthip.scene_lib().tt_dotnet_sort_by_key(items.ctypes.data, n, keys.ctypes.data)
        assert sorted(items.tolist()) == list(range(n))
        assert (np.diff(keys[items]) >= 0).all()
    # partitions of <= 16 use insertion sort, which is stable
    keys = np.array([1, 0, 1, 0, 1, 0], np.float32)
    items = np.arange(6, dtype=np.int32)
    tthip.scene_lib().tt_dotnet_sort_by_key(items.ctypes.data, 6, keys.ctypes.data)
    assert items.tolist() == [1, 3, 5, 0, 2, 4]


def test_bvh2_layout():
    rng = np.random.default_rng(1)
    n = 300
    c = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    aabbs = np.concatenate([c + 0.01, c - 0.01], 1).astype(np.float32)  # {max, min}
    fi = np.zeros(n, np.int32)
    na = np.zeros((2 * n, 6), np.float32)
    nl = np.zeros(2 * n, np.int32)
    nc = np.zeros(2 * n, np.uint32)
    assert tthip.scene_lib().tt_bvh2_build(aabbs.ctypes.data, n, fi.ctypes.data, na.ctypes.data, nl.ctypes.data,
                                           nc.ctypes.data) == 0
    assert sorted(fi.tolist()) == list(range(n))
    assert nc[1] == 0 and (na[1] == 0).all()  # node 1 unused (nodeIndex starts at 2)
    leaves = []

    def walk(i):
        if nc[i] > 0:
            assert nc[i] == 1
            leaves.append(fi[nl[i]])
            return
        for ch in (nl[i], nl[i] + 1):
            assert (na[ch][:3] <= na[i][:3] + 1e-6).all() and (na[ch][3:] >= na[i][3:] - 1e-6).all()
            walk(ch)

    walk(0)
    assert sorted(leaves) == list(range(n))


def test_assembly_layout_with_instances():
    am = tthip.AssetManager()
    b0 = tthip.Blas(tthip.Mesh.soup(11, 500, 1.0, 0.1))
    b1 = tthip.Blas(tthip.Mesh.soup(12, 300, 1.0, 0.1))
    am.add_parent(b0, tthip.trs_matrix((0, 0, 0)), np.zeros(3, tthip.MAT_DTYPE))
    ip = am.add_instance_parent(b1, np.zeros(2, tthip.MAT_DTYPE))
    for k in range(4):
        am.add_instance(ip, tthip.trs_matrix((3.0 * (k + 1), 0, 0), 30.0 * k, 1.0 + 0.25 * k))
    sc = am.build()
    n_mesh = 1 + 4
    assert len(sc.meshdata) == n_mesh and len(sc.tlas) == n_mesh
    assert sc.tlas_nodes <= 2 * n_mesh
    # BLAS of the parent starts at 2*(P+I) (AssetManager.cs:995), then the instance parent's
    assert sc.meshdata["NodeOffset"][0] == 2 * n_mesh == sc.meshdata["mesh_data_bvh_offsets"][0]
    assert (sc.meshdata["NodeOffset"][1:] == 2 * n_mesh + b0.n_nodes).all()
    assert (sc.meshdata["TriOffset"][1:] == b0.n_tris).all() and sc.meshdata["TriOffset"][0] == 0
    assert sc.meshdata["MaterialOffset"].tolist() == [0, 3, 3, 3, 3]
    assert sorted(sc.tlas.tolist()) == list(range(n_mesh))
    assert len(sc.nodes) == 2 * n_mesh + b0.n_nodes + b1.n_nodes
    # W2L is the inverse of each instance's localToWorld, Unity column-major
    w2l = sc.meshdata["W2L"][2].reshape(4, 4).T
    assert np.allclose(w2l @ tthip.trs_matrix((6.0, 0, 0), 30.0, 1.25), np.eye(4), atol=1e-5)
    assert tthip.validate(sc)[0] == tthip.TT_OK


def test_validator_accepts_builder_scenes_and_kats():
    assert tthip.validate(tthip.single_object_scene(tthip.Mesh.cornell()))[0] == tthip.TT_OK
    for case in K.ALL_CASES:
        sc = case()[1]
        assert tthip.validate(sc)[0] == tthip.TT_OK, case.__name__


def test_validator_rejects_malformed():
    sc = tthip.single_object_scene(tthip.Mesh.soup(3, 200, 1.0, 0.1))
    bad = tthip.Scene(sc.nodes.copy(), sc.tris, sc.tlas, sc.meshdata, sc.materials)
    bad.nodes[2]["base_child"] = 10 ** 6
    st, why = tthip.validate(bad)
    assert st == tthip.TT_ERR_INVALID_ARG and "node index" in why
    bad = tthip.Scene(sc.nodes, sc.tris[:10].copy(), sc.tlas, sc.meshdata, sc.materials)
    st, why = tthip.validate(bad)
    assert st == tthip.TT_ERR_INVALID_ARG and "triangle" in why
    bad = tthip.Scene(sc.nodes, sc.tris, np.array([5], np.int32), sc.meshdata, sc.materials)
    assert tthip.validate(bad)[0] == tthip.TT_ERR_INVALID_ARG
    bad = tthip.Scene(sc.nodes, sc.tris, sc.tlas, sc.meshdata, sc.materials.copy())
    bad.materials[0]["MatType"] = tthip.MAT_CUTOUT_INDEX  # structurally valid (needs an atlas to trace)
    assert tthip.validate(bad)[0] == tthip.TT_OK
    # a leaf meta whose triangle bits would spill into the internal-child bits 24..31
    nodes = sc.nodes.copy()
    meta = int(nodes[2]["meta"][0]) & ~0xFF
    nodes[2]["meta"][0] = meta | (0b111 << 5) | 23
    assert tthip.validate(tthip.Scene(nodes, sc.tris, sc.tlas, sc.meshdata, sc.materials))[0] == tthip.TT_ERR_INVALID_ARG


def test_parallel_build_identical_to_serial(monkeypatch):
    """Large meshes build their top BVH2 subtrees, the three per-axis presorts, the top SAH sweeps
    (>= 2^20 primitives) and the BVH8 cost pass on several threads; the sequential depth-first node
    numbering is kept (a subtree of k primitives takes 2(k-1) slots), so nodes, leaf-ordered
    triangles and the leaf map must equal the single-threaded build (TT_BUILD_SERIAL) byte for byte."""
    mesh = tthip.Mesh.soup(77, (1 << 20) + 4096, 4.0, 0.02)
    par = tthip.Blas(mesh)
    monkeypatch.setenv("TT_BUILD_SERIAL", "1")
    ser = tthip.Blas(mesh)
    (pn, pt), (sn, st) = par.arrays(), ser.arrays()
    assert par.info.n_nodes == ser.info.n_nodes and par.info.bvh2_depth == ser.info.bvh2_depth
    assert np.array_equal(pn.view(np.uint8), sn.view(np.uint8))
    assert np.array_equal(pt.view(np.uint8), st.view(np.uint8))
    assert np.array_equal(par.leaf_order(), ser.leaf_order())
