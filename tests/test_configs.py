"""CPU checks of the BASELINE.json config generators (``ttconfigs``): shape
(instance/mesh counts, triangle budgets, the San-Miguel foliage share), determinism, and that
each view sees its scene (oracle at thumbnail size). The full-size GPU parity runs are in
test_gpu_configs.py."""
import numpy as np

import oracle_ctypes as O
import ttconfigs as T
import tthip

FAR = T.FAR


def _thumb(sc, view, W=96, H=54):
    c2w, ip = view.camera(W, H)
    rays = O.generate(c2w, ip, W, H, T.NEAR, FAR)
    st, cnt = O.trace(sc, rays, W * H, 0, FAR, W, H, counts=True, nthreads=8)
    assert st == 0
    hit = rays["hits"][: W * H, 1] != 0xFFFFFFFF
    return hit.mean(), cnt


def test_c1_cornell_shape():
    sc = T.c1_cornell()
    assert len(sc.tris) == 12 and len(sc.meshdata) == 1
    frac, _ = _thumb(sc, T.C1_VIEW)
    assert frac > 0.5


def test_c4_bistro_small_two_level_shape_and_determinism():
    a = T.c4_bistro(n_unique=24, n_instances=96, max_tris=4000)
    b = T.c4_bistro(n_unique=24, n_instances=96, max_tris=4000)
    assert len(a.meshdata) == 1 + 96 and len(a.tlas) == 1 + 96
    assert np.array_equal(a.nodes.view(np.uint8), b.nodes.view(np.uint8))
    assert np.array_equal(a.tris.view(np.uint8), b.tris.view(np.uint8))
    assert np.array_equal(a.meshdata.view(np.uint8), b.meshdata.view(np.uint8))
    # every instance's W2L is rigid + uniform scale: the 3x3 block is s * R
    m = a.meshdata["W2L"].reshape(-1, 4, 4)[1:]  # column-major -> rows are columns
    g = np.einsum("nij,nkj->nik", m[:, :3, :3], m[:, :3, :3])
    s2 = g[:, 0, 0]
    assert np.allclose(g, s2[:, None, None] * np.eye(3)[None], rtol=1e-4, atol=1e-6)
    frac, cnt = _thumb(a, T.C4_VIEW)
    assert 0.5 < frac < 1.0  # street + props below, sky down the street
    assert cnt["blas_entries"].sum() > 0


def test_c5_san_miguel_reduced_shape():
    sc = T.c5_san_miguel(n_tris=1_000_000)
    assert len(sc.tris) == 1_000_000 and len(sc.meshdata) == 1
    foliage = float((sc.tris["MatDat"] == 7).mean())
    assert 0.5 <= foliage <= 0.7, foliage
    frac, cnt = _thumb(sc, T.C5_VIEW)
    assert frac > 0.7
    assert cnt["node_visits"].mean() > 8


def test_generators_reject_bad_sizes():
    import pytest

    with pytest.raises(tthip.TTError):
        tthip.Mesh.san_miguel(1, 1000)
    with pytest.raises(tthip.TTError):
        tthip.Mesh.ground(1.0, 0.0, 0.0, 1.0, 4, 4)


def test_raw_dump_for_csharp_baseline(tmp_path):
    """tools/dump_scene_raw.py writes the byte-exact buffers ScalarTraversal.cs reads, and the
    word offsets that file hard-codes match the C ABI layouts."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import dump_scene_raw as D

    sc, rays, ref = D.dump(str(tmp_path), "c1", 32, 24, threads=2)
    assert (tmp_path / "nodes.bin").stat().st_size == 80 * len(sc.nodes)
    assert (tmp_path / "tris.bin").stat().st_size == 88 * len(sc.tris)
    assert (tmp_path / "meshdata.bin").stat().st_size == 88 * len(sc.meshdata)
    assert (tmp_path / "materials.bin").stat().st_size == 252 * len(sc.materials)
    hits = np.fromfile(tmp_path / "expected_hits.bin", np.uint32).reshape(-1, 4)
    assert np.array_equal(hits, ref["hits"][: 32 * 24])
    assert (tmp_path / "params.txt").read_text().split()[:2] == [str(32 * 24), "0"]
    # word offsets used by ScalarTraversal.cs
    md, mat, tri = tthip.MESH_DTYPE, tthip.MAT_DTYPE, tthip.TRI_DTYPE
    assert [md.fields[k][1] // 4 for k in ("TriOffset", "NodeOffset", "MaterialOffset", "mesh_data_bvh_offsets")] == \
        [16, 17, 18, 19]
    assert mat.fields["Tag"][1] // 4 == 23 and mat.fields["MatType"][1] // 4 == 25 and mat.itemsize == 63 * 4
    assert tri.fields["MatDat"][1] // 4 == 21 and tri.itemsize == 22 * 4
