"""The reference's compile-time trace variants IgnoreGlassMain and IgnoreBackfacing
(IntersectionKernels.compute:42-47, GlobalDefines.cginc:4,11), exposed as the launch flags
TT_TRACE_IGNORE_GLASS / TT_TRACE_IGNORE_BACKFACING: oracle known answers on hand-built scenes (the
expected hits follow from the geometry, not from the oracle). GPU parity of the same flags is in
test_gpu_parity.py (test_trace_variant_flags_random_soup)."""
import numpy as np
import pytest

import oracle_ctypes as O
import tthip

FAR = 1000.0


def quad(z, flip=False):
    p = np.array([[-1, -1, z], [1, -1, z], [1, 1, z], [-1, 1, z]], np.float32)
    idx = np.array([[0, 1, 2], [0, 2, 3]], np.int32)
    if flip:
        idx = idx[:, [0, 2, 1]]
    return p, idx


def two_quads(near_flip, far_flip, near_mat, far_mat, n_mat=2):
    p0, i0 = quad(1.0, near_flip)
    p1, i1 = quad(0.0, far_flip)
    pos = np.concatenate([p0, p1])
    idx = np.concatenate([i0, i1 + 4])
    mat = np.array([near_mat, near_mat, far_mat, far_mat], np.int32)
    sc = tthip.single_object_scene(tthip.Mesh.from_arrays(pos, idx, mat), n_materials=n_mat)
    return sc


def ray_down(n=1):
    r = np.zeros(n, tthip.RAY_DTYPE)
    r["origin"] = [0.1, 0.2, 5.0]
    r["direction"] = [0.0, 0.0, -1.0]
    r["hits"][:, 1] = 0xFFFFFFFF
    r["hits"][:, 2] = np.array([FAR], np.float32).view(np.uint32)[0]
    return r


def trace_t(sc, flags, bounce=0):
    r = ray_down(2)  # bounce 1 reads the second half (W*H = 1)
    st, _ = O.trace(sc, r, 1, bounce, FAR, 1, 1, flags=flags)
    assert st == 0
    return float(r["hits"][bounce, 2:3].view(np.float32)[0])


def test_ignore_glass_skips_specTrans_1():
    sc = two_quads(False, False, near_mat=1, far_mat=0)
    sc.materials[1]["specTrans"] = 1.0
    assert trace_t(sc, 0) == pytest.approx(4.0)
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_GLASS) == pytest.approx(5.0)
    sc.materials[1]["specTrans"] = 0.999
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_GLASS) == pytest.approx(4.0)


def reference_backfacing(sc, tri, d):
    """dot(normalize(cross(normalize(e1), normalize(e2))), d) <= 0 in float64 (sign only)."""
    t = sc.tris[tri]
    e1, e2 = t["posedge1"].astype(np.float64), t["posedge2"].astype(np.float64)
    n = np.cross(e1 / np.linalg.norm(e1), e2 / np.linalg.norm(e2))
    return float(np.dot(n, d)) <= 0.0


@pytest.mark.parametrize("near_flip", [False, True])
def test_ignore_backfacing_bounce0_only(near_flip):
    sc = two_quads(near_flip, not near_flip, 0, 0)
    near = [i for i in range(4) if abs(sc.tris[i]["pos0"][2] - 1.0) < 1e-6]
    skip_near = reference_backfacing(sc, near[0], np.array([0.0, 0.0, -1.0]))
    assert all(reference_backfacing(sc, i, np.array([0.0, 0.0, -1.0])) == skip_near for i in near)
    assert trace_t(sc, 0) == pytest.approx(4.0)
    got = trace_t(sc, tthip.TT_TRACE_IGNORE_BACKFACING)
    if skip_near:  # the far quad has the opposite winding, so it is front-facing by this test
        assert got == pytest.approx(5.0)
    else:
        assert got == pytest.approx(4.0)
    # bounce > 0: the variant only applies at CurBounce == 0
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_BACKFACING, bounce=1) == pytest.approx(4.0)


def test_ignore_backfacing_spares_glass_and_counts_out_of_range_materials():
    sc = two_quads(True, True, near_mat=1, far_mat=5, n_mat=2)  # far quad's material out of range
    near = [i for i in range(4) if abs(sc.tris[i]["pos0"][2] - 1.0) < 1e-6]
    assert reference_backfacing(sc, near[0], np.array([0.0, 0.0, -1.0]))
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_BACKFACING) == FAR  # both quads skipped (zeros: specTrans 0)
    sc.materials[1]["specTrans"] = 1.0  # glass is exempt from the backfacing test
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_BACKFACING) == pytest.approx(4.0)
    assert trace_t(sc, tthip.TT_TRACE_IGNORE_BACKFACING | tthip.TT_TRACE_IGNORE_GLASS) == FAR
