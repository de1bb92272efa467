"""The BLAS build in stages (include/truetrace_scene.h): tt_blas_prepare_aabbs -> a BVH2 ->
tt_blas_build_from_bvh2 reproduces tt_blas_build exactly when the BVH2 is the host's, and rejects a
malformed BVH2 instead of walking it. (The GPU BVH2 stage plugs into the same entry point:
tests/test_gpu_builder.py.)"""
import numpy as np
import pytest

import tthip


def _stages(mesh):
    L = tthip.scene_lib()
    v = mesh.view()
    n = v.n_indices // 3
    aabbs = np.zeros((n, 6), np.float32)
    assert L.tt_blas_prepare_aabbs(v, aabbs.ctypes.data) == 0
    bvh2 = [np.zeros(n, np.int32), np.zeros((2 * n, 6), np.float32), np.zeros(2 * n, np.int32), np.zeros(2 * n, np.uint32)]
    assert L.tt_bvh2_build(aabbs.ctypes.data, n, *[a.ctypes.data for a in bvh2]) == 0
    return L, v, aabbs, bvh2


def _from_bvh2(L, v, bvh2, depth):
    h = tthip.C.c_void_p()
    st = L.tt_blas_build_from_bvh2(v, *[a.ctypes.data for a in bvh2], depth, tthip.C.byref(h))
    return st, h


@pytest.mark.parametrize("mesh_fn", [tthip.Mesh.cornell, lambda: tthip.Mesh.soup(3, 20_000),
                                     lambda: tthip.Mesh.prop(4, 30_000)])
def test_staged_build_equals_blas_build(mesh_fn):
    mesh = mesh_fn()
    ref = tthip.Blas(mesh)
    L, v, aabbs, bvh2 = _stages(mesh)
    st, h = _from_bvh2(L, v, bvh2, ref.info.bvh2_depth)
    assert st == 0
    got = tthip.Blas.__new__(tthip.Blas)
    got.h = h.value
    got.info = tthip.BlasInfo()
    L.tt_blas_get_info(got.h, tthip.C.byref(got.info))
    for a, b in zip(ref.arrays(), got.arrays()):
        assert a.tobytes() == b.tobytes()
    assert np.array_equal(ref.leaf_order(), got.leaf_order())
    assert got.info.bvh2_depth == ref.info.bvh2_depth


def test_presort_is_the_dotnet_sort_of_the_centroids():
    mesh = tthip.Mesh.soup(5, 5_000)
    L, v, aabbs, _ = _stages(mesh)
    n = len(aabbs)
    pre = np.zeros((3, n), np.int32)
    assert L.tt_bvh2_presort(aabbs.ctypes.data, n, pre.ctypes.data) == 0
    for d in range(3):
        c = ((aabbs[:, d] - aabbs[:, 3 + d]) / np.float32(2.0) + aabbs[:, 3 + d]).astype(np.float32)
        items = np.arange(n, dtype=np.int32)
        L.tt_dotnet_sort_by_key(items.ctypes.data, n, c.ctypes.data)
        assert np.array_equal(items, pre[d])
        assert np.all(np.diff(c[pre[d]]) >= 0)


def test_malformed_bvh2_is_rejected():
    mesh = tthip.Mesh.soup(9, 500)  # (v points into the mesh's arrays)
    L, v, aabbs, bvh2 = _stages(mesh)
    fi, boxes, left, count = bvh2
    bad = [a.copy() for a in bvh2]
    bad[2][0] = 0  # root points at itself: a cycle
    assert _from_bvh2(L, v, bad, 1)[0] != 0
    bad = [a.copy() for a in bvh2]
    bad[0][0] = bad[0][1]  # FinalIndices not a permutation
    assert _from_bvh2(L, v, bad, 1)[0] != 0
    bad = [a.copy() for a in bvh2]
    leaf = int(np.nonzero(count == 1)[0][0])
    bad[2][leaf] = 10 ** 6  # leaf position out of range
    assert _from_bvh2(L, v, bad, 1)[0] != 0


@pytest.mark.parametrize("mesh_fn", [tthip.Mesh.cornell, lambda: tthip.Mesh.prop(4, 80_000)])
def test_prepared_handle_reassembles_the_host_blas(mesh_fn):
    """tt_blas_prepare + tt_blas_build_from_cwbvh_prepared (the device build's assembly, triangles
    prepared once) over the host build's own nodes and leaf order reproduce it byte for byte; a
    leaf order that is not a permutation is rejected, and the handle is consumed either way."""
    mesh = mesh_fn()
    ref = tthip.Blas(mesh)
    nodes, tris = ref.arrays()
    cw = np.argsort(ref.leaf_order()).astype(np.int32)  # leaf position -> source triangle
    L = tthip.scene_lib()
    v = mesh.view()
    n = v.n_indices // 3
    aabbs = np.zeros((n, 6), np.float32)
    ref_aabbs = np.zeros((n, 6), np.float32)
    assert L.tt_blas_prepare_aabbs(v, ref_aabbs.ctypes.data) == 0
    prep = tthip.C.c_void_p()
    assert L.tt_blas_prepare(v, aabbs.ctypes.data, tthip.C.byref(prep)) == 0
    assert np.array_equal(aabbs.view(np.uint32), ref_aabbs.view(np.uint32))
    h = tthip.C.c_void_p()
    assert L.tt_blas_build_from_cwbvh_prepared(prep, nodes.ctypes.data, len(nodes), cw.ctypes.data,
                                               ref.info.bvh2_depth, tthip.C.byref(h)) == 0
    got = tthip.Blas.__new__(tthip.Blas)
    got.h = h.value
    got.info = tthip.BlasInfo()
    L.tt_blas_get_info(got.h, tthip.C.byref(got.info))
    for a, b in zip((nodes, tris), got.arrays()):
        assert a.tobytes() == b.tobytes()
    assert np.array_equal(ref.leaf_order(), got.leaf_order())
    bad = cw.copy()
    bad[-1] = bad[0]  # a duplicate: not a permutation
    prep2 = tthip.C.c_void_p()
    assert L.tt_blas_prepare(v, aabbs.ctypes.data, tthip.C.byref(prep2)) == 0
    h2 = tthip.C.c_void_p()
    assert L.tt_blas_build_from_cwbvh_prepared(prep2, nodes.ctypes.data, len(nodes), bad.ctypes.data,
                                               ref.info.bvh2_depth, tthip.C.byref(h2)) == tthip.TT_ERR_INVALID_ARG


def test_a_mesh_view_keeps_its_mesh_alive():
    """A tt_mesh_input view points into its mesh's native arrays: it must keep the mesh alive after the caller's
    last reference to the mesh is gone (the intermittent use-after-free of round 6)."""
    import gc

    v = tthip.Mesh.soup(21, 2_000).view()  # the only reference to the mesh is the view's
    gc.collect()
    for _ in range(50):  # churn the allocator so freed arrays would be reused
        tthip.Mesh.soup(22, 2_000)
    n = v.n_indices // 3
    a = np.zeros((n, 6), np.float32)
    b = np.zeros((n, 6), np.float32)
    L = tthip.scene_lib()
    assert L.tt_blas_prepare_aabbs(v, a.ctypes.data) == 0
    assert L.tt_blas_prepare_aabbs(tthip.Mesh.soup(21, 2_000).view(), b.ctypes.data) == 0
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
