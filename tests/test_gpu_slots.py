"""Frame slots with TLASes of their own (tt_ctx_share_blas): the reference refits the TLAS and rewrites every
_MeshData record each frame before it traces (AssetManager.cs:1767-1826); a frame slot does that on its own
TLAS copy over the lender's shared BLASes. Every slot's records must equal the oracle on the scene as that slot
holds it (its TLAS nodes read back, its _MeshData, the shared BLAS nodes and triangles), whatever the lender and
the other slots do meanwhile; the lender's BLAS-side updates reach every slot."""
import numpy as np
import pytest

import oracle_ctypes as O
import tthip
from parity_util import CPU_THREADS, FAR
from test_gpu_parity import refit_scene

pytestmark = pytest.mark.gpu

W, H = 192, 108


def _rays():
    c2w, ip = tthip.unity_camera((0, 8, 45), (0, -0.2, -1), (0, 1, 0), 70, W, H, 0.3, FAR)
    return O.generate(c2w, ip, W, H, 0.3, FAR, jitter=1, frames=3, max_bounce=1)


def _scene_of(e, base, meshdata):
    """The scene as context e traces it: its nodes read back (its own TLAS on a slot), its _MeshData."""
    return tthip.Scene(e.scene_nodes(0, len(base.nodes)), base.tris, base.tlas, meshdata, base.materials,
                       tlas_nodes=base.tlas_nodes)


def _check(e, sc, rays, bounce_too=True):
    """e's primary (+ bounce-1) records against the oracle on sc."""
    n = W * H
    rg, rc = rays.copy(), rays.copy()
    ig, ic = np.zeros((n, 4), np.uint32), np.zeros((n, 4), np.uint32)
    e.trace(rg, n, 0, FAR, W, H, info=ig)
    assert O.trace(sc, rc, n, 0, FAR, W, H, info=ic, nthreads=CPU_THREADS)[0] == 0
    assert np.array_equal(rg["hits"][:n], rc["hits"][:n]) and np.array_equal(ig, ic)
    if bounce_too:
        nb = e.enqueue_bounce(rg, n, 0, FAR, W, H, frames=3, max_bounce=1)
        assert O.enqueue_bounce(sc, rc, n, 0, FAR, W, H, frames=3, max_bounce=1) == nb
        e.trace(rg, nb, 1, FAR, W, H)
        assert O.trace(sc, rc, nb, 1, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
        assert np.array_equal(rg["hits"][n:n + nb], rc["hits"][n:n + nb])
    return rg["hits"][:n].copy()


def _pose(a, seed, scale=1.5):
    """_MeshData and instance boxes of scene `a` with every instance but the static parent moved."""
    rng = np.random.default_rng(seed)
    md = a.meshdata.copy()
    boxes = np.ascontiguousarray(a.meta["mesh_aabbs"], np.float32).copy()
    for i in range(1, len(md)):
        d = rng.normal(0, scale, 3)
        w2l = md["W2L"][i].astype(np.float64).reshape(4, 4).T
        shift = np.eye(4)
        shift[:3, 3] = -d
        md["W2L"][i] = tthip.unity_colmajor(w2l @ shift)
        boxes[i, 0:3] += d.astype(np.float32)
        boxes[i, 3:6] += d.astype(np.float32)
    return md, boxes


def test_frame_slot_tlases_are_independent():
    a = refit_scene(41)
    rays = _rays()
    lender = tthip.Engine(0)
    slots = [tthip.Engine(0) for _ in range(2)]
    try:
        lender.upload(a)
        for s in slots:
            s.share_blas(lender, a.tlas_nodes)
        base_hits = _check(lender, a, rays)
        for s in slots:  # a fresh slot traces the lender's scene as it was
            assert np.array_equal(_check(s, a, rays), base_hits)
        # slot 0 moves every instance (the reference's per-frame update: all records + TLAS refit)
        md_b, box_b = _pose(a, 5)
        slots[0].update_meshdata(0, md_b)
        slots[0].tlas_refit(a.tlas_nodes, box_b)
        st, want = O.tlas_refit(a, box_b)
        assert st == 0
        sc0 = _scene_of(slots[0], a, md_b)
        assert np.array_equal(sc0.nodes, want), "the slot's refit TLAS equals the oracle's refit"
        moved = _check(slots[0], sc0, rays)
        assert not np.array_equal(moved, base_hits)
        # the lender and the other slot still trace the original pose
        assert np.array_equal(_check(lender, a, rays), base_hits)
        assert np.array_equal(_check(slots[1], a, rays), base_hits)
        assert np.array_equal(lender.scene_nodes(0, a.tlas_nodes), a.nodes[:a.tlas_nodes])
        # the lender moves the other way: only its own TLAS changes
        md_c, box_c = _pose(a, 9)
        lender.update_meshdata(0, md_c)
        lender.tlas_refit(a.tlas_nodes, box_c)
        _check(lender, _scene_of(lender, a, md_c), rays)
        assert np.array_equal(_check(slots[0], sc0, rays), moved)
        assert np.array_equal(_check(slots[1], a, rays), base_hits)
        # a slot's host-side TLAS rewrite (BVH8AggregatedBuffer.SetData of the TLAS region) on its own nodes
        slots[1].update_meshdata(0, md_b)
        slots[1].update_nodes(0, want[:a.tlas_nodes])
        assert np.array_equal(_check(slots[1], sc0, rays), moved)
    finally:
        lender.close()


def test_frame_slot_sees_the_lenders_blas_refit():
    """A BLAS-side update through the lender (a deforming mesh, ParentObject.RefitMesh) reaches the slots,
    ordered against their launches by the library."""
    from test_blas_refit import deform, two_mesh_scene, vertex_buffer

    sc, mesh, blas = two_mesh_scene(seed=13, n=4000)
    pos, nrm, idx = mesh.arrays()
    leaf = blas.leaf_order()
    c2w, ip = tthip.unity_camera((1.0, 3.0, 14.0), (0, -0.15, -1), (0, 1, 0), 60, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    lender, slot = tthip.Engine(0), tthip.Engine(0)
    try:
        lender.upload(sc)
        slot.share_blas(lender, sc.tlas_nodes)
        V = vertex_buffer(deform(pos, 0.7), nrm)
        lender.blas_refit(1, V, idx, leaf)
        st, nodes, tris = O.blas_refit(sc, 1, V, idx, leaf)
        assert st == 0
        # the slot's TLAS is its copy of the lender's at share time; the BLAS nodes and triangles are shared
        sc2 = tthip.Scene(nodes, tris, sc.tlas, sc.meshdata, sc.materials, tlas_nodes=sc.tlas_nodes)
        assert np.array_equal(slot.scene_nodes(0, len(nodes)), nodes)
        _check(slot, sc2, rays, bounce_too=False)
    finally:
        lender.close()


def test_frame_slot_guards():
    a = refit_scene(42)
    lender = tthip.Engine(0)
    try:
        lender.upload(a)
        slots = []
        for _ in range(8):  # the upload reserved 8 TLAS regions
            e = tthip.Engine(0)
            e.share_blas(lender, a.tlas_nodes)
            slots.append(e)
        ninth = tthip.Engine(0)
        with pytest.raises(tthip.TTError) as ex:
            ninth.share_blas(lender, a.tlas_nodes)
        assert ex.value.status == tthip.TT_ERR_UNSUPPORTED
        slots[3].close()  # frees its region
        ninth.share_blas(lender, a.tlas_nodes)
        s = slots[0]
        T = a.tlas_nodes
        L = s.L
        with pytest.raises(tthip.TTError):
            s.update_nodes(T, a.nodes[T:T + 1])  # beyond its TLAS
        assert L.tt_scene_upload(s.h, a.nodes.ctypes.data, len(a.nodes), a.tris.ctypes.data, len(a.tris),
                                 a.tlas.ctypes.data, len(a.tlas), a.meshdata.ctypes.data, len(a.meshdata),
                                 a.materials.ctypes.data, len(a.materials)) == tthip.TT_ERR_INVALID_ARG
        # the lender's BLAS-side node rewrite is refused while slots exist; a TLAS-only one is not
        blas_node = T + 3
        with pytest.raises(tthip.TTError) as ex:
            lender.update_nodes(blas_node, a.nodes[blas_node:blas_node + 1])
        assert ex.value.status == tthip.TT_ERR_UNSUPPORTED
        lender.update_nodes(0, a.nodes[:T])
        e = tthip.Engine(0)
        try:
            with pytest.raises(tthip.TTError):
                e.share_blas(lender, 0)
            with pytest.raises(tthip.TTError):
                e.share_blas(lender, len(a.nodes))  # beyond the TLAS region
            with pytest.raises(tthip.TTError):
                e.share_blas(s, T)  # a borrower never lends
        finally:
            e.close()
    finally:
        lender.close()  # closes every slot first


def test_refused_share_leaves_the_context_as_it_was():
    """a tt_ctx_share_blas refused by the TLAS walk -- n_tlas_nodes inside the lender's TLAS
    region but smaller than the TLAS the walk reaches -- must leave dst as it was: a frame slot keeps its own
    moved TLAS and region, a context with its own scene keeps that scene; both still trace as before."""
    a = refit_scene(43)
    assert a.tlas_nodes > 1
    rays = _rays()
    lender, slot, own = tthip.Engine(0), tthip.Engine(0), tthip.Engine(0)
    try:
        lender.upload(a)
        slot.share_blas(lender, a.tlas_nodes)
        md_b, box_b = _pose(a, 7)
        slot.update_meshdata(0, md_b)
        slot.tlas_refit(a.tlas_nodes, box_b)
        sc_slot = _scene_of(slot, a, md_b)
        moved = _check(slot, sc_slot, rays)
        b = refit_scene(44)
        own.upload(b)
        own_hits = _check(own, b, rays, bounce_too=False)
        for dst in (slot, own):
            with pytest.raises(tthip.TTError) as ex:
                dst.share_blas(lender, 1)  # the TLAS walk leaves [0, 1)
            assert ex.value.status == tthip.TT_ERR_INVALID_ARG
        assert np.array_equal(_scene_of(slot, a, md_b).nodes, sc_slot.nodes)
        assert np.array_equal(_check(slot, sc_slot, rays), moved)
        assert np.array_equal(_check(own, b, rays, bounce_too=False), own_hits)
        # the refused calls reserved no overlay region: the 7 regions besides the slot's are all still free
        extra = [tthip.Engine(0) for _ in range(7)]
        try:
            for e in extra:
                e.share_blas(lender, a.tlas_nodes)
        finally:
            for e in extra:
                e.close()
    finally:
        own.close()
        lender.close()
