"""BLAS refit of deforming / skinned meshes (ParentObject.RefitMesh driving
BVHRefitter.compute Construct / RefitLayer / NodeUpdate / NodeCompress), oracle side: the
restatement re-derives the triangles exactly, keeps the topology, touches only the refit mesh,
and — after a deformation plus the TLAS refit the caller runs next — traverses to the same closest
triangles as brute force over the deformed geometry. GPU parity is in test_gpu_parity.py."""
import numpy as np
import pytest

import oracle_ctypes as O
import tthip
from test_oracle_bruteforce import _check, _random_rays


def two_mesh_scene(seed=7, n=600):
    mesh = tthip.Mesh.prop(seed, n)
    blas = tthip.Blas(mesh)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(1, 120, 3.0, 0.3)), None, np.zeros(1, tthip.MAT_DTYPE))
    am.add_parent(blas, tthip.trs_matrix((1.0, 0.0, 0.5)), np.zeros(3, tthip.MAT_DTYPE))
    return am.build(), mesh, blas


def vertex_buffer(pos, nrm, stride=10):
    """Unity-like interleaved vertex buffer: position, normal, tangent (ignored)."""
    v = np.zeros((len(pos), stride), np.float32)
    v[:, 0:3] = pos
    v[:, 3:6] = nrm
    v[:, 6:10] = 0.5
    return v


def deform(pos, t):
    p = pos.astype(np.float64).copy()
    p[:, 0] += 0.3 * np.sin(1.7 * p[:, 1] + t)
    p[:, 2] += 0.2 * np.cos(1.3 * p[:, 0] - t)
    p[:, 1] *= 1.0 + 0.1 * np.sin(t)
    return p.astype(np.float32)


def test_identity_refit_reproduces_positions_and_keeps_topology():
    sc, mesh, blas = two_mesh_scene()
    pos, nrm, idx = mesh.arrays()
    st, nodes, tris = O.blas_refit(sc, 1, vertex_buffer(pos, nrm), idx, blas.leaf_order())
    assert st == 0
    to, no = int(sc.meshdata["TriOffset"][1]), int(sc.meshdata["NodeOffset"][1])
    k = slice(to, to + blas.n_tris)
    for f in ("pos0", "posedge1", "posedge2"):
        assert np.array_equal(tris[f][k], sc.tris[f][k])
    for f in ("tans", "tex0", "texedge1", "texedge2", "MatDat"):
        assert np.array_equal(tris[f], sc.tris[f])  # Construct leaves these alone
    assert np.array_equal(tris[: to], sc.tris[: to])
    for f in ("base_child", "base_tri", "meta"):
        assert np.array_equal(nodes[f], sc.nodes[f])
    assert np.array_equal(nodes["e_imask"] >> 24, sc.nodes["e_imask"] >> 24)  # imask
    assert np.array_equal(nodes[:no], sc.nodes[:no])  # the TLAS and the other BLAS are untouched


@pytest.mark.parametrize("t", [0.4, 2.1])
def test_deformed_mesh_traces_like_brute_force(t):
    sc, mesh, blas = two_mesh_scene(seed=9, n=900)
    pos, nrm, idx = mesh.arrays()
    # skinned-group transform (worldToLocal * TRS(rootBone)): a rotation + offset in object space
    xf = tthip.trs_matrix((0.2, -0.1, 0.3), 17.0, 1.0)
    st, nodes, tris = O.blas_refit(sc, 1, vertex_buffer(deform(pos, t), nrm), idx, blas.leaf_order(), xf)
    assert st == 0
    # the caller then refits the TLAS from the meshes' new world bounds (RefitTLAS)
    to = int(sc.meshdata["TriOffset"][1])
    p0 = tris["pos0"][to:to + blas.n_tris].astype(np.float64)
    corners = np.concatenate([p0, p0 + tris["posedge1"][to:to + blas.n_tris], p0 + tris["posedge2"][to:to + blas.n_tris]])
    l2w = tthip.trs_matrix((1.0, 0.0, 0.5))
    w = corners @ l2w[:3, :3].T + l2w[:3, 3]
    boxes = sc.meta["mesh_aabbs"].copy()
    boxes[1, 0:3], boxes[1, 3:6] = w.max(0) + 1e-4, w.min(0) - 1e-4
    sc2 = tthip.Scene(nodes, tris, sc.tlas, sc.meshdata, sc.materials, tlas_nodes=sc.tlas_nodes)
    st, nodes2 = O.tlas_refit(sc2, boxes)
    assert st == 0
    sc3 = tthip.Scene(nodes2, tris, sc.tlas, sc.meshdata, sc.materials, tlas_nodes=sc.tlas_nodes)
    rng = np.random.default_rng(int(t * 10))
    rays = _random_rays(rng, 300, np.array([1.0, 2.0, 0.5]), 5.0)
    _check(sc3, rays, 300)


def test_bad_arguments():
    sc, mesh, blas = two_mesh_scene()
    pos, nrm, idx = mesh.arrays()
    v = vertex_buffer(pos, nrm)
    assert O.blas_refit(sc, 5, v, idx, blas.leaf_order())[0] == tthip.TT_ERR_INVALID_ARG  # no such mesh
    assert O.blas_refit(sc, 1, v[:, :5], idx, blas.leaf_order())[0] == tthip.TT_ERR_INVALID_ARG  # stride < 6
    many = np.concatenate([idx, idx[:3]])
    assert O.blas_refit(sc, 0, v, np.tile(many, 100), np.arange(len(many) * 100 // 3, dtype=np.int32))[0] == \
        tthip.TT_ERR_INVALID_ARG  # more triangles than the scene holds after TriOffset
