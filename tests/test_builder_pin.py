"""Builder restatement pinned by a leaf order the reference's C# builder produced.

TrueTrace/ExampleScene.unity:14115-14116 serializes the ParentObject "Pedestal"'s
CWBVHIndicesBufferInverted (source triangle -> CWBVH leaf position, ParentObject.cs:691-694), built
by the reference's BVH2Builder/BVH8Builder from Unity's import of Models/ExampleScene/Pedestal/
Pedestal.obj. The 48 values are committed as tests/golden/pedestal_leaf_order.npz
(tools/pedestal_pin.py --write-fixture). Two inputs of that build are not in the OBJ file:

  * BuildTotal's child->parent transform (ParentObject.cs:987-1014): V = (v + Ofst), 3x3, - Ofst2
    with Ofst = Ofst2 = the prefab's world position (0, -1.14, 0) (ExampleScene.unity:14033-14036),
    i.e. y -> fl(fl(y - 1.14f) + 1.14f) in float32;
  * the triangle order Unity's model importer hands over (its mesh optimizer reorders the
    triangles inside each submesh; the .meta import settings are not in the reference).

The order is recovered, not assumed: with the transform path applied, our builder's leaf sequence
composed with the serialized vector gives a permutation sigma (Unity triangle -> OBJ triangle).
It must (a) keep every triangle inside its own submesh (Bottom 0-19, Top 20-39, Ramp 40-47; a
random permutation almost never does), (b) reorder the two identically-shaped submeshes Bottom
and Top in the same quad order, and (c) rebuilding from the triangles in that order must reproduce the
serialized vector exactly. Without the transform path (a) fails -- the float rounding of BuildTotal
decides two SAH ties.
"""
import os

import numpy as np

import tthip

HERE = os.path.dirname(os.path.abspath(__file__))
PREFAB_Y = np.float32(-1.14)


def _mesh():
    z = np.load(os.path.join(HERE, "golden", "pedestal_mesh.npz"))
    return z["positions"].astype(np.float32), z["indices"]


def _serialized():
    return np.load(os.path.join(HERE, "golden", "pedestal_leaf_order.npz"))["leaf_order"].astype(np.int32)


def _build_total_positions(pos):
    p = pos.copy()
    p[:, 1] = ((p[:, 1] + PREFAB_Y).astype(np.float32) - PREFAB_Y).astype(np.float32)
    return p


def _submesh(a):
    return np.where(a < 20, 0, np.where(a < 40, 1, 2))


def _sigma(pos, idx, ref):
    lo = tthip.Blas(tthip.Mesh.from_arrays(pos, idx)).leaf_order()
    return np.argsort(lo)[ref]


def test_serialized_fixture_is_a_permutation():
    ref = _serialized()
    assert ref.shape == (48,)
    assert sorted(ref.tolist()) == list(range(48))


def test_builder_reproduces_reference_leaf_order():
    pos, idx = _mesh()
    ref = _serialized()
    p = _build_total_positions(pos)
    sigma = _sigma(p, idx, ref)
    assert sorted(sigma.tolist()) == list(range(48))
    assert np.array_equal(_submesh(sigma), _submesh(np.arange(48))), "import order must stay inside submeshes"
    # the two identically-shaped submeshes come out of the importer in the same quad order (the two
    # triangles of a quad may swap: their order is decided by index tie-breaks inside the build)
    assert np.array_equal((sigma[20:40] - 20) // 2, sigma[0:20] // 2), "identical submeshes, same quad order"
    assert np.array_equal(sigma[40:48], np.arange(40, 48))
    lo = tthip.Blas(tthip.Mesh.from_arrays(p, idx[sigma])).leaf_order()
    assert np.array_equal(lo, ref), f"{int((lo == ref).sum())}/48 leaf positions match"


def test_build_total_rounding_is_needed():
    pos, idx = _mesh()
    sigma = _sigma(pos, idx, _serialized())
    assert not np.array_equal(_submesh(sigma), _submesh(np.arange(48)))


# ---------------------------------------------------------------------------------------------
# Unity built-in Cube ParentObjects of the same scene (tools/unity_prim_pin.py --write-fixture):
# 18 serialized 12-entry leaf orders (4 distinct), positions = Unity's Cube mesh through BuildTotal's
# (v + Ofst) -> TransMat -> - Ofst2 path with each object's transform chain.


def _cube_pins():
    return np.load(os.path.join(HERE, "golden", "unity_cube_pins.npz"))


def test_unity_cube_leaf_orders_reproduced():
    z = _cube_pins()
    ok = []
    for pos, order in zip(z["positions"], z["orders"]):
        lo = tthip.Blas(tthip.Mesh.from_arrays(pos.astype(np.float32), z["cube_i"])).leaf_order()
        ok.append(bool(np.array_equal(lo, order)))
    assert ok == z["reproduced"].tolist()
    assert sum(ok) >= 14
    # the reproduced set includes orders other than the unit cube's: BuildTotal's float offset path
    # decides SAH ties there, exactly as in the reference's build
    repro = {tuple(o) for o, k in zip(z["orders"].tolist(), ok) if k}
    assert len(repro) >= 3


def test_unity_cube_raw_mesh_gives_the_common_order():
    z = _cube_pins()
    lo = tthip.Blas(tthip.Mesh.from_arrays(z["cube_v"], z["cube_i"])).leaf_order()
    common = max({tuple(o) for o in z["orders"].tolist()}, key=lambda o: sum(tuple(x) == o for x in z["orders"].tolist()))
    assert tuple(lo.tolist()) == common
