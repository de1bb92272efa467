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
# 18 serialized 12-entry leaf orders (6 distinct). Inputs, all from the scene's serialized fields:
# positions = Unity's Cube mesh through BuildTotal's (v + Ofst) -> TransMat -> - Ofst2 path on each
# object's CachedTransforms (exact float32 worldToLocalMatrix + position; Matrix4x4.inverse evaluated
# in double, rounded once), and the lossy scale whose 0.001f / lossy is the serialized ParentScale --
# the AABB.Validate padding of the flat faces (CommonVars.cs:385-395), which decides the SAH ties of
# the scaled cubes.


def _cube_pins():
    return np.load(os.path.join(HERE, "golden", "unity_cube_pins.npz"))


def _cube_order(pos, idx, lossy):
    return tthip.Blas(tthip.Mesh.from_arrays(pos.astype(np.float32), idx),
                      lossy_scale=tuple(float(x) for x in lossy)).leaf_order()


def test_unity_cube_leaf_orders_reproduced():
    z = _cube_pins()
    ok = [bool(np.array_equal(_cube_order(p, z["cube_i"], l), o))
          for p, o, l in zip(z["positions"], z["orders"], z["lossy"])]
    assert ok == z["reproduced"].tolist()
    assert all(ok), f"{sum(ok)}/18 serialized cube leaf orders reproduced"
    assert len({tuple(o) for o in z["orders"].tolist()}) == 6  # all 6 distinct serialized orders are covered


def test_unity_cube_parent_scale_padding_is_needed():
    """Without the serialized ParentScale (lossy scale 1: padding 0.001 on every axis) the scaled cubes'
    ties break differently: the padding is an input of the reference's build, not a detail."""
    z = _cube_pins()
    ok = [bool(np.array_equal(_cube_order(p, z["cube_i"], (1.0, 1.0, 1.0)), o))
          for p, o in zip(z["positions"], z["orders"])]
    assert sum(ok) < 18
    assert not all(np.allclose(l, 1.0) for l in z["lossy"])


def test_unity_cube_raw_mesh_gives_the_common_order():
    z = _cube_pins()
    lo = tthip.Blas(tthip.Mesh.from_arrays(z["cube_v"], z["cube_i"])).leaf_order()
    common = max({tuple(o) for o in z["orders"].tolist()}, key=lambda o: sum(tuple(x) == o for x in z["orders"].tolist()))
    assert tuple(lo.tolist()) == common


# Multi-child ParentObjects made of built-in meshes (tools/unity_prim_pin.py --write-fixture): "Ceiling"
# (4 cubes, 48 triangles) and "Wall1" (4 cubes + a Quad, 50) reproduce every leaf position, "Quad" its 2.
# "Entrance" (3 cubes, one under a 90-degree x rotation stored with 1e-8-level float noise) matches 32 of
# 36: two within-leaf swaps of the two triangles of a face whose boxes tie up to that noise.


def test_unity_multi_object_leaf_orders():
    z = np.load(os.path.join(HERE, "golden", "unity_multi_pins.npz"))
    got = {}
    for k, name in enumerate(z["names"].tolist()):
        lo = tthip.Blas(tthip.Mesh.from_arrays(z[f"positions_{k}"], z[f"indices_{k}"]),
                        lossy_scale=tuple(float(x) for x in z[f"lossy_{k}"])).leaf_order()
        got[name] = int((lo == z[f"order_{k}"]).sum())
        assert sorted(lo.tolist()) == list(range(len(lo)))
    assert got == dict(zip(z["names"].tolist(), z["matched"].tolist()))
    assert got["Ceiling"] == 48 and got["Wall1"] == 50 and got["Quad"] == 2
    assert got["Entrance"] >= 32
