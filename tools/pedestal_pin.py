#!/usr/bin/env python3
"""Builder pin against a leaf order the reference's own C# builder produced.

TrueTrace/ExampleScene.unity serializes, for the ParentObject "Pedestal" (line 14115-14116), the
CWBVHIndicesBufferInverted its editor build wrote: source triangle i -> position in the CWBVH
leaf order (ParentObject.cs:691-694). The mesh is the reference's Models/ExampleScene/Pedestal/
Pedestal.obj (48 triangles, three submeshes already grouped by material in file order). This
script rebuilds the BLAS from those triangles under hypotheses about what ParentObject.BuildTotal
(ParentObject.cs:973-1058) feeds the builder and prints how many of the 48 positions match:

  * obj:        the OBJ positions with Unity's import convention (x negated), as fed so far;
  * offset:     BuildTotal's child->parent transform path: V = (v + Ofst) then TransMat (3x3,
                identity here) then - Ofst2, Ofst = Ofst2 = the prefab's world position
                (0, -1.14, 0) (ExampleScene.unity:14033-14036; parent transform at the origin,
                :12703-12705) -- so y becomes fl(fl(y - 1.14f) + 1.14f) in float32;
  * no-negate:  the same without the x negation.

The serialized vector is data from the reference (a fixture), copied into
tests/golden/pedestal_leaf_order.npz by --write-fixture.
"""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))

# ExampleScene.unity:14116, CWBVHIndicesBufferInverted of "Pedestal" (48 little-endian int32)
SERIALIZED_HEX = (
    "2c0000002d00000012000000110000000b0000000a000000180000001900000025000000240000001b000000220000"
    "00000000002b000000130000001a000000030000002000000010000000290000002f0000002e000000160000001700"
    "00000e0000000f0000001d0000001e00000026000000270000001f00000023000000010000002a000000150000001c"
    "00000002000000210000001400000028000000090000000800000004000000050000000c0000000d00000006000000"
    "07000000")
PREFAB_Y = np.float32(-1.14)


def serialized() -> np.ndarray:
    return np.frombuffer(bytes.fromhex(SERIALIZED_HEX), np.int32).copy()


def variants(pos: np.ndarray):
    out = {"obj": pos.copy()}
    p = pos.copy()
    p[:, 1] = ((p[:, 1] + PREFAB_Y).astype(np.float32) - PREFAB_Y).astype(np.float32)
    out["offset"] = p
    q = pos.copy()
    q[:, 0] = -q[:, 0]
    out["no-negate"] = q
    r = q.copy()
    r[:, 1] = ((r[:, 1] + PREFAB_Y).astype(np.float32) - PREFAB_Y).astype(np.float32)
    out["no-negate+offset"] = r
    return out


def main():
    import tthip

    z = np.load(os.path.join(REPO, "tests", "golden", "pedestal_mesh.npz"))
    pos, idx = z["positions"].astype(np.float32), z["indices"]
    ref = serialized()
    for name, p in variants(pos).items():
        lo = tthip.Blas(tthip.Mesh.from_arrays(p, idx)).leaf_order()
        print(f"{name:18s} {int((lo == ref).sum()):2d}/48  {lo[:16].tolist()}")
    print(f"{'serialized':18s}        {ref[:16].tolist()}")
    if "--write-fixture" in sys.argv:
        np.savez_compressed(os.path.join(REPO, "tests", "golden", "pedestal_leaf_order.npz"), leaf_order=ref)


if __name__ == "__main__":
    main()
