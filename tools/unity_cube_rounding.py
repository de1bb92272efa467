#!/usr/bin/env python3
"""Which Matrix4x4.inverse reproduces the Unity Cube builder pins.

BuildTotal (ParentObject.cs:975-1014) consumes the serialized CachedTransforms (exact float32
worldToLocalMatrix + position, ExampleScene.unity) and the serialized ParentScale (the AABB.Validate
padding of the flat cube faces). What the scene does not hold is how Unity rounds
`CachedTransforms[i].WTL.inverse` (native code). This script rebuilds all 18 cube ParentObjects
with each candidate inverse and prints how many serialized leaf orders each reproduces:

  gj_f32      Gauss-Jordan with partial pivoting in float32
  gj_f64      the same in double, rounded to float32 once (tools/unity_prim_pin.mat_inverse)
  numpy_f64   numpy's double inverse rounded to float32
  mesa3d_f32  Mesa's affine inverse (3x3 cofactors * 1/det) in float32
  mesa3d_f64  the same in double

Result (recorded in DESIGN.md §4): only the double-precision inverses reproduce all 18; without the
ParentScale padding (lossy scale 1) every candidate stays at 13-14.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "truetrace-unity-pathtracer_amd", "python"))
import unity_prim_pin as U  # noqa: E402


def gj_f32(m):
    f = np.float32
    r = [np.concatenate([m[i].astype(f), np.eye(4, dtype=f)[i]]) for i in range(4)]
    for c in range(4):
        piv = max(range(c, 4), key=lambda i: abs(float(r[i][c])))
        r[c], r[piv] = r[piv], r[c]
        for i in range(c + 1, 4):
            k = f(r[i][c] / r[c][c])
            r[i] = (r[i] - (k * r[c]).astype(f)).astype(f)
    for c in range(3, -1, -1):
        s = f(f(1) / r[c][c])
        r[c] = (r[c] * s).astype(f)
        for i in range(c):
            r[i] = (r[i] - (r[i][c] * r[c]).astype(f)).astype(f)
    return np.stack([x[4:] for x in r]).astype(f)


def mesa3d(m, dt):
    m = m.astype(dt)
    M = lambda r, c: m[r, c]  # noqa: E731
    pos = neg = dt(0)
    for t in (M(0, 0) * M(1, 1) * M(2, 2), M(1, 0) * M(2, 1) * M(0, 2), M(2, 0) * M(0, 1) * M(1, 2),
              -M(2, 0) * M(1, 1) * M(0, 2), -M(1, 0) * M(0, 1) * M(2, 2), -M(0, 0) * M(2, 1) * M(1, 2)):
        t = dt(t)
        if t >= 0:
            pos = dt(pos + t)
        else:
            neg = dt(neg + t)
    det = dt(dt(1) / dt(pos + neg))
    o = np.zeros((4, 4), dt)
    o[0, 0] = dt((M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * det)
    o[0, 1] = dt(-(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * det)
    o[0, 2] = dt((M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * det)
    o[1, 0] = dt(-(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * det)
    o[1, 1] = dt((M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * det)
    o[1, 2] = dt(-(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * det)
    o[2, 0] = dt((M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * det)
    o[2, 1] = dt(-(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * det)
    o[2, 2] = dt((M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * det)
    o[3, 3] = 1
    return o.astype(np.float32)


CANDIDATES = {
    "gj_f32": gj_f32,
    "gj_f64": U.mat_inverse,
    "numpy_f64": lambda m: np.linalg.inv(m.astype(np.float64)).astype(np.float32),
    "mesa3d_f32": lambda m: mesa3d(m, np.float32),
    "mesa3d_f64": lambda m: mesa3d(m, np.float64),
}


def positions(cached, inv):
    (w0, p0), (w1, p1) = cached
    trans = U.unity_mul(w0, inv(w1))
    ofst = U.unity_mv(w1, p1[None, :])[0]
    ofst2 = U.unity_mv(w0, p0[None, :])[0]
    return (U.unity_mv(trans, (U.CUBE_V + ofst).astype(np.float32)) - ofst2).astype(np.float32)


def main():
    import tthip

    docs = U.parse_scene()
    objs = [o for o in U.parent_objects(docs) if [U.PRIMS.get(k[2], "") for k in o["kids"]] == ["Cube"]]
    for pad in ("ParentScale", "none"):
        for name, inv in CANDIDATES.items():
            ok = []
            for o in objs:
                lossy = U.lossy_for(U.parent_scale(o["text"])) if pad == "ParentScale" else (1.0, 1.0, 1.0)
                pos = positions(U.cached_transforms(o["text"]), inv)
                lo = tthip.Blas(tthip.Mesh.from_arrays(pos, U.CUBE_I), lossy_scale=lossy).leaf_order()
                ok.append(bool(np.array_equal(lo, o["order"])))
            print(f"padding={pad:12s} {name:11s} {sum(ok):2d}/18 {''.join('1' if k else '.' for k in ok)}")
    print("objects:", [o["name"] for o in objs])


if __name__ == "__main__":
    main()
