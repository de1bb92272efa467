#!/usr/bin/env python3
"""Builder pins from Unity's built-in primitives in the reference scene (widened).

TrueTrace/ExampleScene.unity serializes, for every ParentObject, the CWBVHIndicesBufferInverted its
editor build wrote (source triangle -> CWBVH leaf position, ParentObject.cs:691-694). Most of those
objects are Unity built-in meshes (MeshFilter m_Mesh fileID 10202 = Cube, 10207 = Sphere,
10209 = Plane, 10210 = Quad). The built-in Cube's vertex and index order is Unity's fixed asset
(24 vertices, 12 triangles, below); this script feeds it through ParentObject.BuildTotal's
child -> parent transform path (ParentObject.cs:973-1014):

    V = TransMat * (v + Ofst) - Ofst2,   Ofst = WTL_child * P_child,  Ofst2 = WTL_parent * P_parent

with Matrix4x4 * Vector3 taken as the 3x3 part (Vector3 -> Vector4 with w = 0), rebuilds the BLAS
with the C++ builder restatement and compares the leaf order with the serialized vector. The
transform inputs are not reconstructed from the Transform hierarchy: every ParentObject serializes
the exact float32 CachedTransforms (worldToLocalMatrix + position of itself and its children) that
BuildTotal consumed, and its ParentScale (0.001 / lossyScale), the padding AABB.Validate gives the
flat cube faces (CommonVars.cs:385-395) -- the input that decides the SAH ties of the scaled cubes.

  --write-fixture   writes tests/golden/unity_cube_pins.npz (the serialized vectors + the transform
                    inputs of every cube ParentObject; data only) for tests/test_builder_pin.py.
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
SCENE = "/root/reference/TrueTrace/ExampleScene.unity"

# Unity's built-in Cube mesh (Library/unity default resources, fileID 10202): vertices and triangles
CUBE_V = np.array([
    (0.5, -0.5, 0.5), (-0.5, -0.5, 0.5), (0.5, 0.5, 0.5), (-0.5, 0.5, 0.5),
    (0.5, 0.5, -0.5), (-0.5, 0.5, -0.5), (0.5, -0.5, -0.5), (-0.5, -0.5, -0.5),
    (0.5, 0.5, 0.5), (-0.5, 0.5, 0.5), (0.5, 0.5, -0.5), (-0.5, 0.5, -0.5),
    (0.5, -0.5, -0.5), (0.5, -0.5, 0.5), (-0.5, -0.5, 0.5), (-0.5, -0.5, -0.5),
    (-0.5, -0.5, 0.5), (-0.5, 0.5, 0.5), (-0.5, 0.5, -0.5), (-0.5, -0.5, -0.5),
    (0.5, -0.5, -0.5), (0.5, 0.5, -0.5), (0.5, 0.5, 0.5), (0.5, -0.5, 0.5)], np.float32)
CUBE_I = np.array([0, 2, 3, 0, 3, 1, 8, 4, 5, 8, 5, 9, 10, 6, 7, 10, 7, 11,
                   12, 13, 14, 12, 14, 15, 16, 17, 18, 16, 18, 19, 20, 21, 22, 20, 22, 23], np.int32)
# Unity's built-in Quad (fileID 10210): 4 vertices in the z = 0 plane, 2 triangles
QUAD_V = np.array([(-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (-0.5, 0.5, 0.0), (0.5, 0.5, 0.0)], np.float32)
QUAD_I = np.array([0, 3, 1, 3, 0, 2], np.int32)
MESHES = {"Cube": (CUBE_V, CUBE_I), "Quad": (QUAD_V, QUAD_I)}
PRIMS = {10202: "Cube", 10206: "Cylinder", 10207: "Sphere", 10208: "Capsule", 10209: "Plane", 10210: "Quad"}


def parse_scene(path=SCENE):
    """{fileID: (class_id, text)} for every document of the scene."""
    docs = {}
    cur = None
    buf = []
    for line in open(path, encoding="utf-8", errors="replace"):
        m = re.match(r"^--- !u!(\d+) &(\d+)", line)
        if m:
            if cur is not None:
                docs[cur[1]] = (cur[0], "".join(buf))
            cur = (int(m.group(1)), int(m.group(2)))
            buf = []
        else:
            buf.append(line)
    if cur is not None:
        docs[cur[1]] = (cur[0], "".join(buf))
    return docs


def _vec(text, key, n):
    m = re.search(key + r": \{([^}]*)\}", text)
    vals = dict(kv.split(": ") for kv in m.group(1).split(", "))
    return np.array([float(vals[c]) for c in "xyzw"[:n]], np.float32)


def _fid(text, key):
    m = re.search(key + r": \{fileID: (\d+)", text)
    return int(m.group(1)) if m else 0


def transforms(docs):
    """GameObject fileID -> Transform text."""
    out = {}
    for fid, (cls, t) in docs.items():
        if cls == 4:
            out[_fid(t, "m_GameObject")] = (fid, t)
    return out


def quat_mat(q):
    x, y, z, w = [float(v) for v in q]
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float64)


def world_trs(docs, tr_by_fid, tfid):
    """(world position, world 3x3 (rotation*scale)) of a Transform, composed up the hierarchy."""
    cls, t = docs[tfid]
    p = _vec(t, "m_LocalPosition", 3).astype(np.float64)
    r = quat_mat(_vec(t, "m_LocalRotation", 4))
    s = _vec(t, "m_LocalScale", 3).astype(np.float64)
    m = r * s[None, :]
    father = _fid(t, "m_Father")
    if father and father in docs:
        fp, fm = world_trs(docs, tr_by_fid, father)
        return fp + fm @ p, fm @ m
    return p, m


def parent_objects(docs):
    """Every ParentObject with a serialized leaf order: name, order, its GameObject, child meshes."""
    tr = transforms(docs)
    mesh_of = {}
    for fid, (cls, t) in docs.items():
        if cls == 33:  # MeshFilter
            mesh_of[_fid(t, "m_GameObject")] = _fid(t, "m_Mesh")
    out = []
    for fid, (cls, t) in docs.items():
        if cls != 114 or "CWBVHIndicesBufferInverted:" not in t:
            continue
        hexs = re.search(r"CWBVHIndicesBufferInverted: ?([0-9a-f]*)", t).group(1)
        order = np.frombuffer(bytes.fromhex(hexs), np.int32).copy()
        go = _fid(t, "m_GameObject")
        name = re.search(r"\n  Name: (.*)", t).group(1).strip()
        kids = [int(k) for k in re.findall(r"- \{fileID: (\d+)\}", t.split("ChildObjects:")[1].split("MeshCountChanged")[0])]
        kid_gos = [_fid(docs[k][1], "m_GameObject") for k in kids if k in docs]
        out.append(dict(name=name, order=order, go=go, tfid=tr.get(go, (0, ""))[0], text=t,
                        kids=[(g, tr.get(g, (0, ""))[0], mesh_of.get(g, 0)) for g in kid_gos]))
    return out


def cached_transforms(text):
    """The ParentObject's serialized CachedTransforms (ParentObject.cs:54, filled at :516-521 right before
    the build): [(worldToLocalMatrix as float32 4x4 [row][col], world position)], parent first."""
    blk = text.split("CachedTransforms:")[1].split("CurMeshData:")[0]
    out = []
    for ent in blk.split("- WTL:")[1:]:
        m = np.zeros((4, 4), np.float32)
        for r in range(4):
            for c in range(4):
                m[r, c] = np.float32(float(re.search(rf"e{r}{c}: ([^\n]+)", ent).group(1)))
        p = re.search(r"Position: \{x: ([^,]+), y: ([^,]+), z: ([^}]+)\}", ent)
        out.append((m, np.array([float(p.group(i)) for i in (1, 2, 3)], np.float32)))
    return out


def parent_scale(text):
    """The serialized ParentScale = 0.001 / lossyScale (ParentObject.cs:462-463), the flat-box padding of
    AABB.Validate (CommonVars.cs:385-395) in BuildTotal (ParentObject.cs:1058)."""
    m = re.search(r"ParentScale: \{x: ([^,]+), y: ([^,]+), z: ([^}]+)\}", text)
    return np.array([float(m.group(i)) for i in (1, 2, 3)], np.float32)


def lossy_for(ps):
    """A float32 lossyScale whose 0.001f / lossy is exactly the serialized ParentScale (the builder
    restatement takes the lossy scale, host/tt_scene.cpp)."""
    f = np.float32
    out = []
    for v in ps:
        c = f(f(0.001) / f(v))
        for k in range(64):
            if f(f(0.001) / c) == f(v):
                break
            c = np.nextafter(c, f(np.inf) if f(f(0.001) / c) > f(v) else f(0))
        assert f(f(0.001) / c) == f(v), v
        out.append(float(c))
    return tuple(out)


def mat_inverse(m):
    """Matrix4x4.inverse: Gauss-Jordan with partial pivoting evaluated in DOUBLE precision, each element
    rounded to float32 once at the end. Of the inverses tried against all 18 pins (this one, numpy's
    double inverse, the float32 Gauss-Jordan, Mesa's 3x3-cofactor affine inverse in float32 and in
    double), only the double-precision ones reproduce the rotated "Cube (5)"; the float32 cofactor form
    also misses two scaled cubes (tools/unity_cube_rounding.py)."""
    r = [np.concatenate([m[i].astype(np.float64), np.eye(4)[i]]) for i in range(4)]
    for c in range(4):
        piv = max(range(c, 4), key=lambda i: abs(r[i][c]))
        r[c], r[piv] = r[piv], r[c]
        for i in range(c + 1, 4):
            r[i] = r[i] - (r[i][c] / r[c][c]) * r[c]
    for c in range(3, -1, -1):
        r[c] = r[c] * (1.0 / r[c][c])
        for i in range(c):
            r[i] = r[i] - r[i][c] * r[c]
    return np.stack([x[4:] for x in r]).astype(np.float32)


def unity_mul(a, b):
    """Matrix4x4 * Matrix4x4: res.m_rc = a.m_r0 * b.m_0c + a.m_r1 * b.m_1c + a.m_r2 * b.m_2c + a.m_r3 * b.m_3c."""
    f = np.float32
    out = np.zeros((4, 4), f)
    for r in range(4):
        for c in range(4):
            s = f(a[r, 0] * b[0, c])
            for k in range(1, 4):
                s = f(s + f(a[r, k] * b[k, c]))
            out[r, c] = s
    return out


def unity_mv(m, v):
    """Matrix4x4 * (Vector4)Vector3 (w = 0), back to Vector3: the translation column drops out."""
    f = np.float32
    out = np.zeros(v.shape, f)
    for r in range(3):
        s = (m[r, 0] * v[..., 0]).astype(f)
        s = (s + (m[r, 1] * v[..., 1]).astype(f)).astype(f)
        s = (s + (m[r, 2] * v[..., 2]).astype(f)).astype(f)
        out[..., r] = (s + m[r, 3] * f(0)).astype(f)
    return out


def build_total_positions(v, cached):
    """BuildTotal (ParentObject.cs:975-1014) on the serialized CachedTransforms: TransMat =
    WTL_parent * WTL_child.inverse, Ofst = WTL_child * Position_child, Ofst2 = WTL_parent *
    Position_parent, V = TransMat * (v + Ofst) - Ofst2, every operation in float32."""
    (w0, p0), (w1, p1) = cached[0], cached[1]
    trans = unity_mul(w0, mat_inverse(w1))
    ofst = unity_mv(w1, p1[None, :])[0]
    ofst2 = unity_mv(w0, p0[None, :])[0]
    a = (v + ofst).astype(np.float32)
    return (unity_mv(trans, a) - ofst2).astype(np.float32)


def cube_cases():
    """[(name, serialized order, BuildTotal-path float32 positions, lossy scale)] for every Cube ParentObject."""
    docs = parse_scene()
    out = []
    for o in parent_objects(docs):
        if [PRIMS.get(k[2], "") for k in o["kids"]] != ["Cube"]:
            continue
        out.append((o["name"], o["order"], build_total_positions(CUBE_V, cached_transforms(o["text"])),
                    lossy_for(parent_scale(o["text"]))))
    return out


def multi_cases():
    """[(name, serialized order, positions, indices, lossy scale)] for every ParentObject whose children
    are several known built-in meshes (Cube / Quad): BuildTotal appends the children in ChildObjects order,
    child i through CachedTransforms[0] and CachedTransforms[i + 1] (ParentObject.cs:983-1014)."""
    docs = parse_scene()
    out = []
    for o in parent_objects(docs):
        kinds = [PRIMS.get(k[2], "") for k in o["kids"]]
        if kinds in ([], ["Cube"]) or any(k not in MESHES for k in kinds):
            continue
        ct = cached_transforms(o["text"])
        pos, idx, base = [], [], 0
        for i, k in enumerate(kinds):
            v, ix = MESHES[k]
            pos.append(build_total_positions(v, [ct[0], ct[i + 1]]))
            idx.append(ix + base)
            base += len(v)
        out.append((o["name"], o["order"], np.concatenate(pos), np.concatenate(idx).astype(np.int32),
                    lossy_for(parent_scale(o["text"]))))
    return out


def main():
    import tthip

    multi = multi_cases()
    mres = []
    for name, order, pos, idx, lossy in multi:
        lo = tthip.Blas(tthip.Mesh.from_arrays(pos, idx), lossy_scale=lossy).leaf_order()
        mres.append(int((lo == order).sum()))
        print(f"{name:16s} {len(order):3d} triangles: {mres[-1]}/{len(order)} leaf positions match")

    cases = cube_cases()
    raw = tthip.Blas(tthip.Mesh.from_arrays(CUBE_V, CUBE_I)).leaf_order()
    ok = []
    for name, order, pos, lossy in cases:
        lo = tthip.Blas(tthip.Mesh.from_arrays(pos, CUBE_I), lossy_scale=lossy).leaf_order()
        ok.append(bool(np.array_equal(lo, order)))
        print(f"{name:16s} raw={bool(np.array_equal(raw, order))!s:5s} build_total={ok[-1]!s:5s} "
              f"serialized={order.tolist()} ours={lo.tolist()}")
    print(f"cubes: {len(cases)}, BuildTotal-path matches {sum(ok)}")
    if "--write-fixture" in sys.argv:
        np.savez_compressed(os.path.join(REPO, "tests", "golden", "unity_cube_pins.npz"),
                            names=np.array([c[0] for c in cases]), orders=np.stack([c[1] for c in cases]),
                            positions=np.stack([c[2] for c in cases]), lossy=np.array([c[3] for c in cases], np.float32),
                            reproduced=np.array(ok),
                            cube_v=CUBE_V, cube_i=CUBE_I)
        d = {"names": np.array([m[0] for m in multi]), "matched": np.array(mres, np.int32)}
        for k, (name, order, pos, idx, lossy) in enumerate(multi):
            d[f"order_{k}"], d[f"positions_{k}"], d[f"indices_{k}"], d[f"lossy_{k}"] = order, pos, idx, np.array(lossy, np.float32)
        np.savez_compressed(os.path.join(REPO, "tests", "golden", "unity_multi_pins.npz"), **d)


if __name__ == "__main__":
    main()
