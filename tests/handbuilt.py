"""Hand-built CWBVH8 scenes with exactly known traversal outcomes (test infrastructure).

Nodes are written directly in the 80-byte BVHNode8Data layout (CommonData.cginc:174-181,
packed like CommonFunctions.Aggregate, CommonVars.cs:662-688) so the tests do not depend on the
builder restatement. Quantisation scale is a power of two and every coordinate is a small
dyadic rational, so all slab/triangle arithmetic in these scenes is exact and the expected
results hold under any legal rounding of the reference HLSL.
"""
from __future__ import annotations

import numpy as np

import tthip

IDENTITY_W2L = tthip.unity_colmajor(np.eye(4))


def pack_bytes(b):
    b = list(b) + [0] * (8 - len(b))
    lo = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)
    hi = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24)
    return lo, hi


def make_node(p, exp, base_child, base_tri, children):
    """children: list of up to 8 (slot, kind, qlo(3), qhi(3), payload)
    kind 'inner': payload = internal ordinal k (child = base_child + k, meta = 0x20 | (24+k))
    kind 'leaf' : payload = (tri_offset, n_tris) (meta = mask<<5 | tri_offset)
    exp: biased float exponent byte per axis (scale 2^(exp-127))."""
    meta = [0] * 8
    qlo = [[0] * 8 for _ in range(3)]
    qhi = [[0] * 8 for _ in range(3)]
    imask = 0
    for slot, kind, lo, hi, payload in children:
        for a in range(3):
            qlo[a][slot] = lo[a]
            qhi[a][slot] = hi[a]
        if kind == "inner":
            meta[slot] = 0x20 | (24 + payload)
            imask |= 1 << payload
        else:
            off, n = payload
            meta[slot] = (((1 << n) - 1) << 5) | off
    n = np.zeros(1, tthip.NODE_DTYPE)[0]
    n["p"] = p
    n["e_imask"] = exp[0] | (exp[1] << 8) | (exp[2] << 16) | (imask << 24)
    n["base_child"] = base_child
    n["base_tri"] = base_tri
    n["meta"] = pack_bytes(meta)
    n["qlo_x"], n["qhi_x"] = pack_bytes(qlo[0]), pack_bytes(qhi[0])
    n["qlo_y"], n["qhi_y"] = pack_bytes(qlo[1]), pack_bytes(qhi[1])
    n["qlo_z"], n["qhi_z"] = pack_bytes(qlo[2]), pack_bytes(qhi[2])
    return n


def tri(p0, e1, e2, matdat=0):
    t = np.zeros(1, tthip.TRI_DTYPE)[0]
    t["pos0"], t["posedge1"], t["posedge2"], t["MatDat"] = p0, e1, e2, matdat
    return t


def mesh_record(node_offset, tri_offset, root, w2l=None, mat_offset=0):
    m = np.zeros(1, tthip.MESH_DTYPE)[0]
    m["W2L"] = IDENTITY_W2L if w2l is None else w2l
    m["TriOffset"], m["NodeOffset"], m["MaterialOffset"], m["mesh_data_bvh_offsets"] = tri_offset, node_offset, mat_offset, root
    return m


E0 = 127  # scale 1.0
FULL = ((0, 0, 0), (255, 255, 255))


def tlas_one_instance(node_offset=2):
    """TLAS region of a single-instance scene: node 0 has one leaf child (instance slot 0)."""
    return make_node((-128.0, -128.0, -128.0), (E0, E0, E0), 0, 0, [(0, "leaf", FULL[0], FULL[1], (0, 1))])


def scene(blas_nodes, tris, materials=None, w2l=None, n_instances=1):
    """Single-instance two-level scene: TLAS at [0, 2), BLAS at 2 (AssetManager.cs:995)."""
    nodes = np.zeros(2 + len(blas_nodes), tthip.NODE_DTYPE)
    nodes[0] = tlas_one_instance()
    nodes[2:] = blas_nodes
    md = np.zeros(1, tthip.MESH_DTYPE)
    md[0] = mesh_record(2, 0, 2, w2l)
    mats = np.zeros(1, tthip.MAT_DTYPE) if materials is None else materials
    return tthip.Scene(nodes, np.array(tris, tthip.TRI_DTYPE), np.zeros(1, np.int32), md, mats, tlas_nodes=1)


def rays_buffer(origins, dirs, far=1000.0, width=None, height=1):
    n = len(origins)
    width = width or n
    r = np.zeros(2 * width * height, tthip.RAY_DTYPE)
    r["origin"][:n] = origins
    r["direction"][:n] = dirs
    r["PixelIndex"][:n] = np.arange(n)
    r["hits"][:n, 2] = np.float32(far).view(np.uint32)
    return r


def expected_hit(mesh_id, tri_id, t, u, v):
    uv = int(np.uint32(np.float32(u) * np.float32(65535.0))) | (int(np.uint32(np.float32(v) * np.float32(65535.0))) << 16)
    return [mesh_id, tri_id & 0xFFFFFFFF, int(np.float32(t).view(np.uint32)), uv]


def shadow_rays(origins, dirs, ts, illum=(1.0, 2.0, 4.0)):
    """ShadowRayData array (CommonData.cginc:116-123), PixelIndex = ray index."""
    n = len(origins)
    r = np.zeros(n, tthip.SHADOW_DTYPE)
    r["origin"] = origins
    r["direction"] = dirs
    r["t"] = ts
    r["illumination"] = illum
    r["PixelIndex"] = np.arange(n)
    return r


def nee_rays_from_hits(rays, n, light, seed=0, far=1000.0):
    """Shadow rays toward a point light from the hit points of the first n traced rays (misses
    skipped): origin backed off 1e-3 along the incoming direction, t = +-distance with a random
    sign (the reference uses the sign to pick the accumulation target). Test input only."""
    rng = np.random.default_rng(seed)
    h = rays["hits"][:n]
    t = h[:, 2].view(np.float32)
    hit = t < np.float32(far)
    o = rays["origin"][:n][hit].astype(np.float32)
    d = rays["direction"][:n][hit].astype(np.float32)
    p = o + d * t[hit][:, None] - d * np.float32(1e-3)
    to = np.asarray(light, np.float32)[None, :] - p
    dist = np.sqrt((to * to).sum(1)).astype(np.float32)
    sr = np.zeros(int(hit.sum()), tthip.SHADOW_DTYPE)
    sr["origin"] = p
    sr["direction"] = to / dist[:, None]
    sr["t"] = dist * np.where(rng.random(len(sr)) < 0.75, 1.0, -1.0).astype(np.float32)
    sr["illumination"] = rng.random((len(sr), 3)).astype(np.float32)
    sr["PixelIndex"] = rays["PixelIndex"][:n][hit]
    return sr
