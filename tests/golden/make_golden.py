"""Generates the committed golden fixtures under tests/golden/ (run in the build container).

Each fixture holds the scene buffers produced by the builder restatement, input RayData
(primary rays from the camera restatement and seeded bounce-1 rays), and the expected
outputs (hit records, _PrimaryTriangleInfo, per-ray visit counts) computed by the CPU oracle.
The reference itself cannot run here (HLSL/Unity/.NET are absent), so these vectors pin the
oracle and the builder over time and are what the GPU must reproduce bit-for-bit; they are not
outputs of the reference (parity against reference outputs is unpinned).

pedestal_mesh.npz is the geometry of the reference's sample asset
TrueTrace/Models/ExampleScene/Pedestal/Pedestal.obj (48 triangles) converted to arrays with
Unity's OBJ import convention (x negated, face winding reversed); the .obj is only read when
/root/reference is present.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_ctypes as O  # noqa: E402
import tthip  # noqa: E402

FAR = 1000.0
PEDESTAL_OBJ = "/root/reference/TrueTrace/Models/ExampleScene/Pedestal/Pedestal.obj"


def pedestal_arrays():
    path = os.path.join(HERE, "pedestal_mesh.npz")
    if not os.path.exists(path):
        verts, faces = [], []
        for line in open(PEDESTAL_OBJ):
            t = line.split()
            if not t:
                continue
            if t[0] == "v":
                verts.append([-float(t[1]), float(t[2]), float(t[3])])
            elif t[0] == "f":
                idx = [int(x.split("/")[0]) - 1 for x in t[1:]]
                for k in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[k + 1], idx[k]])
        np.savez_compressed(path, positions=np.array(verts, np.float32), indices=np.array(faces, np.int32))
    z = np.load(path)
    return z["positions"], z["indices"]


def bounce_rays(scene, rays, W, H, seed):
    """Seeded bounce-1 rays from the primary hits: origin = hit point + 1e-3 * geometric normal
    (world space), direction = random unit vector in that hemisphere."""
    n = W * H
    rng = np.random.default_rng(seed)
    h = rays["hits"][:n]
    hit = h[:, 1] != 0xFFFFFFFF
    idx = np.nonzero(hit)[0]
    t = h[idx, 2].view(np.float32)
    o = rays["origin"][idx] + rays["direction"][idx] * t[:, None]
    tri = scene.tris[h[idx, 1].astype(np.int64)]
    ng = np.cross(tri["posedge1"], tri["posedge2"]).astype(np.float64)
    md = scene.meshdata[h[idx, 0].astype(np.int64)]
    w2l = md["W2L"].reshape(-1, 4, 4).transpose(0, 2, 1)[:, :3, :3]
    ng = np.einsum("nji,nj->ni", w2l, ng)  # normal to world: W2L^T n
    ng /= np.linalg.norm(ng, axis=1, keepdims=True) + 1e-30
    face = np.where((ng * rays["direction"][idx]).sum(1, keepdims=True) > 0, -1.0, 1.0)
    ng *= face
    d = rng.normal(size=(len(idx), 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = np.where((d * ng).sum(1, keepdims=True) < 0, -d, d)
    out = rays.copy()
    m = len(idx)
    out["origin"][n:n + m] = (o + 1e-3 * ng).astype(np.float32)
    out["direction"][n:n + m] = d.astype(np.float32)
    out["PixelIndex"][n:n + m] = rays["PixelIndex"][idx]
    out["hits"][n:n + m] = h[idx]
    return out, m


def make(name, scene, cam, W, H, seed):
    c2w, ip = tthip.unity_camera(*cam, W, H, 0.3, FAR)
    rays = O.generate(c2w, ip, W, H, 0.3, FAR)
    r0 = rays.copy()
    info0 = np.zeros((W * H, 4), np.uint32)
    st, c0 = O.trace(scene, r0, W * H, 0, FAR, W, H, info=info0, counts=True)
    assert st == 0, st
    r1, nb = bounce_rays(scene, r0, W, H, seed)
    r1_in = r1.copy()
    colors = np.zeros(W * H, tthip.COL_DTYPE)
    colors["Data"][:, 3] = np.where(np.arange(W * H) % 3 == 0, -1.0, 1.0)
    info1 = np.zeros((W * H, 4), np.uint32)
    st, c1 = O.trace(scene, r1, nb, 1, FAR, W, H, info=info1, colors=colors, counts=True)
    assert st == 0, st
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"), nodes=scene.nodes.view(np.uint8), tris=scene.tris.view(np.uint8),
        tlas=scene.tlas, meshdata=scene.meshdata.view(np.uint8), materials=scene.materials.view(np.uint8),
        tlas_nodes=np.int64(scene.tlas_nodes), width=W, height=H, far=FAR,
        rays0=rays[: W * H].view(np.uint8), hits0=r0["hits"][: W * H], info0=info0, counts0=c0.view(np.uint8),
        rays1=r1_in[W * H:W * H + nb].view(np.uint8), n1=np.int64(nb), hits1=r1["hits"][W * H:W * H + nb], info1=info1,
        colors=colors.view(np.uint8), counts1=c1.view(np.uint8))
    print(f"{name}: {len(scene.tris)} tris {len(scene.nodes)} nodes, {W}x{H}, "
          f"hits {(r0['hits'][:W*H,1] != 0xFFFFFFFF).sum()}, bounce rays {nb}, "
          f"nodes/ray {c0['node_visits'].mean():.1f}")


def scenes():
    out = {}
    out["cornell"] = (tthip.single_object_scene(tthip.Mesh.cornell()), ((0, 0, 3.4), (0, 0, -1), (0, 1, 0), 40))
    pos, idx = pedestal_arrays()
    out["pedestal"] = (tthip.single_object_scene(tthip.Mesh.from_arrays(pos, idx)),
                       ((0, 3.0, -9.0), (0, -0.3, 1), (0, 1, 0), 60))
    out["soup"] = (tthip.single_object_scene(tthip.Mesh.soup(2024, 2000, 1.0, 0.08)),
                   ((0.3, 0.2, 3.0), (0, 0, -1), (0, 1, 0), 50))
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(31, 600, 1.0, 0.1)), tthip.trs_matrix((0, 0, 0), 10.0, 1.0),
                  np.zeros(2, tthip.MAT_DTYPE))
    ip = am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(32, 800)), np.zeros(3, tthip.MAT_DTYPE))
    for k in range(6):
        am.add_instance(ip, tthip.trs_matrix((-6.0 + 2.5 * k, -1.0, -3.0 - k), 37.0 * k, 0.3 + 0.05 * k))
    out["instanced"] = (am.build(), ((0, 0.5, 2.5), (0, -0.15, -1), (0, 1, 0), 70))
    inv = tthip.single_object_scene(tthip.Mesh.cornell(), n_materials=4)
    inv.materials[1]["Tag"] = 1 << tthip.FLAG_INVISIBLE  # left wall invisible to primary rays
    out["invisible"] = (inv, ((0, 0, 3.4), (0, 0, -1), (0, 1, 0), 40))
    return out


if __name__ == "__main__":
    for i, (name, (scene, cam)) in enumerate(scenes().items()):
        make(name, scene, cam, 64, 48, 100 + i)
