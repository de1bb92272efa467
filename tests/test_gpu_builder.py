"""Row f4, builder half: the BVH2 stage of the BLAS build on the GPU (tt_bvh2_build_device,
csrc/tt_build.hip) must give exactly the trees the sequential BVH2Builder gives (BVH2Builder.cs:9-217,
restated on the host in host/tt_scene.cpp and pinned there by leaf orders the reference serialized,
tests/test_builder_pin.py). Compared byte for byte: FinalIndices, every BVH2 node (box, left, count),
the BVH2 depth, and after the BVH8 stage the CWBVH8 nodes, the leaf-ordered triangles and the leaf
order. Inputs cover SAH ties (duplicated and axis-aligned triangles, a grid), signed zeros, the
reference's own Pedestal asset, Unity's Cube, and the C2 Sponza-shaped mesh at full size.
"""
import os

import numpy as np
import pytest

import tthip

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _bvh2_host_and_device(engine, mesh):
    L = tthip.scene_lib()
    v = mesh.view()
    n = v.n_indices // 3
    aabbs = np.zeros((n, 6), np.float32)
    assert L.tt_blas_prepare_aabbs(v, aabbs.ctypes.data) == 0
    host = [np.zeros(n, np.int32), np.zeros((2 * n, 6), np.float32), np.zeros(2 * n, np.int32),
            np.zeros(2 * n, np.uint32)]
    assert L.tt_bvh2_build(aabbs.ctypes.data, n, *[a.ctypes.data for a in host]) == 0
    pre = np.zeros((3, n), np.int32)
    assert L.tt_bvh2_presort(aabbs.ctypes.data, n, pre.ctypes.data) == 0
    dev = [np.zeros_like(a) for a in host]
    depth = tthip.C.c_uint32(0)
    st = engine.L.tt_bvh2_build_device(engine.h, aabbs.ctypes.data, n, pre.ctypes.data,
                                       *[a.ctypes.data for a in dev], tthip.C.byref(depth))
    assert st == 0
    return host, dev, depth.value


def _same_blas(a: tthip.Blas, b: tthip.Blas):
    na, ta = a.arrays()
    nb, tb = b.arrays()
    assert na.tobytes() == nb.tobytes(), "CWBVH8 nodes differ"
    assert ta.tobytes() == tb.tobytes(), "leaf-ordered triangles differ"
    assert np.array_equal(a.leaf_order(), b.leaf_order())
    assert a.info.bvh2_depth == b.info.bvh2_depth


def _grid(nx, nz):  # a flat grid of quads: every SAH sweep is full of exact ties
    xs, zs = np.meshgrid(np.arange(nx + 1, dtype=np.float32), np.arange(nz + 1, dtype=np.float32), indexing="ij")
    pos = np.stack([xs.ravel(), np.zeros(xs.size, np.float32), zs.ravel()], 1)
    idx = []
    for i in range(nx):
        for j in range(nz):
            a, b, c, d = i * (nz + 1) + j, (i + 1) * (nz + 1) + j, i * (nz + 1) + j + 1, (i + 1) * (nz + 1) + j + 1
            idx += [a, b, c, c, b, d]
    return tthip.Mesh.from_arrays(pos, np.array(idx, np.int32))


def _meshes():
    z = np.load(os.path.join(HERE, "golden", "pedestal_mesh.npz"))
    cube = np.load(os.path.join(HERE, "golden", "unity_cube_pins.npz"))
    rng = np.random.default_rng(7)
    dup = rng.random((300, 3), dtype=np.float32) * 4 - 2
    dup_pos = np.concatenate([dup, dup, np.round(dup)])  # duplicated and snapped triangles
    dup_idx = np.arange(len(dup_pos), dtype=np.int32)
    signed = rng.integers(-2, 3, (600, 3)).astype(np.float32)
    signed[rng.random(signed.shape) < 0.3] = -0.0  # -0 and +0 coordinates
    return {
        "cornell": tthip.Mesh.cornell(),
        "pedestal": tthip.Mesh.from_arrays(z["positions"].astype(np.float32), z["indices"]),
        "unity_cube": tthip.Mesh.from_arrays(cube["cube_v"], cube["cube_i"]),
        "grid_40x25": _grid(40, 25),
        "duplicates": tthip.Mesh.from_arrays(dup_pos, dup_idx),
        "signed_zeros": tthip.Mesh.from_arrays(signed, np.arange(600, dtype=np.int32)),
        "soup_50k": tthip.Mesh.soup(11, 50_000),
        "single": tthip.Mesh.from_arrays(np.eye(3, dtype=np.float32), np.array([0, 1, 2], np.int32)),
    }


@pytest.mark.parametrize("name", list(_meshes().keys()))
def test_device_bvh2_equals_host_bvh2(engine, name):
    mesh = _meshes()[name]
    host, dev, depth = _bvh2_host_and_device(engine, mesh)
    for h, d, what in zip(host, dev, ("FinalIndices", "node boxes", "node left", "node count")):
        assert h.tobytes() == d.tobytes(), f"{name}: {what} differ"
    assert depth == tthip.Blas(mesh).info.bvh2_depth


@pytest.mark.parametrize("stages", ["bvh2", "bvh2+bvh8"])
@pytest.mark.parametrize("name", list(_meshes().keys()))
def test_blas_built_on_the_device_is_identical(engine, name, stages):
    mesh = _meshes()[name]
    _same_blas(tthip.Blas(mesh), tthip.Blas(mesh, engine=engine, device_stages=stages))


def test_sponza_c2_blas_device_build_identical_and_traces(engine):
    mesh = tthip.Mesh.sponza()
    t = {}
    a, b = tthip.Blas(mesh), tthip.Blas(mesh, engine=engine, timings=t)
    _same_blas(a, b)
    assert set(t) == {"prepare_s", "presort_s", "device_s", "assemble_s"}
    # and the device-built BLAS traces exactly like the host-built one (the same buffers)
    import ttconfigs as T
    am = tthip.AssetManager()
    am.add_parent(b, None, np.zeros(7, tthip.MAT_DTYPE))
    sc = am.build()
    W, H = 320, 180
    c2w, ip = T.C2_VIEW.camera(W, H)
    rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    engine.upload(sc)
    engine.generate(rays, c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1)
    import oracle_ctypes as O
    ref = rays.copy()
    engine.trace(rays, W * H, 0, T.FAR, W, H)
    assert O.trace(sc, ref, W * H, 0, T.FAR, W, H, nthreads=8)[0] == 0
    assert np.array_equal(rays["hits"], ref["hits"])


def _presorts(engine, mesh):
    L = tthip.scene_lib()
    v = mesh.view()
    n = v.n_indices // 3
    aabbs = np.zeros((n, 6), np.float32)
    assert L.tt_blas_prepare_aabbs(v, aabbs.ctypes.data) == 0
    host = np.zeros((3, n), np.int32)
    assert L.tt_bvh2_presort(aabbs.ctypes.data, n, host.ctypes.data) == 0
    dev = np.full((3, n), -1, np.int32)
    st = engine.L.tt_bvh2_presort_device(engine.h, aabbs.ctypes.data, n, dev.ctypes.data)
    return st, host, dev


def _snapped(n, seed):  # grid-snapped triangles: most centroid keys tie (the introsort's swap order decides)
    rng = np.random.default_rng(seed)
    pos = (np.round(rng.uniform(-4, 4, (3 * n, 3)) * 2) / 2).astype(np.float32)
    return tthip.Mesh.from_arrays(pos, np.arange(3 * n, dtype=np.int32))


@pytest.mark.parametrize("name", ["pedestal", "grid_40x25", "duplicates", "signed_zeros", "soup_50k", "snapped_80k"])
def test_device_presort_replays_the_dotnet_introsort(engine, name):
    mesh = _snapped(80_000, 5) if name == "snapped_80k" else _meshes()[name]
    st, host, dev = _presorts(engine, mesh)
    assert st == 0
    assert np.array_equal(host, dev)


def test_device_presort_declines_tiny_inputs(engine):
    st, _, _ = _presorts(engine, _meshes()["unity_cube"])  # 12 triangles: the host sorts
    assert st == tthip.TT_ERR_UNSUPPORTED
