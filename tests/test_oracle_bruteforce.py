"""An independent check of the oracle and the builder restatement: CWBVH8 traversal must find the
same closest triangle as a brute-force Moller-Trumbore over every triangle of every instance
(float64, numpy). Golden fixtures only pin the oracle against itself over time; this pins it
against geometry. Rays whose answer is numerically fragile in float32 (a hit within 1e-4 of a
triangle edge, or two candidates within 1e-4 relative in t) are excluded; everything else must
agree exactly on (mesh, triangle) and to 1e-5 relative in t, and misses must be misses."""
import numpy as np
import pytest

import oracle_ctypes as O
import tthip

FAR = 1000.0


def _brute(sc, origins, dirs, tri_ranges):
    """Closest hit per ray over all meshes: returns (t, mesh, tri, fragile) as float64 results."""
    n = len(origins)
    best_t = np.full(n, np.inf)
    best_mesh = np.zeros(n, np.int64)
    best_tri = np.full(n, -1, np.int64)
    second = np.full(n, np.inf)
    fragile = np.zeros(n, bool)
    p0_all = sc.tris["pos0"].astype(np.float64)
    e1_all = sc.tris["posedge1"].astype(np.float64)
    e2_all = sc.tris["posedge2"].astype(np.float64)
    for m, (lo, hi) in enumerate(tri_ranges):
        W = sc.meshdata["W2L"][m].reshape(4, 4).T.astype(np.float64)  # column-major -> row-major
        o = origins @ W[:3, :3].T + W[:3, 3]
        d = dirs @ W[:3, :3].T
        p0, e1, e2 = p0_all[lo:hi], e1_all[lo:hi], e2_all[lo:hi]
        for c in range(0, hi - lo, 2048):
            P0, E1, E2 = p0[c:c + 2048], e1[c:c + 2048], e2[c:c + 2048]
            h = np.cross(d[:, None, :], E2[None, :, :])
            a = np.einsum("tk,rtk->rt", E1, h)
            with np.errstate(divide="ignore", invalid="ignore"):
                f = 1.0 / a
                s = o[:, None, :] - P0[None, :, :]
                u = f * np.einsum("rtk,rtk->rt", s, h)
                q = np.cross(s, E1[None, :, :])
                v = f * np.einsum("rk,rtk->rt", d, q)
                t = f * np.einsum("tk,rtk->rt", E2, q)
            ok = (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t > 0) & (t < FAR)
            edge = ok & ((u < 1e-4) | (v < 1e-4) | (u + v > 1 - 1e-4) | (np.abs(a) < 1e-12))
            tt = np.where(ok, t, np.inf)
            for r in range(n):  # merge this chunk's candidates into the per-ray top two
                row = tt[r]
                k = int(np.argmin(row))
                if not np.isfinite(row[k]):
                    continue
                part = np.partition(row, 1)[:2] if len(row) > 1 else np.array([row[0], np.inf])
                cand_t, cand_2 = part[0], part[1]
                if cand_t < best_t[r]:
                    second[r] = min(best_t[r], cand_2)
                    best_t[r], best_mesh[r], best_tri[r] = cand_t, m, lo + c + k
                    fragile[r] = bool(edge[r, k])
                else:
                    second[r] = min(second[r], cand_t)
    with np.errstate(invalid="ignore"):
        close = np.isfinite(second) & (np.abs(second - best_t) <= 1e-4 * np.maximum(best_t, 1e-6))
    return best_t, best_mesh, best_tri, fragile | close


def _tri_ranges(sc):
    starts = sorted(set(int(x) for x in sc.meshdata["TriOffset"]))
    ends = {s: e for s, e in zip(starts, starts[1:] + [len(sc.tris)])}
    return [(int(t), ends[int(t)]) for t in sc.meshdata["TriOffset"]]


def _check(sc, rays, n):
    r = rays.copy()
    st, _ = O.trace(sc, r, n, 0, FAR, n, 1, nthreads=4)
    assert st == 0
    o = rays["origin"][:n].astype(np.float64)
    d = rays["direction"][:n].astype(np.float64)
    bt, bm, btri, fragile = _brute(sc, o, d, _tri_ranges(sc))
    hits = r["hits"][:n]
    got_t = hits[:, 2].view(np.float32).astype(np.float64)
    miss = ~np.isfinite(bt)
    assert np.all(hits[miss, 1] == 0xFFFFFFFF), "oracle hit something brute force misses"
    robust = ~miss & ~fragile
    assert robust.sum() > 0.3 * n
    assert np.array_equal(hits[robust, 1].astype(np.int64), btri[robust]), "different closest triangle"
    assert np.array_equal(hits[robust, 0].astype(np.int64), bm[robust]), "different mesh"
    assert np.allclose(got_t[robust], bt[robust], rtol=1e-5, atol=0)


def _random_rays(rng, n, center, spread):
    rays = np.zeros(2 * n, tthip.RAY_DTYPE)
    rays["origin"][:n] = center + rng.uniform(-spread, spread, (n, 3))
    d = rng.normal(size=(n, 3))
    rays["direction"][:n] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays["PixelIndex"][:n] = np.arange(n)
    return rays


@pytest.mark.parametrize("seed", [1, 2])
def test_single_blas_soup_matches_brute_force(seed):
    sc = tthip.single_object_scene(tthip.Mesh.soup(seed, 3000, 2.0, 0.2))
    rng = np.random.default_rng(seed)
    rays = _random_rays(rng, 400, np.zeros(3), 3.0)
    _check(sc, rays, 400)


def test_two_level_instances_match_brute_force():
    rng = np.random.default_rng(11)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.soup(5, 800, 6.0, 0.6)), tthip.trs_matrix((0, 0, 0)), np.zeros(2, tthip.MAT_DTYPE))
    props = [am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(100 + k, int(rng.integers(60, 400)))),
                                    np.zeros(2, tthip.MAT_DTYPE)) for k in range(3)]
    for i in range(12):
        am.add_instance(props[i % 3], tthip.trs_matrix(rng.uniform(-8, 8, 3) * [1, 0.2, 1],
                                                       float(rng.uniform(0, 360)), float(rng.uniform(0.4, 1.5))))
    sc = am.build()
    rays = _random_rays(rng, 300, np.array([0.0, 2.0, 0.0]), 8.0)
    _check(sc, rays, 300)


def test_sponza_shaped_c2_matches_brute_force():
    """C2's 262k-triangle BLAS (the bench scene), random rays from around the bench camera."""
    import ttconfigs as T

    sc = T.c2_sponza()
    rng = np.random.default_rng(3)
    rays = _random_rays(rng, 128, np.array(T.C2_VIEW.position), 1.0)
    _check(sc, rays, 128)
