"""Shared GPU-vs-oracle helpers for the -m gpu parity tests (test infrastructure: the oracle is
only ever the checker here)."""
import numpy as np

import oracle_ctypes as O

FAR = 1000.0
CPU_THREADS = 16


def trace_both(engine, sc, rays, n, bounce, W, H, info=True, colors=None, flags=0, upload=True):
    if upload:
        engine.upload(sc)
    rg, rc = rays.copy(), rays.copy()
    ig = np.zeros((W * H, 4), np.uint32) if info else None
    ic = np.zeros((W * H, 4), np.uint32) if info else None
    s = engine.trace(rg, n, bounce, FAR, W, H, info=ig, colors=colors, flags=flags, stats=True)
    st, cnt = O.trace(sc, rc, n, bounce, FAR, W, H, info=ic, colors=colors, flags=flags, counts=True,
                      nthreads=CPU_THREADS)
    assert st == 0
    return rg, rc, ig, ic, s, cnt


def assert_same(rg, rc, ig, ic, off, n):
    hg, hc = rg["hits"][off:off + n], rc["hits"][off:off + n]
    bad = np.nonzero((hg != hc).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} of {n} hit records differ, first {bad[:5]}: {hg[bad[:3]]} vs {hc[bad[:3]]}"
    # byte comparison: ray fields may legitimately hold NaNs (degenerate inputs)
    assert np.array_equal(np.ascontiguousarray(rg).view(np.uint8), np.ascontiguousarray(rc).view(np.uint8)), \
        "bytes outside the hit records must be untouched"
    if ig is not None:
        badi = np.nonzero((ig != ic).any(1))[0]
        assert len(badi) == 0, f"{len(badi)} _PrimaryTriangleInfo texels differ"


def same_floats(a, b) -> bool:
    """Float outputs compare bit for bit, except that any two NaNs are equal: the NaN a CPU and a
    GPU produce for the same invalid operation differ in sign / payload (x86 default NaN is
    0xFFC00000, gfx950 0x7FC00000) and neither the reference nor D3D defines it."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    same_bits = a.view(np.uint32) == b.view(np.uint32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(same_bits | both_nan))


def bounce_rays(scene, rays, W, H, seed):
    """Seeded bounce-1 rays from the primary hits in rays[:W*H] (second half of the ping-pong
    buffer): origin = hit point + 1e-3 * geometric normal (world space, facing the incoming ray),
    direction = a random unit vector in that hemisphere. Returns (rays, count)."""
    import tthip  # noqa: F401  (dtype only)

    n = W * H
    rng = np.random.default_rng(seed)
    h = rays["hits"][:n]
    idx = np.nonzero(h[:, 1] != 0xFFFFFFFF)[0]
    t = h[idx, 2].view(np.float32)
    o = rays["origin"][idx] + rays["direction"][idx] * t[:, None]
    tri = scene.tris[h[idx, 1].astype(np.int64)]
    ng = np.cross(tri["posedge1"], tri["posedge2"]).astype(np.float64)
    md = scene.meshdata[h[idx, 0].astype(np.int64)]
    w2l = md["W2L"].reshape(-1, 4, 4).transpose(0, 2, 1)[:, :3, :3]
    ng = np.einsum("nji,nj->ni", w2l, ng)
    ng /= np.linalg.norm(ng, axis=1, keepdims=True) + 1e-30
    ng *= np.where((ng * rays["direction"][idx]).sum(1, keepdims=True) > 0, -1.0, 1.0)
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
