#!/usr/bin/env python3
"""Experiment: how much of a launch is load-balance tail? Traces the C2 (--config c4: C4) primary (and bounce-1) rays
in three chunk orders -- the natural tile order, longest-chunk-first (LPT, per-ray step counts from
the oracle) and shortest-first -- as compacted batches (n_rays = W*H - 1 disables the tile swizzle, so
chunk c = records [64c, 64c+64)). Results are order-independent (each ray's traversal is its own);
only the kernel time changes. --ranks N uses rank 0's tile shard of an N-GPU frame.
Prints one JSON document."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ranks = int(sys.argv[sys.argv.index("--ranks") + 1]) if "--ranks" in sys.argv else 1
    cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c2"
    import torch
    import tthip
    import ttconfigs as T
    import ttdist
    import oracle_ctypes as O

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    sc, view = (T.c2_sponza(), T.C2_VIEW) if cfg == "c2" else (T.c4_bistro(), T.C4_VIEW)
    eng.upload(sc)
    W, H = view.width, view.height
    WH = W * H
    c2w, ip = view.camera()
    r = O.generate(c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1)
    # tile order (8x8 tiles row-major), or rank 0's 64x64 tiles of an N-rank frame
    if ranks > 1:
        pix = ttdist.tile_pixels(W, H, ranks, 0)
    else:
        pix = np.arange(WH).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1)
    base = np.zeros(2 * WH, tthip.RAY_DTYPE)
    n0 = len(pix)
    base[:n0] = r[pix]
    st, cnt = O.trace(sc, base.copy(), n0, 0, T.FAR, W, H, counts=True, nthreads=16)
    steps0 = cnt["node_visits"].astype(np.int64) + cnt["tri_tests"].astype(np.int64)
    out = {"tool": "tools/exp_lpt.py", "config": cfg, "ranks": ranks, "launches": {}}

    def chunk_max(steps, n):
        nch = (n + 63) // 64
        pad = np.zeros(nch * 64, np.int64)
        pad[:n] = steps
        return pad.reshape(nch, 64).max(1)

    def seg_sorted(cm, key_sign):
        """longest-first inside each of the kernel's 8 XCD segments (the screen bands stay per XCD)"""
        nch = len(cm)
        out = []
        for k in range(8):
            lo, hi = nch * k // 8, nch * (k + 1) // 8
            out.append(lo + np.argsort(key_sign * cm[lo:hi], kind="stable"))
        return np.concatenate(out)

    def run(name, recs, n, bounce, steps, steps_other=None, extra=None):
        nch = (n + 63) // 64
        cmax = chunk_max(steps, n)
        buckets = np.minimum(np.log2(cmax + 1).astype(np.int64) * 2, 31)  # ~16 coarse cost classes
        orders = {"natural": np.arange(nch), "lpt": np.argsort(-cmax, kind="stable"),
                  "spt": np.argsort(cmax, kind="stable"), "lpt_seg": seg_sorted(cmax, -1),
                  "lpt_bucket": np.argsort(-buckets, kind="stable")}
        if steps_other is not None:  # the cost map of ANOTHER jittered frame (temporal reuse)
            co = chunk_max(steps_other, n)
            orders["lpt_other_frame"] = np.argsort(-co, kind="stable")
            orders["lpt_seg_other_frame"] = seg_sorted(co, -1)
        for k, co in (extra or {}).items():  # chunk cost estimates from another frame, keyed by pixel tile
            orders["lpt_" + k] = np.argsort(-co, kind="stable")
            orders["lpt_seg_" + k] = seg_sorted(co, -1)
        res = {}
        for oname, o in orders.items():
            idx = (o[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)
            idx = idx[idx < n]
            buf = np.zeros(2 * WH, tthip.RAY_DTYPE)
            off = WH if bounce == 1 else 0
            buf[off: off + n] = recs[idx]
            t = torch.from_numpy(buf.view(np.uint8)).to(dev)
            nn = n - 1 if n == WH else n  # never the full-frame swizzle
            eng.trace(t, nn, bounce, T.FAR, W, H, device=True)
            eng.timing_reset()
            for _ in range(9):
                eng.trace(t, nn, bounce, T.FAR, W, H, device=True)
            ms = eng.timing_read()
            res[oname] = round(float(np.median(ms)), 4)
        res["rays"] = n
        res["steps_mean"] = round(float(steps.mean()), 2)
        res["steps_max"] = int(steps.max())
        out["launches"][name] = res
        print(name, res, file=sys.stderr, flush=True)

    r1 = O.generate(c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=1, max_bounce=1)
    b1 = np.zeros(2 * WH, tthip.RAY_DTYPE)
    b1[:n0] = r1[pix]
    st, cnt1 = O.trace(sc, b1, n0, 0, T.FAR, W, H, counts=True, nthreads=16)
    steps0_other = cnt1["node_visits"].astype(np.int64) + cnt1["tri_tests"].astype(np.int64)
    nodes0_other = cnt1["node_visits"].astype(np.int64)
    run("primary", base[:n0], n0, 0, steps0, steps0_other,
        {"reps_other_frame": chunk_max(nodes0_other, n0)})
    # bounce-1 rays from the oracle's own enqueue of the traced primaries
    traced = base.copy()
    O.trace(sc, traced, n0, 0, T.FAR, W, H, nthreads=16)
    nb = O.enqueue_bounce(sc, traced, n0, 0, T.FAR, W, H)
    brec = traced[WH: WH + nb].copy()
    st, cb = O.trace(sc, traced, nb, 1, T.FAR, W, H, counts=True, nthreads=16)
    steps1 = cb["node_visits"].astype(np.int64) + cb["tri_tests"].astype(np.int64)
    # temporal estimate for the compacted bounce list: frame 1's bounce-1 cost per 8x8 pixel tile,
    # looked up through each chunk's PixelIndex (first record, or the max over all its records)
    tr1 = b1.copy()
    O.trace(sc, tr1, n0, 0, T.FAR, W, H, nthreads=16)
    nb1 = O.enqueue_bounce(sc, tr1, n0, 0, T.FAR, W, H, frames=1)
    st, cb1 = O.trace(sc, tr1, nb1, 1, T.FAR, W, H, counts=True, nthreads=16)
    s1 = cb1["node_visits"].astype(np.int64) + cb1["tri_tests"].astype(np.int64)
    r1n = cb1["node_visits"].astype(np.int64)
    ntile = (W // 8) * (H // 8)

    def tile_of(p):
        p = p.astype(np.int64)
        return (p // W // 8) * (W // 8) + (p % W) // 8

    def tile_map(pixels, cost):
        m = np.zeros(ntile, np.int64)
        np.maximum.at(m, tile_of(pixels), cost)
        return m

    p1 = tr1[WH: WH + nb1]["PixelIndex"] if "PixelIndex" in tr1.dtype.names else tr1[WH: WH + nb1]["pixel_index"]
    pb = brec["PixelIndex"] if "PixelIndex" in brec.dtype.names else brec["pixel_index"]
    M, Mr = tile_map(p1, s1), tile_map(p1, r1n)
    first = np.arange(0, nb, 64)
    # the SAME frame's primary costs per 8x8 tile (known before the bounce launch), through the
    # chunk's first record / all its records
    Mp = tile_map(base[:n0]["PixelIndex"], steps0)
    Mpr = tile_map(base[:n0]["PixelIndex"], cnt["node_visits"].astype(np.int64))
    est = {"prim_tile_first_rec": Mp[tile_of(pb[first])], "prim_tile_allrec": chunk_max(Mp[tile_of(pb)], nb),
           "prim_reps_tile_first_rec": Mpr[tile_of(pb[first])],
           "first_rec_other_frame": M[tile_of(pb[first])],
           "reps_first_rec_other_frame": Mr[tile_of(pb[first])],
           "allrec_other_frame": chunk_max(M[tile_of(pb)], nb)}
    run("bounce1", brec, nb, 1, steps1, None, est)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
