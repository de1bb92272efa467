#!/usr/bin/env python3
"""How evenly a tile-to-rank deal spreads a frame's work (CPU only: the oracle's per-ray counts).

Traces the C2 frame (primary + bounce 1, the bench's jittered Generate) with the oracle, takes every
ray's dependent steps (node visits + triangle tests) and its pixel's 64x64 (or --tile) screen tile,
and reports per deal and N: the largest rank's summed steps over the mean (the issue-bound part of a
rank's frame time) and the longest single-ray chain per rank (the latency floor of its launches).

Deals: rr = tile t to rank t mod N (ttdist.tile_pixels); diag-K = tile (col, row) to rank
(col + K * row) mod N. Usage: tools/tile_balance.py [--config c2] [--tile 64] [--ns 2,4,8] [--threads 8]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--deals", default="rr,diag-1,diag-3")
    args = ap.parse_args()
    import oracle_ctypes as O
    import ttconfigs as T

    if args.config != "c2":
        raise SystemExit("only c2 (the metric's frame) is wired")
    sc = T.c2_sponza()
    W, H = 1920, 1080
    c2w, ip = T.C2_VIEW.camera(W, H)
    rays = O.generate(c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1)
    WH = W * H
    pix0 = rays["PixelIndex"][:WH].astype(np.int64) if "PixelIndex" in rays.dtype.names else np.arange(WH)
    st, c0 = O.trace(sc, rays, WH, 0, T.FAR, W, H, counts=True, nthreads=args.threads)
    assert st == 0
    nb = O.enqueue_bounce(sc, rays, WH, 0, T.FAR, W, H, frames=0, max_bounce=1)
    bounce = rays[WH:WH + nb].copy()
    both = np.zeros(WH + nb, rays.dtype)
    both[WH:] = bounce
    st, c1 = O.trace(sc, both, nb, 1, T.FAR, W, H, counts=True, nthreads=args.threads)
    assert st == 0
    c1 = c1[:nb]
    pix1 = bounce["PixelIndex"].astype(np.int64)
    steps0 = c0["node_visits"].astype(np.int64) + c0["tri_tests"]
    steps1 = c1["node_visits"].astype(np.int64) + c1["tri_tests"]
    tx, ty = (W + args.tile - 1) // args.tile, (H + args.tile - 1) // args.tile

    def tile_of(p):
        return (p // W // args.tile) * tx + (p % W) // args.tile

    n_t = tx * ty
    work = np.bincount(tile_of(pix0), steps0, n_t) + np.bincount(tile_of(pix1), steps1, n_t)
    chain = np.zeros(n_t, np.int64)
    np.maximum.at(chain, tile_of(pix0), steps0)
    np.maximum.at(chain, tile_of(pix1), steps1)
    col, row = np.arange(n_t) % tx, np.arange(n_t) // tx
    out = {"tool": "tools/tile_balance.py", "config": args.config, "tile": args.tile, "tiles": [tx, ty],
           "steps_total": int(work.sum()), "deals": {}}
    for deal in args.deals.split(","):
        rows = []
        for n in [int(x) for x in args.ns.split(",")]:
            if deal == "rr":
                rank = np.arange(n_t) % n
            else:
                k = int(deal.split("-")[1])
                rank = (col + k * row) % n
            per = np.bincount(rank, work, n)
            ch = np.zeros(n, np.int64)
            np.maximum.at(ch, rank, chain)
            rows.append({"n": n, "max_over_mean_steps": round(float(per.max() / per.mean()), 4),
                         "per_rank_steps_rel": [round(float(v / per.mean()), 3) for v in per],
                         "longest_chain_per_rank": ch.tolist()})
        out["deals"][deal] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
