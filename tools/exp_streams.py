#!/usr/bin/env python3
"""Launch tails vs concurrent streams (one GPU): the C2 frame (or one rank's tile shard of it) split
into S tile-interleaved parts, each traced by its own engine context on its own stream.

A persistent trace launch ends with a drain: once its queue is dry, the ~16% of its rays in flight
finish on ever fewer, sparser waves. On one stream the next launch waits for that
tail; with S streams, part s's launches overlap the other parts' tails. Dependencies are kept per
part: part s's bounce-1 launch follows its own primary launch on its stream (as shading would).

Usage: exp_streams.py [--world N --rank R] [--parts 1,2,3,4] [--weights "2:1;3:2"] [--native] [--steps 20]
--weights: unequal splits (part s takes w_s of every sum(w) consecutive tiles of the shard), so the
parts' launches end at different times. --native (world 1): a row for the single full-frame launch
in the kernel's own 8x8-tile swizzle order (a 1-part tile-order batch of W*H rays would be
swizzled a second time).
Prints one JSON document: per S, wall ms per frame step and Grays/s, and whether the union of the
parts' primary hit records equals one launch over the whole shard.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--parts", default="1,2,3,4")
    ap.add_argument("--weights", default="")
    ap.add_argument("--native", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch
    import tthip
    import ttdist

    W, H, far = 1920, 1080, 1000.0
    WH = W * H
    dev = torch.device("cuda:0")
    blas = tthip.Blas(tthip.Mesh.sponza())
    am = tthip.AssetManager()
    am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
    scene = am.build()
    c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    base = torch.cuda.Stream(dev)
    torch.cuda.set_stream(base)
    eng0 = tthip.Engine(0, stream=base.cuda_stream)
    eng0.upload(scene)
    full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
    eng0.generate(full, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
    # reference: one launch over the whole shard
    shard = torch.from_numpy(ttdist.tile_pixels(W, H, a.world, a.rank)).to(dev)
    one = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    one.view(2 * WH, 48)[: shard.shape[0]] = full.view(WH, 48)[shard]
    eng0.trace(one, int(shard.shape[0]), 0, far, W, H, device=True)
    ref_hits = one.view(2 * WH, 48)[: shard.shape[0], 32:48].clone()
    del one
    out = {"tool": "tools/exp_streams.py", "world": a.world, "rank": a.rank, "shard_rays": int(shard.shape[0]),
           "rows": []}
    engines = [eng0]
    shard_np = ttdist.tile_pixels(W, H, a.world, a.rank)
    # tile id (within the shard's tile sequence) of every shard pixel, for the weighted splits
    tx = (W + 63) // 64
    gt = (shard_np // W) // 64 * tx + (shard_np % W) // 64
    _, tile_of = np.unique(gt, return_inverse=True)  # shard tiles are in increasing global id order

    def split_pixels(weights):
        SW = sum(weights)
        cum = np.cumsum([0] + list(weights))
        slot = tile_of % SW
        return [shard_np[(slot >= cum[s]) & (slot < cum[s + 1])] for s in range(len(weights))]

    def timed(step, parts_rays):
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / a.steps

    if a.native and a.world == 1:
        rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
        rays[: WH * 48] = full
        eng0.trace(rays, WH, 0, far, W, H, info=info, device=True)
        nb = eng0.enqueue_bounce(rays, WH, 0, far, W, H, frames=0, max_bounce=1, device=True)

        def nstep():
            eng0.trace(rays, WH, 0, far, W, H, info=info, device=True, asynchronous=True)
            eng0.trace(rays, nb, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)

        dt = timed(nstep, None)
        row = {"parts": "native", "ms_per_step": round(dt * 1e3, 4), "grays_s": round((WH + nb) / dt / 1e9, 3),
               "rays_per_step": WH + nb}
        out["rows"].append(row)
        print(f"[streams] {row}", file=sys.stderr, flush=True)
        del rays, info
    specs = [[1] * int(x) for x in a.parts.split(",") if x] + \
        [[int(w) for w in x.split(":")] for x in a.weights.split(";") if x]
    for weights in specs:
        S = len(weights)
        streams = [base] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
        while len(engines) < S:
            e = tthip.Engine(0, stream=streams[len(engines)].cuda_stream)
            e.upload(scene)
            engines.append(e)
        parts = []
        for s in range(S):
            eng = engines[s]
            pix = torch.from_numpy(split_pixels(weights)[s]).to(dev)
            n = int(pix.shape[0])
            with torch.cuda.stream(streams[s]):
                rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
                info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            rays.view(2 * WH, 48)[:n] = full.view(WH, 48)[pix]
            torch.cuda.synchronize(dev)
            eng.trace(rays, n, 0, far, W, H, info=info, device=True)
            nb = eng.enqueue_bounce(rays, n, 0, far, W, H, frames=0, max_bounce=1, device=True)
            torch.cuda.synchronize(dev)
            parts.append((eng, rays, info, pix, n, nb))
        # parity: the parts' primary hit records, in shard order, equal one launch over the shard
        got = torch.zeros((WH, 16), dtype=torch.uint8, device=dev)
        for eng, rays, info, pix, n, nb in parts:
            got[pix] = rays.view(2 * WH, 48)[:n, 32:48]
        same = bool(torch.equal(got[shard], ref_hits))

        def step():
            for eng, rays, info, pix, n, nb in parts:
                eng.trace(rays, n, 0, far, W, H, info=info, device=True, asynchronous=True)
            for eng, rays, info, pix, n, nb in parts:
                eng.trace(rays, nb, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)

        dt = timed(step, None)
        rays_step = sum(p[4] + p[5] for p in parts)
        row = {"parts": S, "weights": weights, "ms_per_step": round(dt * 1e3, 4), "grays_s": round(rays_step / dt / 1e9, 3),
               "rays_per_step": rays_step, "identical_primary_hits": same}
        out["rows"].append(row)
        print(f"[streams] {row}", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
