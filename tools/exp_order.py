#!/usr/bin/env python3
"""Experiment: TT_TRACE_ADAPTIVE_ORDER on the bench workloads, as a renderer uses it -- every step is a
new jittered frame (two frames' rays resident, alternating), so the order a launch dequeues in comes
from the previous frame's per-tile costs, never from its own rays.

  --config c2|c4|c5   scene + view (C2 Sponza-shaped 1080p, C4 Bistro-shaped 1080p, C5 4K primary only)
  --parts P           1: one launch per bounce; P > 1: the bench's tile-interleaved parts on P streams

Per mode (off / adaptive) and interleaved rounds: wall ms per step (primary + bounce-1 of one frame;
all parts) and, for P = 1, the per-launch HIP-event ms. Prints one JSON document."""
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
    ap.add_argument("--config", default="c2")
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ranks", type=int, default=1, help="trace rank 0's 64x64-tile shard of an N-GPU frame")
    ap.add_argument("--primary-only", action="store_true", help="flag the primary launches only")
    ap.add_argument("--tile", type=int, default=64, help="part split tile edge (ttdist's default 64)")
    ap.add_argument("--share", action="store_true", help="parts > 0 trace part 0's scene (tt_ctx_share_scene)")
    args = ap.parse_args()
    import torch
    import tthip
    import ttconfigs as T
    import ttdist

    dev = torch.device("cuda", 0)
    main_stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(main_stream)
    if args.config == "c2":
        sc, view, W, H, nb = T.c2_sponza(), T.C2_VIEW, 1920, 1080, 1
    elif args.config == "c4":
        sc, view, W, H, nb = T.c4_bistro(), T.C4_VIEW, 1920, 1080, 1
    else:
        sc, view, W, H, nb = T.c5_san_miguel(), T.C5_VIEW, 3840, 2160, 0
    WH = W * H
    far = T.FAR
    P = args.parts
    engs, streams = [], []
    for s in range(P):
        st = main_stream if s == 0 else torch.cuda.Stream(dev)
        e = tthip.Engine(0, stream=st.cuda_stream)
        if s > 0 and args.share:
            e.share_scene(engs[0])
        else:
            e.upload(sc)
        engs.append(e)
        streams.append(st)
    c2w, ip = view.camera(W, H)
    info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    if args.ranks > 1:
        pix_parts = ttdist.part_pixels(W, H, args.ranks, 0, P, tile=args.tile)
    else:
        pix_parts = [np.arange(WH)] if P == 1 else ttdist.part_pixels(W, H, 1, 0, P, tile=args.tile)
    # frames[f][s] = (rays buffer, n primary, n bounce) of part s of jittered frame f
    frames = []
    full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
    for f in range(2):
        engs[0].generate(full, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=f, max_bounce=1, device=True)
        fr = []
        for s, pix in enumerate(pix_parts):
            buf = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            n = len(pix)
            buf.view(2 * WH, 48)[:n] = full.view(WH, 48)[torch.from_numpy(np.asarray(pix)).to(dev)]
            torch.cuda.synchronize(dev)
            m = 0
            if nb:
                engs[s].trace(buf, n, 0, far, W, H, device=True)
                m = engs[s].enqueue_bounce(buf, n, 0, far, W, H, frames=f, max_bounce=1, device=True)
            fr.append((buf, n, m))
        frames.append(fr)
    torch.cuda.synchronize(dev)
    rays_per = [sum(n + m for _, n, m in fr) for fr in frames]

    def step(k, flags):
        fr = frames[k & 1]
        for s in range(P):
            buf, n, m = fr[s]
            engs[s].trace(buf, n, 0, far, W, H, info=info, device=True, asynchronous=True, flags=flags)
        if nb:
            for s in range(P):
                buf, n, m = fr[s]
                engs[s].trace(buf, m, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True,
                              flags=0 if args.primary_only else flags)

    out = {"tool": "tools/exp_order.py", "config": args.config, "parts": P, "ranks": args.ranks, "primary_only": args.primary_only, "share": args.share, "width": W, "height": H,
           "rays_per_step": rays_per, "rounds": []}
    for r in range(args.rounds):
        rec = {}
        for mode, flags in (("off", 0), ("adaptive", tthip.TT_TRACE_ADAPTIVE_ORDER)):
            for k in range(6):
                step(k, flags)
            torch.cuda.synchronize(dev)
            for e in engs:
                e.timing_reset()
            t0 = time.perf_counter()
            for k in range(args.steps):
                step(k, flags)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            rays = sum(rays_per[k & 1] for k in range(args.steps))
            d = {"ms_per_step": round(ms, 4), "grays_s": round(rays / args.steps / ms / 1e6, 3)}
            if P == 1:
                per = (nb + 1)
                t = np.asarray(engs[0].timing_read(), np.float64)
                rows = min(args.steps, 256 // per)
                t = t[-rows * per:].reshape(rows, per)
                d["launch_ms"] = [round(float(x), 4) for x in t.mean(0)]
            rec[mode] = d
        out["rounds"].append(rec)
        print(r, json.dumps(rec), file=sys.stderr, flush=True)
    for e in reversed(engs):
        e.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
