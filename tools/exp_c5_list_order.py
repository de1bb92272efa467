#!/usr/bin/env python3
"""Experiment: why one full-frame C5 4K primary launch (8.3 M rays) takes longer than two sequential
half-frame launches of 64x64-tile-interleaved rays (profiles/r03/ray_count_sweep_cur.json: 2.25 ms vs
2 x 1.0 ms). The same 4K rays, one launch each way, interleaved rounds, HIP events on the stream:

  swizzle    the full frame in the kernel's 8x8-tile order (full-frame launches, what bench.py times)
  rowmajor   the full frame as a plain list (no swizzle: rays in pixel order)
  tile64     the full frame compacted in 64x64-tile order (ttdist.tile_pixels), as one list
  halves     the two tile-interleaved halves (ttdist.part_pixels, 2 parts) launched one after the other
  *_info     the same with _PrimaryTriangleInfo written (the INFO = 1 kernel bench.py's aux legs time)

Every form's hit records are compared with the swizzled launch's, pixel by pixel. Prints JSON."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--before", default="", help="comma list of configs uploaded + traced first on the same "
                    "engine (as bench.py's aux legs run), e.g. c2,c4")
    ap.add_argument("--burn", type=float, default=0.0, help="then trace the swizzled frame back to back for this "
                    "many seconds, reporting the launch time per 0.5 s window (clock / power drift)")
    ap.add_argument("--max-bounce", type=int, default=0, help="Generate's MaxBounce (seeds the jitter hash)")
    ap.add_argument("--only", default="", help="comma list of forms to time (default: all)")
    args = ap.parse_args()
    import torch
    import tthip
    import ttconfigs as T
    import ttdist

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    if args.config == "c5":
        sc, view, W, H = T.c5_san_miguel(), T.C5_VIEW, 3840, 2160
    elif args.config == "c4":
        sc, view, W, H = T.c4_bistro(), T.C4_VIEW, 1920, 1080
    else:
        sc, view, W, H = T.c2_sponza(), T.C2_VIEW, 1920, 1080
    WH = W * H
    far = T.FAR
    eng = tthip.Engine(0, stream=st.cuda_stream)
    for pre in [x for x in args.before.split(",") if x]:
        psc, pview = {"c2": (T.c2_sponza, T.C2_VIEW), "c4": (T.c4_bistro, T.C4_VIEW)}[pre]
        psc = psc()
        eng.upload(psc)
        pW, pH = 1920, 1080
        pc2w, pip = pview.camera(pW, pH)
        pb = torch.zeros(2 * pW * pH * 48, dtype=torch.uint8, device=dev)
        eng.generate(pb, pc2w, pip, pW, pH, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
        eng.trace(pb, pW * pH, 0, far, pW, pH, device=True)
        torch.cuda.synchronize()
        del pb, psc
    eng.upload(sc)
    c2w, ip = view.camera(W, H)
    base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    eng.generate(base, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=args.max_bounce, device=True)
    torch.cuda.synchronize()

    def compacted(pix):
        buf = torch.zeros(2 * max(len(pix), 1) * 48, dtype=torch.uint8, device=dev)
        idx = torch.from_numpy(np.asarray(pix, np.int64)).to(dev)
        buf.view(-1, 48)[: len(pix)] = base.view(-1, 48)[idx]
        return buf, idx

    tile_all = ttdist.tile_pixels(W, H, 1, 0)
    halves = ttdist.part_pixels(W, H, 1, 0, 2)
    bufs = {"swizzle": (base.clone(), None), "rowmajor": (base.clone(), None),
            "tile64": compacted(tile_all)}
    bufs["swizzle_info"] = (base.clone(), None)
    bufs["tile64_info"] = compacted(tile_all)
    info = torch.zeros((WH + W) * 16, dtype=torch.uint8, device=dev)
    half_bufs = [compacted(p) for p in halves]

    def run(name):
        """One launch (or the two halves back to back); ms from HIP events on the stream."""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if name == "halves":
            e0.record()
            for (b, _), p in zip(half_bufs, halves):
                eng.trace(b, len(p), 0, far, W, H + 1, device=True, asynchronous=True)
            e1.record()
        else:
            b, _ = bufs[name]
            h = H if name.startswith("swizzle") else H + 1  # W x (H+1) != n: a plain list, no 8x8-tile swizzle
            e0.record()
            eng.trace(b, WH, 0, far, W, h, info=info if name.endswith("_info") else None, device=True,
                      asynchronous=True)
            e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    names = ["swizzle", "rowmajor", "tile64", "halves", "swizzle_info", "tile64_info"]
    for n in names:
        run(n)  # warm-up + the records the check reads
    if args.only:
        names = args.only.split(",")
    ref = bufs["swizzle"][0].view(-1, 48)[:WH, 32:48]
    same = {"rowmajor": bool(torch.equal(bufs["rowmajor"][0].view(-1, 48)[:WH, 32:48], ref))}
    b, idx = bufs["tile64"]
    same["tile64"] = bool(torch.equal(b.view(-1, 48)[:WH, 32:48], ref[idx]))
    same["swizzle_info"] = bool(torch.equal(bufs["swizzle_info"][0].view(-1, 48)[:WH, 32:48], ref))
    same["halves"] = all(bool(torch.equal(hb.view(-1, 48)[: len(p), 32:48], ref[hidx]))
                         for (hb, hidx), p in zip(half_bufs, halves))
    times = {n: [] for n in names}
    for _ in range(args.rounds):
        for n in names:
            for _ in range(args.reps):
                times[n].append(run(n))
    # the same launch timed the way bench.py's aux legs time it: the engine's HIP-event ring
    b, _ = bufs["swizzle_info"]
    eng.timing_reset()
    for _ in range(args.reps):
        eng.trace(b, WH, 0, far, W, H, info=info, device=True, asynchronous=True)
    torch.cuda.synchronize()
    ring = [round(float(x), 4) for x in eng.timing_read()]
    out0 = {"ring_ms_swizzle_info": ring}
    out = {"config": args.config, "before": args.before, "rays": WH, **out0, "identical_to_swizzle": same,
           "ms_median": {n: round(float(np.median(v)), 4) for n, v in times.items()},
           "ms_min": {n: round(float(np.min(v)), 4) for n, v in times.items()}}
    if args.burn > 0:
        import time
        series, t_end = [], time.time() + args.burn
        b, _ = bufs["swizzle"]
        while time.time() < t_end:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k, t_w = 0, time.time() + 0.5
            e0.record()
            while time.time() < t_w:
                eng.trace(b, WH, 0, far, W, H, device=True, asynchronous=True)
                k += 1
                if k % 16 == 0:
                    torch.cuda.synchronize()
            e1.record()
            torch.cuda.synchronize()
            series.append(round(e0.elapsed_time(e1) / k, 4))
        out["burn_ms_per_launch_per_window"] = series
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
