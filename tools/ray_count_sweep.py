#!/usr/bin/env python3
"""Single-GPU trace throughput against launch size (SURVEY.md §8(e) strong scaling).

Under tile sharding a rank traces only its 64x64 tiles: at 8 GPUs a 1080p frame is ~260k primary
rays per rank, fewer than the persistent grid's resident lanes. This measures, on one GPU, the
launches each rank of an N-GPU run would issue (rank 0's tiles = the largest shard) for N = 1, 2,
4, 8, and predicts the strong-scaling efficiency of the frame from them:

    t_frame(N) = t_primary(shard_N) + t_bounce(shard_N) [+ gather, reported separately]
    eff(N)     = t_frame(1) / (N * t_frame(N))

C2 (Sponza-shaped 1080p, primary + bounce 1, the reference's default jittered Generate), C4 (Bistro-shaped two-level 1080p, primary + bounce 1; --configs c4) and C5 (San-Miguel-shaped 4K primary). Every time is
a HIP-event launch time on the shared torch/engine stream (tt_timing_read), median of --steps.
Output: one JSON document on stdout (commit under profiles/).
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
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--configs", default="c2,c5")
    args = ap.parse_args()
    import torch
    import tthip
    import ttconfigs as T
    import ttdist

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    assert eng.stream == stream.cuda_stream
    out = {"tool": "tools/ray_count_sweep.py", "device": torch.cuda.get_device_name(0),
           "resident_lanes": None, "configs": {}}

    def timed(fn, steps):
        fn()
        eng.timing_reset()
        for _ in range(steps):
            fn()
        return np.asarray(eng.timing_read(), np.float64)

    def sweep(name, scene, view, W, H, bounces):
        eng.upload(scene)
        WH = W * H
        c2w, ip = view.camera(W, H)
        full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(full, c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1, device=True)
        rows = []
        for n_gpus in (1, 2, 4, 8):
            pix = torch.from_numpy(ttdist.tile_pixels(W, H, n_gpus, 0)).to(dev)
            n = int(pix.shape[0])
            rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
            rays.view(2 * WH, 48)[:n] = full.view(WH, 48)[pix]
            pristine = rays.clone()
            eng.trace(rays, n, 0, T.FAR, W, H, device=True)
            nb = eng.enqueue_bounce(rays, n, 0, T.FAR, W, H, frames=0, max_bounce=1, device=True) if bounces else 0
            ms_p = timed(lambda: eng.trace(pristine, n, 0, T.FAR, W, H, device=True, asynchronous=True), args.steps)
            ms_b = (timed(lambda: eng.trace(rays, nb, 1, T.FAR, W, H, device=True, asynchronous=True), args.steps)
                    if bounces else np.zeros(1))
            tp, tb = float(np.median(ms_p)), float(np.median(ms_b))
            rows.append({"n_gpus": n_gpus, "primary_rays": n, "bounce_rays": nb, "t_primary_ms": round(tp, 4),
                         "t_bounce_ms": round(tb, 4), "mrays_s_primary": round(n / tp / 1e3, 1),
                         "mrays_s_bounce": round(nb / tb / 1e3, 1) if bounces else None,
                         "t_frame_ms": round(tp + tb, 4)})
            del rays, pristine
            print(f"[sweep] {name} N={n_gpus}: {rows[-1]}", file=sys.stderr, flush=True)
        t1 = rows[0]["t_frame_ms"]
        for r in rows:
            r["predicted_efficiency"] = round(t1 / (r["n_gpus"] * r["t_frame_ms"]), 3)
            r["predicted_frame_mrays_s"] = round((rows[0]["primary_rays"] + rows[0]["bounce_rays"]) /
                                                 r["t_frame_ms"] / 1e3, 1)
        out["configs"][name] = {"width": W, "height": H, "tris": int(len(scene.tris)), "rows": rows}

    which = set(args.configs.split(","))
    if "c2" in which:
        sweep("c2_sponza_1080p_primary_plus_bounce1", T.c2_sponza(), T.C2_VIEW, 1920, 1080, True)
    if "c4" in which:
        t0 = time.time()
        sc = T.c4_bistro()
        print(f"[sweep] c4 build {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        sweep("c4_bistro_1080p_primary_plus_bounce1", sc, T.C4_VIEW, T.C4_VIEW.width, T.C4_VIEW.height, True)
    if "c5" in which:
        t0 = time.time()
        sc = T.c5_san_miguel()
        print(f"[sweep] c5 build {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        sweep("c5_san_miguel_4k_primary", sc, T.C5_VIEW, 3840, 2160, False)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
