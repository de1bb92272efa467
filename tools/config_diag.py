#!/usr/bin/env python3
"""Per-config work and SIMD-efficiency counters of the closest-hit kernel (the inputs of the
issue-bound ceiling model): for each config's launches, the HIP-event time of the
product kernel (median of --steps) and, from the TT_TRACE_STATS instantiation, rays, node visits,
triangle tests, BLAS entries per ray and the wave-iteration counters (iterations, lanes busy in the
node / triangle phases, active lanes). Usage: python tools/config_diag.py [--configs c2,c4,c5,c2s]
(c2s = rank 0's C2 shard at 8 GPUs: ~260k primary rays). Prints one JSON document."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c4,c5,c2s")
    ap.add_argument("--steps", type=int, default=7)
    a = ap.parse_args()
    import torch
    import tthip
    import ttconfigs as T
    import ttdist

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    out = {"tool": "tools/config_diag.py", "configs": {}}
    scenes = {}

    def scene(k):
        if k not in scenes:
            scenes.clear()
            scenes[k] = {"c2": T.c2_sponza, "c4": T.c4_bistro, "c5": T.c5_san_miguel}[k]()
        return scenes[k]

    for cfg in a.configs.split(","):
        base = "c2" if cfg == "c2s" else cfg
        sc = scene(base)
        view = {"c2": T.C2_VIEW, "c4": T.C4_VIEW, "c5": T.C5_VIEW}[base]
        eng.upload(sc)
        W, H = view.width, view.height
        WH = W * H
        c2w, ip = view.camera()
        rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        if cfg == "c2s":
            full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
            eng.generate(full, c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1, device=True)
            pix = torch.from_numpy(ttdist.tile_pixels(W, H, 8, 0)).to(dev)
            n0 = int(pix.shape[0])
            rays.view(2 * WH, 48)[:n0] = full.view(WH, 48)[pix]
            del full
        else:
            n0 = WH
            eng.generate(rays, c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1, device=True)
        pristine = rays.clone()
        launches = [(0, n0)]
        eng.trace(rays, n0, 0, T.FAR, W, H, device=True)
        if base != "c5":
            nb = eng.enqueue_bounce(rays, n0, 0, T.FAR, W, H, device=True)
            launches.append((1, nb))
        res = []
        for bounce, n in launches:
            def go(stats=False):
                return eng.trace(rays, n, bounce, T.FAR, W, H, device=True, stats=stats)
            go()
            eng.timing_reset()
            for _ in range(a.steps):
                go()
            ms = float(np.median(eng.timing_read()))
            s = go(stats=True)
            d = eng.diagnostics()
            it = max(d["iterations"], 1)
            res.append({"bounce": bounce, "rays": n, "kernel_ms": round(ms, 4),
                        "mrays_s": round(n / ms / 1e3, 1),
                        "nodes_per_ray": round(s.node_visits / max(n, 1), 3),
                        "tris_per_ray": round(s.tri_tests / max(n, 1), 3),
                        "blas_per_ray": round(s.blas_entries / max(n, 1), 3) if hasattr(s, "blas_entries") else None,
                        "wave_iters_per_ray": round(d["iterations"] / max(n, 1), 4),
                        "active_lanes_per_iter": round(d["active_lanes"] / it, 2),
                        "node_lanes_per_node_iter": round(d["node_lanes"] / max(d["node_iters"], 1), 2),
                        "node_iter_frac": round(d["node_iters"] / it, 3),
                        "tri_lanes_per_tri_iter": round(d["tri_lanes"] / max(d["tri_iters"], 1), 2),
                        "tri_iter_frac": round(d["tri_iters"] / it, 3),
                        "stats_kernel_ms": round(float(s.kernel_ms), 4)})
            rays.copy_(pristine)
            if bounce == 0 and len(launches) > 1:
                eng.trace(rays, n0, 0, T.FAR, W, H, device=True)
                eng.enqueue_bounce(rays, n0, 0, T.FAR, W, H, device=True)
        out["configs"][cfg] = res
        print(cfg, json.dumps(res), file=sys.stderr, flush=True)
        del rays, pristine
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
