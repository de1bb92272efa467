#!/usr/bin/env python3
"""Latency of the longest rays of the C2 no-jitter primary batch (the launch tail).

With SURVEY §8(d)'s unjittered camera, screen column x = 960 has direction.z == -0.0 exactly, so
its rays' z slabs are NaN (inf * 0) and every box passes in z: ~900 node visits and ~1,600
triangle tests per ray (oracle counts), one of them exhausting Reps. A launch cannot end before
its longest ray, so these serial chains set the primary launch time. This times, on one GPU,
launches that contain only such rays (1, 8, 64, the whole column) and the full frame, and prints
the per-step latency of a lone ray (launch time / (nodes + triangles)).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    import torch
    import tthip
    import ttconfigs as T

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    sc = T.c2_sponza()
    eng.upload(sc)
    W, H = 1920, 1080
    WH = W * H
    c2w, ip = T.C2_VIEW.camera(W, H)
    full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
    eng.generate(full, c2w, ip, W, H, T.NEAR, T.FAR, jitter=0, frames=0, max_bounce=1, device=True)
    st = eng.trace(full.clone(), WH, 0, T.FAR, W, H, device=True, stats=True)
    out = {"tool": "tools/long_rays.py", "full_frame": {"rays": WH, "nodes": st.node_visits, "tris": st.tri_tests}}

    def timed(rays_u8, n, steps=10):
        buf = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        buf[: n * 48] = rays_u8[: n * 48]
        s = eng.trace(buf.clone(), n, 0, T.FAR, W, H, device=True, stats=True)
        eng.timing_reset()
        for _ in range(steps):
            eng.trace(buf, n, 0, T.FAR, W, H, device=True, asynchronous=True)
        ms = float(np.median(eng.timing_read()))
        return ms, s

    ms, s = timed(full, WH)
    out["full_frame"]["ms"] = ms
    col = torch.arange(H, device=dev) * W + 960
    sel = {"lone_reps_ray": torch.tensor([540 * W + 960], device=dev), "col960_8": col[500:508],
           "col960_64": col[480:544], "col960_all": col, "col959_all": col - 1}
    for name, idx in sel.items():
        r = full.view(WH, 48)[idx].contiguous().view(-1)
        n = int(idx.shape[0])
        ms, s = timed(r, n)
        steps = (s.node_visits + s.tri_tests) / n
        out[name] = {"rays": n, "ms": round(ms, 4), "nodes_per_ray": round(s.node_visits / n, 1),
                     "tris_per_ray": round(s.tri_tests / n, 1), "reps_exhausted": s.reps_exhausted,
                     "ns_per_step_if_serial": round(ms * 1e6 / max(steps, 1), 1)}
        print(f"[long_rays] {name}: {out[name]}", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
