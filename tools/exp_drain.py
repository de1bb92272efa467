#!/usr/bin/env python3
"""Experiment: the cost of a launch's drain. Traces the C2 primary rays (tile order, compacted) as
one batch of N rays and as two back-to-back copies in ONE launch (2N rays, a fake 1920x2160 screen
so the buffer holds them): steady-state time of N rays = t(2N) - t(N), drain overhead of one launch
= 2 t(N) - t(2N). Same for the bounce-1 rays. Prints one JSON document."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import tthip
    import ttconfigs as T
    import oracle_ctypes as O

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    sc = T.c2_sponza()
    eng.upload(sc)
    W, H = 1920, 1080
    WH = W * H
    c2w, ip = T.C2_VIEW.camera()
    r = O.generate(c2w, ip, W, H, T.NEAR, T.FAR, jitter=1, frames=0, max_bounce=1)
    pix = np.arange(WH).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1)
    prim = r[pix]
    traced = np.zeros(2 * WH, tthip.RAY_DTYPE)
    traced[:WH] = prim
    O.trace(sc, traced, WH, 0, T.FAR, W, H, nthreads=os.cpu_count() or 8)
    nb = O.enqueue_bounce(sc, traced, WH, 0, T.FAR, W, H)
    bnc = traced[WH: WH + nb].copy()
    out = {"tool": "tools/exp_drain.py", "launches": {}}
    H2 = 2 * H
    for name, recs, bounce in (("primary", prim, 0), ("bounce1", bnc, 1)):
        n = len(recs)
        res = {"rays": n}
        for reps in (1, 2):
            buf = np.zeros(2 * W * H2, tthip.RAY_DTYPE)
            off = W * H2 if bounce == 1 else 0
            for k in range(reps):
                buf[off + k * n: off + (k + 1) * n] = recs
            t = torch.from_numpy(buf.view(np.uint8)).to(dev)
            nn = reps * n
            eng.trace(t, nn, bounce, T.FAR, W, H2, device=True)
            eng.timing_reset()
            for _ in range(9):
                eng.trace(t, nn, bounce, T.FAR, W, H2, device=True)
            res[f"ms_x{reps}"] = round(float(np.median(eng.timing_read())), 4)
        res["steady_ms"] = round(res["ms_x2"] - res["ms_x1"], 4)
        res["drain_overhead_ms"] = round(2 * res["ms_x1"] - res["ms_x2"], 4)
        res["drain_frac"] = round(res["drain_overhead_ms"] / res["ms_x1"], 3)
        out["launches"][name] = res
        print(name, res, file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
