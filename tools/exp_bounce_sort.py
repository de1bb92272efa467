#!/usr/bin/env python3
"""Experiment: does tracing the bounce-1 rays in a coherent order speed up the dominant launch?

The node fetch of the closest-hit kernel runs at ~0.59 of the scattered-fetch rate one MI355X sustains from
L2 (roofline.models.node_fetch), so secondary-ray coherence -- neighbouring lanes and waves visiting the same
nodes -- is the lever a reordering would pull. The trace's records do not depend on the order rays are
processed in, so a product form would dequeue through a permutation and write every record back to its own
slot; this experiment only asks what the launch time would be: it physically permutes the C2 bounce-1 ray
array by a key, traces it, and compares with the reference order (records in permuted slots, not compared).

Keys (per ray: origin o, direction d of the 48-B RayData):
  octant      direction octant only (3 bits)
  morton      30-bit Morton code of the origin in the scene box
  oct_morton  octant in the top 3 bits, then a 27-bit Morton code of the origin
  dir_morton  27-bit Morton code of the origin, then the direction octant in the low bits
The sort itself is timed too (torch.argsort + one gather of the 48-B records on the GPU).
Prints one JSON document."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def part1by2(x):
    import torch

    x = x & 0x3FF
    x = (x | (x << 16)) & 0x030000FF
    x = (x | (x << 8)) & 0x0300F00F
    x = (x | (x << 4)) & 0x030C30C3
    x = (x | (x << 2)) & 0x09249249
    return x


def main():
    import torch

    import tthip
    import ttconfigs as T

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    sc, view, W, H = T.c2_sponza(), T.C2_VIEW, 1920, 1080
    WH = W * H
    far = T.FAR
    eng = tthip.Engine(0, stream=st.cuda_stream)
    eng.upload(sc)
    c2w, ip = view.camera(W, H)
    rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    eng.generate(rays, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
    eng.trace(rays, WH, 0, far, W, H, device=True)
    nb = eng.enqueue_bounce(rays, WH, 0, far, W, H, frames=0, max_bounce=1, device=True)
    torch.cuda.synchronize(dev)
    bnc = rays.view(-1, 48)[WH:WH + nb].clone()
    f = bnc[:, :32].contiguous().view(torch.float32).view(nb, 8)
    o, d = f[:, 0:3], f[:, 4:7]
    lo, hi = o.min(0).values, o.max(0).values
    q = ((o - lo) / (hi - lo).clamp_min(1e-20) * 1023.0).clamp(0, 1023).to(torch.int64)
    mort = part1by2(q[:, 0]) | (part1by2(q[:, 1]) << 1) | (part1by2(q[:, 2]) << 2)
    octant = ((d[:, 0] < 0).to(torch.int64) << 2) | ((d[:, 1] < 0).to(torch.int64) << 1) | (d[:, 2] < 0).to(torch.int64)
    keys = {"octant": octant, "morton": mort, "oct_morton": (octant << 27) | (mort >> 3),
            "dir_morton": ((mort >> 3) << 3) | octant}

    def timed(buf, reps=30):
        for _ in range(3):
            eng.trace(buf, nb, 1, far, W, H, device=True, asynchronous=True)
        torch.cuda.synchronize(dev)
        eng.timing_reset()
        for _ in range(reps):
            eng.trace(buf, nb, 1, far, W, H, device=True, asynchronous=True)
        ms = np.asarray(eng.timing_read(), np.float64)
        return float(np.median(ms)), float(ms.mean())

    out = {"tool": "tools/exp_bounce_sort.py", "config": "c2 bounce-1", "rays": int(nb), "runs": {}}
    base = rays.clone()
    for rnd in range(2):
        med, mean = timed(base)
        out["runs"].setdefault("reference_order", []).append(round(med, 4))
        for name, k in keys.items():
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            perm = torch.argsort(k, stable=True)
            srt = base.clone()
            srt.view(-1, 48)[WH:WH + nb] = bnc[perm]
            torch.cuda.synchronize(dev)
            sort_ms = (time.perf_counter() - t0) * 1e3
            med, mean = timed(srt)
            out["runs"].setdefault(name, []).append(round(med, 4))
            out.setdefault("sort_and_gather_ms_host_timed", {})[name] = round(sort_ms, 3)
            del srt
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
