#!/usr/bin/env python3
"""The C5 one-launch tail: the 4K San-Miguel-shaped frame bench.py generates
(frames_accumulated = 0 jitter) holds one ray with direction.x == +0.0 (pixel 5,652,973) whose
infinite / NaN x slabs make it visit ~529 nodes and test ~1,134 triangles; its dependent chain sets the
one-launch frame time. Measured here, HIP events on the engine stream, median of --reps:

  alone            the ray as a one-ray launch (the whole chip to itself: the drain phase gives it 8 lanes)
  frame            the full frame, one launch, the kernel's own 8x8 tile order
  list             the full frame as a compacted ray list (tile order, no swizzle)
  list_first       the same list with the long ray's 64-ray chunk moved to the front (dequeued first)
  list_without     the same list without the long ray (its chunk's other 63 rays kept)

Per-step latency alone = alone / (node visits + triangle passes of the ray, TT_TRACE_STATS counts);
under load the chain ends no earlier than list_first's launch. Output: JSON on stdout."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))

PIXEL = 5652973


def main():
    import torch

    import tthip
    import ttconfigs as T

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    tthip.set_build_engine(eng, min_tris=100_000)
    sc = T.c5_san_miguel()
    eng.upload(sc)
    W, H, far = 3840, 2160, T.FAR
    WH = W * H
    c2w, ip = T.C5_VIEW.camera(W, H)
    full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
    eng.generate(full, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
    torch.cuda.synchronize(dev)
    d = full.view(WH, 48)[PIXEL, 16:28].view(torch.float32).cpu().numpy()
    out = {"tool": "tools/long_ray_chain.py", "pixel": PIXEL, "direction": [float(x) for x in d],
           "direction_x_bits": hex(int(np.float32(d[0]).view(np.uint32))), "reps": reps}

    def timed(buf, n, w=W, h=H):
        src = buf.clone()
        for _ in range(2):
            eng.trace(buf, n, 0, far, w, h, device=True, asynchronous=True)
        eng.timing_reset()
        for _ in range(reps):
            buf.copy_(src)
            eng.trace(buf, n, 0, far, w, h, device=True, asynchronous=True)
        ms = np.asarray(eng.timing_read(), np.float64)
        return round(float(np.median(ms)), 4)

    one = full.view(WH, 48)[PIXEL:PIXEL + 1].contiguous().view(-1)
    st = eng.trace(one.clone(), 1, 0, far, W, H, device=True, stats=True)
    out["ray_node_visits"] = int(st.node_visits)
    out["ray_tri_tests"] = int(st.tri_tests)
    out["alone_ms"] = timed(one, 1)
    steps = st.node_visits + st.tri_tests
    out["alone_ns_per_step_upper"] = round(out["alone_ms"] * 1e6 / max(steps, 1), 1)
    out["frame_ms"] = timed(full.clone(), WH)
    import ttdist

    order = torch.from_numpy(ttdist.tile_pixels(W, H, 1, 0)).to(dev)
    lst = full.view(WH, 48)[order].contiguous().view(-1)
    # (a list of exactly W*H rays would get the kernel's full-frame 8x8 swizzle on top: a screen height of
    # H + 8 keeps the list order; no _PrimaryTriangleInfo is written, so H is not used otherwise)
    out["list_ms"] = timed(lst.clone(), WH, h=H + 8)
    pos = int((order == PIXEL).nonzero()[0, 0].item())
    c0 = pos // 64 * 64
    idx = torch.cat([torch.arange(c0, c0 + 64, device=dev), torch.arange(0, c0, device=dev),
                     torch.arange(c0 + 64, WH, device=dev)])
    first = lst.view(WH, 48)[idx].contiguous().view(-1)
    out["list_first_ms"] = timed(first, WH, h=H + 8)
    keep = torch.ones(WH, dtype=torch.bool, device=dev)
    keep[pos] = False
    without = lst.view(WH, 48)[keep].contiguous().view(-1)
    out["list_without_ms"] = timed(without, WH - 1, h=H + 8)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
