#!/usr/bin/env python3
"""Does the order of the bounce-1 batch matter? The C2 bench's compacted bounce rays (source order,
as tt_enqueue_diffuse_bounce writes them) re-ordered on the GPU by direction octant at several
granularities -- within each 64-ray chunk (one wave's dequeue), within 4096-ray blocks, or over the
whole batch -- and traced; per-ray results are order-independent (checked), only the launch time
changes. Prints one JSON document."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    import torch
    import tthip

    W, H, far = 1920, 1080, 1000.0
    WH = W * H
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    blas = tthip.Blas(tthip.Mesh.sponza())
    am = tthip.AssetManager()
    am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
    sc = am.build()
    eng = tthip.Engine(0, stream=st.cuda_stream)
    eng.upload(sc)
    rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
    eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
    eng.trace(rays, WH, 0, far, W, H, device=True)
    nb = eng.enqueue_bounce(rays, WH, 0, far, W, H, frames=0, max_bounce=1, device=True)
    src = rays.view(2 * WH, 48)[WH:WH + nb].clone()
    d = src[:, 16:28].contiguous().view(torch.float32)
    octant = ((d[:, 0] < 0).int() * 4 + (d[:, 1] < 0).int() * 2 + (d[:, 2] < 0).int()).long()
    idx = torch.arange(nb, device=dev)

    def order_within(block):
        key = (idx // block) * 8 + octant
        return torch.sort(key * nb + idx).indices  # stable: by block, then octant, then source position

    orders = {"source": idx, "octant_in_64": order_within(64), "octant_in_4096": order_within(4096),
              "octant_global": order_within(nb)}
    ref = None
    out = {"tool": "tools/exp_bounce_sort.py", "bounce_rays": nb, "rows": {}}
    for name, perm in orders.items():
        buf = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        buf.view(2 * WH, 48)[WH:WH + nb] = src[perm]
        base = buf.clone()
        ms = []
        for k in range(13):
            buf.copy_(base)
            s = eng.trace(buf, nb, 1, far, W, H, device=True)
            if k >= 3:
                ms.append(s.kernel_ms)
        hits = torch.empty_like(src[:, 32:48])
        hits[perm] = buf.view(2 * WH, 48)[WH:WH + nb, 32:48]
        if ref is None:
            ref = hits
        same = bool(torch.equal(hits, ref))
        out["rows"][name] = {"trace_ms_median": round(float(np.median(ms)), 4),
                             "grays_s": round(nb / float(np.median(ms)) / 1e6, 3), "same_hits": same}
        print(f"[sort] {name}: {out['rows'][name]}", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
