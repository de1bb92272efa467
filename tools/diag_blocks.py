#!/usr/bin/env python3
"""Per-block execution counts of the closest-hit kernel (TT_DIAG_BLOCKS build: `make variant NAME=diag
VFLAGS=-DTT_DIAG_BLOCKS`, run with TT_HIP_LIB=lib/variants/libtruetrace_hip_diag.so) on the bench's C2
workload -- the 1080p jittered primary launch and its compacted bounce-1 launch, one launch each -- or
C4 (argument c4). Counters (csrc/tt_trace.hip, tt_wide.h; wave executions unless noted):

  0 loop iterations        1 record-write batches   2 refill blocks        3 dequeues (atomics)
  4 ray setups             5 node-phase entries     6 node steps           7 pushes
  8 TLAS leaf -> BLAS      9 triangle passes       10 advance blocks      11 pops
 12 BLAS exits            13 drain-phase entries   14/15/16 drain iterations (G = 2/4/8)
 17 lanes in node steps   18 lanes in triangle passes   19 lanes refilled
 20/21/22 drain node steps (G = 2/4/8)   23 rays in drain node steps
 24/25/26 drain triangle passes (G = 2/4/8)   27 rays in drain triangle passes

Weighted by each block's static VALU count (tools/isa_blocks.py on the product kernel's ISA; the
table is --static JSON), this gives VALU per ray by block. Output: JSON on stdout."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))

NAMES = ["iterations", "record_batches", "refills", "dequeues", "ray_setups", "node_phase", "node_steps", "pushes",
         "tlas_leaf", "tri_passes", "advance", "pops", "blas_exits", "drain_entries", "drain_iters_g2",
         "drain_iters_g4", "drain_iters_g8", "lanes_node", "lanes_tri", "lanes_refilled", "drain_node_g2",
         "drain_node_g4", "drain_node_g8", "drain_node_rays", "drain_tri_g2", "drain_tri_g4", "drain_tri_g8",
         "drain_tri_rays"]


def main():
    import torch

    import tthip
    import ttconfigs as T

    assert "diag" in os.environ.get("TT_HIP_LIB", ""), "run with TT_HIP_LIB=<the TT_DIAG_BLOCKS build>"
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    scene_fn, view = {"c2": (T.c2_sponza, T.C2_VIEW), "c4": (T.c4_bistro, T.C4_VIEW)}[cfg]
    sc = scene_fn()
    dev = torch.device("cuda:0")
    cnt = torch.zeros(32, dtype=torch.int64, device=dev)
    os.environ["TT_DIAG_PTR"] = str(cnt.data_ptr())
    eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
    eng.upload(sc)
    W, H, far = 1920, 1080, T.FAR
    rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
    info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
    import numpy as np

    colors = np.zeros(W * H, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    c2w, ip = view.camera(W, H)
    eng.generate(rays, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
    out = {"tool": "tools/diag_blocks.py", "config": cfg, "launches": {}}
    n = W * H
    for b in (0, 1):
        if b == 1:
            n = eng.enqueue_bounce(rays, W * H, 0, far, W, H, frames=0, max_bounce=1, device=True)
        reps = 5
        torch.cuda.synchronize()
        cnt.zero_()
        for _ in range(reps):
            eng.trace(rays, n, b, far, W, H, info=info, colors=colors_t if b else None, device=True)
        torch.cuda.synchronize()
        c = [int(v) / reps for v in cnt.cpu().tolist()]
        rec = {"rays": int(n), "per_ray": {NAMES[k]: round(c[k] / n, 5) for k in range(len(NAMES))},
               "per_iteration": {NAMES[k]: round(c[k] / max(c[0], 1), 4) for k in range(1, 13)}}
        rec["lanes_per_node_step"] = round(c[17] / max(c[6], 1), 2)
        rec["lanes_per_tri_pass"] = round(c[18] / max(c[9], 1), 2)
        rec["lanes_per_refill"] = round(c[19] / max(c[4], 1), 2)
        rec["drain_node_share"] = round(c[23] / max(c[17] + c[23], 1), 4)
        out["launches"][f"bounce{b}"] = rec
        print(f"[diag] bounce {b}: {rec}", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
