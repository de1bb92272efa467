"""Minimal driver for rocprofv3 passes: builds the C2 workload (Sponza-shaped, 1080p primary +
bounce 1) and runs the trace kernel `--reps` times per bounce. No CPU baseline, no oracle."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402,F401
import tthip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--jitter", type=int, default=1)
ap.add_argument("--which", default="both")
args = ap.parse_args()
W, H, far = 1920, 1080, 1000.0
blas = tthip.Blas(tthip.Mesh.sponza())
am = tthip.AssetManager()
am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
sc = am.build()
dev = torch.device("cuda:0")
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=args.jitter, frames=0, max_bounce=1, device=True)
eng.trace(rays, W * H, 0, far, W, H, info=info, device=True)
nb = eng.enqueue_bounce(rays, W * H, 0, far, W, H, frames=0, max_bounce=1, device=True)
eng.timing_reset()
for _ in range(args.reps):
    if args.which in ("both", "primary"):
        eng.trace(rays, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
    if args.which in ("both", "bounce"):
        eng.trace(rays, nb, 1, far, W, H, device=True, asynchronous=True)
ms = eng.timing_read()
print("launch ms", np.round(ms, 4).tolist(), flush=True)
s = eng.trace(rays, W * H, 0, far, W, H, info=info, device=True, stats=True)
d = eng.diagnostics()
print("primary stats", s.as_dict(), d, flush=True)
print("  node-phase lane util %.3f tri-phase lane util %.3f active %.3f node iters/iter %.3f tri iters/iter %.3f" % (
    d["node_lanes"] / max(1, 64 * d["node_iters"]), d["tri_lanes"] / max(1, 64 * d["tri_iters"]),
    d["active_lanes"] / max(1, 64 * d["iterations"]), d["node_iters"] / d["iterations"], d["tri_iters"] / d["iterations"]))
s = eng.trace(rays, nb, 1, far, W, H, device=True, stats=True)
d = eng.diagnostics()
print("bounce stats", s.as_dict(), d, flush=True)
print("  node-phase lane util %.3f tri-phase lane util %.3f active %.3f node iters/iter %.3f tri iters/iter %.3f" % (
    d["node_lanes"] / max(1, 64 * d["node_iters"]), d["tri_lanes"] / max(1, 64 * d["tri_iters"]),
    d["active_lanes"] / max(1, 64 * d["iterations"]), d["node_iters"] / d["iterations"], d["tri_iters"] / d["iterations"]))
