"""Profiling driver for one BASELINE config (rocprofv3 passes): builds the config's scene, traces its
primary (+ bounce-1 for c2/c4) rays `--reps` times. Usage: python tools/prof_config.py c4 [--reps 3]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config", choices=["c2", "c4", "c5"])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--adaptive", action="store_true",
                help="primary launches with TT_TRACE_ADAPTIVE_ORDER, frames alternating (jitter frame = rep % 2)")
a = ap.parse_args()
sc, view, bounce = {"c2": (T.c2_sponza, T.C2_VIEW, True), "c4": (T.c4_bistro, T.C4_VIEW, True),
                    "c5": (T.c5_san_miguel, T.C5_VIEW, False)}[a.config]
sc = sc()
dev = torch.device("cuda:0")
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
W, H, far = view.width, view.height, T.FAR
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = view.camera()
eng.generate(rays, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
base = rays.clone()
frames = [base]
if a.adaptive:
    eng.generate(rays, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=1, max_bounce=1, device=True)
    frames.append(rays.clone())
for rep in range(a.reps):
    rays.copy_(frames[rep % len(frames)])
    s0 = eng.trace(rays, W * H, 0, far, W, H, device=True,
                   flags=tthip.TT_TRACE_ADAPTIVE_ORDER if a.adaptive else 0)
    if bounce:
        nb = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
        s1 = eng.trace(rays, nb, 1, far, W, H, device=True)
torch.cuda.synchronize()
print(f"{a.config}: primary {s0.kernel_ms:.3f} ms" + (f", bounce {s1.kernel_ms:.3f} ms ({nb} rays)" if bounce else ""))
