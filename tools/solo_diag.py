#!/usr/bin/env python3
"""Cycle breakdown of the solo phase (tt_solo.h) on the lone Reps-exhausting C2 ray and on the
screen column x = 960 (run with TT_HIP_LIB=.../variants/libtruetrace_hip_diagsolo.so, a
-DTT_DIAG_SOLO build): s_memtime cycles in the node step, the triangle pass and the advance."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

dev = torch.device("cuda:0")
buf = torch.zeros(16, dtype=torch.int64, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(buf.data_ptr())
import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

eng = tthip.Engine(0)
eng.upload(T.c2_sponza())
W, H = 1920, 1080
WH = W * H
c2w, ip = T.C2_VIEW.camera(W, H)
full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
eng.generate(full, c2w, ip, W, H, T.NEAR, T.FAR, jitter=0, frames=0, max_bounce=1, device=True)
for name, idx in (("lone_reps_ray", [540 * W + 960]), ("col960_ray_500", [500 * W + 960])):
    sel = torch.tensor(idx, device=dev)
    rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
    rays[: len(idx) * 48] = full.view(WH, 48)[sel].contiguous().view(-1)
    for k in range(3):
        buf.zero_()
        s = eng.trace(rays.clone(), len(idx), 0, T.FAR, W, H, device=True, stats=(k == 2))
    d = buf.cpu().numpy()
    it = max(int(d[3]), 1)
    print(f"{name}: kernel {s.kernel_ms * 1e3:.0f} us, iterations {d[3]}, node steps {d[4]}, tri passes {d[5]}, "
          f"rays in solo {d[6]}; cycles/iteration: node {d[0] / it:.0f} tri {d[1] / it:.0f} adv {d[2] / it:.0f}; "
          f"per tri pass {d[1] / max(int(d[5]), 1):.0f}; node-data wait {d[7] / max(int(d[4]), 1):.0f}/step, "
          f"tri-data wait {d[8] / max(int(d[5]), 1):.0f}/pass; nodes {s.node_visits} tris {s.tri_tests}")
