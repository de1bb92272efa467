"""Visits per node (TT_DIAG_NODEHIST build) on the C2 bench workload: how concentrated node traffic
is (the case for an LDS cache of the hottest nodes) and how visits spread over BVH depth."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

dev = torch.device("cuda:0")
sc = T.c2_sponza()
N = len(sc.nodes)
hist = torch.zeros(N + 64, dtype=torch.int32, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(hist.data_ptr())
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
W, H, far = 1920, 1080, 1000.0
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = T.C2_VIEW.camera()
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
# depth of every node (BFS from node 0 / the BLAS root through base_child + internal ranks)
depth = np.full(N, -1)
root = int(sc.meshdata["mesh_data_bvh_offsets"][0] & 0x7FFFFFFF)
no = int(sc.meshdata["NodeOffset"][0])
depth[0] = 0
q = [(root, 1, no)]
while q:
    n, d, off = q.pop()
    depth[n] = d
    meta = [(int(sc.nodes["meta"][n][k >> 2]) >> (8 * (k & 3))) & 0xFF for k in range(8)]
    for m in meta:
        if (m & 0x1F) >= 24:
            q.append((int(sc.nodes["base_child"][n]) + (m & 0x1F) - 24 + off, d + 1, off))
for b in (0, 1):
    hist.zero_()
    if b == 0:
        eng.trace(rays, W * H, 0, far, W, H, device=True)
    else:
        nb = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
        hist.zero_()
        eng.trace(rays, nb, 1, far, W, H, device=True)
    torch.cuda.synchronize()
    h = hist.cpu().numpy()[:N].astype(np.int64)
    tot = h.sum()
    srt = np.sort(h)[::-1]
    print(f"bounce {b}: node visits {tot}  nodes visited {int((h > 0).sum())} of {N}")
    print("  share of visits to the hottest K nodes:",
          {K: round(float(srt[:K].sum() / tot), 3) for K in (16, 64, 128, 256, 512, 1024, 2048)})
    print("  share by depth:", {int(d): round(float(h[depth == d].sum() / tot), 3) for d in range(0, 8)})
