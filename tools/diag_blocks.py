"""Wave executions of each block of the closest-hit loop (TT_DIAG_BLOCKS build, run with
TT_HIP_LIB=<that build>) on the C2 bench workload (or C4: argument c4): how often a wave enters the refill, node,
TLAS-leaf, triangle, advance, BLAS-exit, pop, finish and record-write blocks per loop iteration.
Weighted by each block's static VALU count (from the ISA), this says where the loop's VALU goes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

NAMES = ["iteration", "refill", "node_phase", "tlas_leaf", "tri_phase", "advance", "blas_exit", "pop",
         "finish", "record_write"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
sc, view = {"c2": (T.c2_sponza, T.C2_VIEW), "c4": (T.c4_bistro, T.C4_VIEW)}[cfg]
sc = sc()
dev = torch.device("cuda:0")
cnt = torch.zeros(16, dtype=torch.int64, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(cnt.data_ptr())
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
W, H, far = 1920, 1080, 1000.0
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
c2w, ip = view.camera()
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
for b in (0, 1):
    n = W * H
    if b == 1:
        n = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
    torch.cuda.synchronize()
    cnt.zero_()
    eng.trace(rays, n, b, far, W, H, info=info if b == 0 else None, device=True)
    torch.cuda.synchronize()
    c = cnt.cpu().tolist()
    it = max(c[0], 1)
    print(f"bounce {b}: {n} rays, {it} wave-iterations ({it / n:.3f} per ray)")
    print("  per wave-iteration: " + ", ".join(f"{NAMES[k]} {c[k] / it:.3f}" for k in range(1, 10)))
