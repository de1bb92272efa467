"""SIMD efficiency of the closest-hit kernel on the C2 bench workload (TT_TRACE_STATS counters):
mean active lanes per loop iteration, and lanes busy in the node phase / triangle phase."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
sc, view = {"c2": (T.c2_sponza, T.C2_VIEW), "c4": (T.c4_bistro, T.C4_VIEW)}[cfg]
sc = sc()
dev = torch.device("cuda:0")
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
W, H, far = 1920, 1080, 1000.0
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = view.camera()
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
for b in (0, 1):
    n = W * H
    if b == 1:
        n = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
    s = eng.trace(rays, n, b, far, W, H, device=True, stats=True)
    d = eng.diagnostics()
    it = max(d["iterations"], 1)
    print(f"bounce {b}: {n} rays, wave-iterations {it}, node visits {s.node_visits}, tri tests {s.tri_tests}")
    print(f"  active lanes / iteration {d['active_lanes'] / it:.1f} of 64")
    print(f"  node phase: {d['node_iters'] / it:.1%} of iterations run it, {d['node_lanes'] / max(d['node_iters'], 1):.1f} lanes each")
    print(f"  tri phase:  {d['tri_iters'] / it:.1%} of iterations run it, {d['tri_lanes'] / max(d['tri_iters'], 1):.1f} lanes each")
    print(f"  node uniformity: {d['lead_same_lanes'] / max(d['node_lanes'], 1):.1%} of node visits share the first lane's node, "
          f"{d['uniform_node_iters'] / max(d['node_iters'], 1):.1%} of node phases are wave-uniform")
    print(f"  node visits per wave-iteration {s.node_visits / it:.1f}, tri tests per wave-iteration {s.tri_tests / it:.1f}")
    print(f"  per ray: nodes {s.node_visits / n:.2f}, tris {s.tri_tests / n:.2f}, BLAS entries {s.blas_entries / n:.2f}, "
          f"kernel (stats build) {s.kernel_ms:.3f} ms")
