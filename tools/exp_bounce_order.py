"""Experiment: how much does the ORDER of the bounce-1 rays in GlobalRays change the trace time?
The reference appends survivors with a global atomic (RayTracingShader.compute:498-506), so the
order is not semantic (every RayData carries its PixelIndex). Orders timed on the C2 bench
workload: as enqueued (pixel/tile order), grouped by direction octant, octant + Morton code of the
origin, octant + Morton of origin and direction, and a random shuffle (coherence lower bound).
Each order's hit records are un-permuted and compared with the enqueued order's (must be equal)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402

import tthip  # noqa: E402


def morton3(x, y, z, bits=10):
    def spread(v):
        v = v.astype(np.uint64) & np.uint64(0x3FF)
        v = (v | (v << np.uint64(16))) & np.uint64(0x030000FF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x0300F00F)
        v = (v | (v << np.uint64(4))) & np.uint64(0x030C30C3)
        v = (v | (v << np.uint64(2))) & np.uint64(0x09249249)
        return v
    return spread(x) | (spread(y) << np.uint64(1)) | (spread(z) << np.uint64(2))


def quant(a, lo, hi, bits=10):
    return np.clip(((a - lo) / max(hi - lo, 1e-9) * ((1 << bits) - 1)).astype(np.int64), 0, (1 << bits) - 1)


W, H, far = 1920, 1080, 1000.0
WH = W * H
dev = torch.device("cuda:0")
blas = tthip.Blas(tthip.Mesh.sponza())
am = tthip.AssetManager()
am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
sc = am.build()
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream)
eng.upload(sc)
rays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
eng.trace(rays, WH, 0, far, W, H, device=True)
nb = eng.enqueue_bounce(rays, WH, 0, far, W, H, frames=0, max_bounce=1, device=True)
torch.cuda.synchronize()
host = rays.cpu().numpy().view(tthip.RAY_DTYPE)[WH:WH + nb].copy()
f = host.view(np.float32).reshape(nb, 12)
ox, oy, oz, dx, dy, dz = f[:, 0], f[:, 1], f[:, 2], f[:, 4], f[:, 5], f[:, 6]
octant = ((dx < 0).astype(np.int64) << 2) | ((dy < 0).astype(np.int64) << 1) | (dz < 0).astype(np.int64)
mo = morton3(quant(ox, ox.min(), ox.max()), quant(oy, oy.min(), oy.max()), quant(oz, oz.min(), oz.max())).astype(np.int64)
md = morton3(quant(dx, -1, 1, 4), quant(dy, -1, 1, 4), quant(dz, -1, 1, 4)).astype(np.int64)
rng = np.random.default_rng(1)
orders = {
    "enqueued": np.arange(nb),
    "octant": np.argsort(octant, kind="stable"),
    "octant_morton_o": np.lexsort((mo, octant)),
    "morton_o": np.argsort(mo, kind="stable"),
    "morton_o_dir": np.lexsort((md, mo >> 9)),
    "shuffle": rng.permutation(nb),
}
ref_hits = None
res = {}
buf = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
for name, perm in orders.items():
    arr = np.zeros(2 * WH, tthip.RAY_DTYPE)
    arr[WH:WH + nb] = host[perm]
    buf.copy_(torch.from_numpy(arr.view(np.uint8)))
    for _ in range(3):
        eng.trace(buf, nb, 1, far, W, H, device=True, asynchronous=True)
    torch.cuda.synchronize()
    buf.copy_(torch.from_numpy(arr.view(np.uint8)))
    eng.timing_reset()
    for _ in range(10):
        eng.trace(buf, nb, 1, far, W, H, device=True, asynchronous=True)
    torch.cuda.synchronize()
    ms = float(np.median(eng.timing_read()))
    out = buf.cpu().numpy().view(tthip.RAY_DTYPE)[WH:WH + nb]
    hits = np.empty_like(out["hits"])
    hits[perm] = out["hits"]
    if ref_hits is None:
        ref_hits = hits
    res[name] = {"ms": round(ms, 4), "mrays_s": round(nb / ms / 1e3, 1), "same_hits": bool(np.array_equal(hits, ref_hits))}
    print(name, json.dumps(res[name]), flush=True)
