"""Times every kernel variant in lib/variants/ on the C2 workload (RV_CFG=c4 / c5: that config) (each in a fresh process) and
checks a strided sample of its hits against the oracle."""
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.path.join(os.environ["REPO"], "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
import torch, tthip, oracle_ctypes as O
cfg = os.environ.get("RV_CFG", "c2")
if cfg == "c2":
    W, H, far = 1920, 1080, 1000.0
    blas = tthip.Blas(tthip.Mesh.sponza()); am = tthip.AssetManager(); am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE)); sc = am.build()
    cam = ((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), 60.0)
else:  # another BASELINE config from ttconfigs (c4: Bistro-shaped two-level, c5: San-Miguel-shaped)
    import ttconfigs as T
    sc = {"c4": T.c4_bistro, "c5": T.c5_san_miguel}[cfg]()
    v = {"c4": T.C4_VIEW, "c5": T.C5_VIEW}[cfg]
    W, H, far = v.width, v.height, T.FAR
    cam = (v.position, v.forward, v.vfov)
dev = torch.device("cuda:0")
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream); eng.upload(sc)
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera(cam[0], cam[1], (0.0, 1.0, 0.0), cam[2], W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
eng.trace(rays, W * H, 0, far, W, H, info=info, device=True)
nb = eng.enqueue_bounce(rays, W * H, 0, far, W, H, frames=0, max_bounce=1, device=True)
colors = np.zeros(W * H, tthip.COL_DTYPE); colors["Data"][:, 3] = 1.0  # as bench.py: info written at bounce 1
colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
eng.trace(rays, nb, 1, far, W, H, info=info, colors=colors_t, device=True)
host = rays.cpu().numpy().view(tthip.RAY_DTYPE).copy()
ok = True
for off, n, b in ((0, W * H, 0), (W * H, nb, 1)):
    idx = off + np.arange(0, n, 97)
    s = np.zeros(2 * len(idx), tthip.RAY_DTYPE); s[:len(idx)] = host[idx]
    st, _ = O.trace(sc, s, len(idx), 0, far, len(idx), 1, nthreads=16)
    ok &= bool(np.array_equal(s["hits"][:len(idx)], host["hits"][idx]))
for _ in range(3):
    eng.trace(rays, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
    eng.trace(rays, nb, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)
eng.timing_reset()
for _ in range(10):
    eng.trace(rays, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
    eng.trace(rays, nb, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)
ms = eng.timing_read()
p, b = float(np.median(ms[0::2])), float(np.median(ms[1::2]))
rec = {"ok": ok, "primary_ms": round(p, 4), "bounce_ms": round(b, 4), "grays": round((W * H + nb) / (p + b) / 1e6, 3)}
if os.environ.get("RV_RECUR") == "1":  # + the unjittered (UseReCur) primary launch: the long-ray tail
    rr = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
    eng.generate(rr, c2w, ip, W, H, 0.3, far, jitter=0, frames=0, max_bounce=1, device=True)
    for _ in range(2):
        eng.trace(rr, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
    eng.timing_reset()
    for _ in range(5):
        eng.trace(rr, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
    rec["recur_primary_ms"] = round(float(np.median(eng.timing_read())), 4)
print(json.dumps(rec))
'''
libs = sorted(glob.glob(os.path.join(REPO, "truetrace-unity-pathtracer_amd", "lib", "variants", "*.so")))
names = [os.path.basename(l)[len("libtruetrace_hip_"):-3] for l in libs]
order = sys.argv[1:] or names  # a name may repeat (re-measure for noise)
for spec in order:  # "name" or "name@B": B = TT_BLOCKS_PER_CU cap (256-thread blocks per CU)
    name, _, bpc = spec.partition("@")
    lib = (os.path.join(REPO, "truetrace-unity-pathtracer_amd", "lib", "libtruetrace_hip.so") if name == "product"
           else libs[names.index(name)])
    env = dict(os.environ, TT_HIP_LIB=lib, REPO=REPO)
    if bpc:
        env["TT_BLOCKS_PER_CU"] = bpc
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
    print(f"{spec:10s} {line}", flush=True)
