"""Quick end-to-end GPU check: parity vs the oracle on Cornell + Sponza-shaped scenes, and timing."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_ctypes as O  # noqa
import tthip  # noqa

print("devices", tthip.device_count(), flush=True)
eng = tthip.Engine(0)

def check(name, sc, W, H, rays, n, bounce, far=1000.0, info=True):
    r_gpu = rays.copy(); r_cpu = rays.copy()
    inf_g = np.zeros((W * H, 4), np.uint32) if info else None
    inf_c = np.zeros((W * H, 4), np.uint32) if info else None
    eng.upload(sc)
    t0 = time.time(); s = eng.trace(r_gpu, n, bounce, far, W, H, info=inf_g, stats=True); t1 = time.time()
    st, cnt = O.trace(sc, r_cpu, n, bounce, far, W, H, info=inf_c, counts=True, nthreads=16)
    t2 = time.time()
    off = W * H if bounce % 2 else 0
    hg, hc = r_gpu["hits"][off:off + n], r_cpu["hits"][off:off + n]
    mism = np.nonzero((hg != hc).any(1))[0]
    print(f"[{name}] n={n} gpu {t1-t0:.3f}s kernel {s.kernel_ms:.3f}ms cpu {t2-t1:.3f}s mismatches={len(mism)} "
          f"gpu nodes {s.node_visits} cpu nodes {cnt['node_visits'].sum()} gpu tris {s.tri_tests} cpu tris {cnt['tri_tests'].sum()} "
          f"rays {s.rays} reps_exh {s.reps_exhausted}", flush=True)
    if len(mism):
        print("  first mismatches", mism[:5], hg[mism[:5]], hc[mism[:5]])
    if info:
        print("  info mismatches", int((inf_g != inf_c).any(1).sum()))
    return r_gpu

# Cornell
W = H = 256
sc = tthip.single_object_scene(tthip.Mesh.cornell())
c2w, ip = tthip.unity_camera((0, 0, 3.4), (0, 0, -1), (0, 1, 0), 40, W, H, 0.3, 1000)
rays = O.generate(c2w, ip, W, H, 0.3, 1000.0)
check("cornell", sc, W, H, rays, W * H, 0)

# soup
sc2 = tthip.single_object_scene(tthip.Mesh.soup(7, 20000, 1.0, 0.05))
c2w, ip = tthip.unity_camera((0, 0, 3.0), (0, 0, -1), (0, 1, 0), 50, W, H, 0.3, 1000)
rays = O.generate(c2w, ip, W, H, 0.3, 1000.0)
check("soup20k", sc2, W, H, rays, W * H, 0)

# Sponza
W, H = 1920, 1080
t0 = time.time()
blas = tthip.Blas(tthip.Mesh.sponza())
am = tthip.AssetManager(); am.add_parent(blas, None, np.zeros(8, tthip.MAT_DTYPE)); sc3 = am.build()
print("sponza build", time.time() - t0, flush=True)
c2w, ip = tthip.unity_camera((-10, 2, 0), (1, 0, 0), (0, 1, 0), 60, W, H, 0.3, 1000)
rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
eng.upload(sc3)
eng.generate(rays, c2w, ip, W, H, 0.3, 1000.0)
rays_o = O.generate(c2w, ip, W, H, 0.3, 1000.0)
print("raygen bitwise equal", bool((rays.view(np.uint32) == rays_o.view(np.uint32)).all()),
      "max dir diff", float(np.abs(rays["direction"] - rays_o["direction"]).max()), flush=True)
r1 = check("sponza-primary", sc3, W, H, rays, W * H, 0)
nb = eng.enqueue_bounce(r1, W * H, 0, 1000.0, W, H)
print("bounce rays", nb, flush=True)
check("sponza-bounce1", sc3, W, H, r1, nb, 1, info=False)

# timing with device pointers
import torch
dev = torch.device("cuda:0")
rt = torch.from_numpy(r1.view(np.uint8)).to(dev)
ptr = rt.data_ptr()
for it in range(3):
    eng.trace(ptr, W * H, 0, 1000.0, W, H, device=True)
ts = []
for it in range(10):
    s = eng.trace(ptr, W * H, 0, 1000.0, W, H, device=True)
    ts.append(s.kernel_ms)
print("primary kernel ms", np.median(ts), "Mrays/s", W * H / np.median(ts) / 1e3)
ts = []
for it in range(10):
    s = eng.trace(ptr, nb, 1, 1000.0, W, H, device=True)
    ts.append(s.kernel_ms)
print("bounce kernel ms", np.median(ts), "Mrays/s", nb / np.median(ts) / 1e3)
