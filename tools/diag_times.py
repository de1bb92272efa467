"""Per-wave start/end timestamps (TT_DIAG_TIMES build) for the C2 primary trace: shows the
load-balance tail of the persistent kernel. --ranks N traces rank 0's 64x64 tiles of an N-GPU
tile-sharded frame instead (the per-rank launch under strong scaling)."""
import os, sys
import numpy as np
RANKS = int(sys.argv[sys.argv.index("--ranks") + 1]) if "--ranks" in sys.argv else 1
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch
dev = torch.device("cuda:0")
buf = torch.zeros(4 * 8192, dtype=torch.int64, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(buf.data_ptr())
import tthip
W, H, far = 1920, 1080, 1000.0
blas = tthip.Blas(tthip.Mesh.sponza()); am = tthip.AssetManager(); am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE)); sc = am.build()
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream); eng.upload(sc)
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
n0 = W * H
if RANKS > 1:
    import ttdist
    pix = torch.from_numpy(ttdist.tile_pixels(W, H, RANKS, 0)).to(dev)
    full = rays[: W * H * 48].clone()
    n0 = int(pix.shape[0])
    rays.view(2 * W * H, 48)[:n0] = full.view(W * H, 48)[pix]
    del full
for b in (0, 1):
    if b == 1:
        nb = eng.enqueue_bounce(rays, n0, 0, far, W, H, device=True)
    for _ in range(3):
        s = eng.trace(rays, n0 if b == 0 else nb, b, far, W, H, device=True)
    t = buf.cpu().numpy().reshape(-1, 4)
    used = t[:, 1] > 0
    t = t[used]
    st, en, n, cyc = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    t0 = st.min()
    span = (en.max() - t0) / 100.0  # memrealtime 100 MHz -> us
    life = (en - st) / 100.0
    print(f"bounce {b}: waves {used.sum()} kernel {s.kernel_ms*1e3:.0f}us span {span:.0f}us start spread {(st.max()-t0)/100:.1f}us "
          f"wave life mean {life.mean():.0f} min {life.min():.0f} p10 {np.percentile(life,10):.0f} p50 {np.percentile(life,50):.0f} p90 {np.percentile(life,90):.0f} max {life.max():.0f}us; "
          f"rays/wave mean {n.mean():.0f} min {n.min()} max {n.max()}")
    wide = cyc > 0  # slot 3: memrealtime at entry into the cooperative drain phase (tt_wide.h)
    if wide.any():
        we = (cyc[wide] - t0) / 100.0
        dur = (en[wide] - cyc[wide]) / 100.0
        print(f"   drain phase: {wide.sum()} waves; entry percentiles", [round(float(np.percentile(we, q))) for q in (1, 10, 50, 90, 99)],
              "us; time in drain p50/p90/max", [round(float(np.percentile(dur, q))) for q in (50, 90, 100)], "us")
    end_rel = (en - t0) / 100.0
    print("   end-time percentiles", [round(float(np.percentile(end_rel, q))) for q in (1, 10, 25, 50, 75, 90, 99, 100)])
    # waves alive / in the drain phase over time (10 buckets of the span)
    grid = np.linspace(0, span, 11)[1:]
    alive = [int(((st - t0) / 100.0 <= g).sum() - ((en - t0) / 100.0 <= g).sum()) for g in grid]
    draining = [int((wide & ((cyc - t0) / 100.0 <= g) & ((en - t0) / 100.0 > g)).sum()) for g in grid]
    print("   waves alive at 10%..100% of span", alive, "of which in the drain phase", draining)
