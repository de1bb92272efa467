"""Per-ray start/end/iterations (TT_DIAG_RAYS build) for the C2 primary and bounce traces: who
forms the drain (tail) of the persistent kernel."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch
dev = torch.device("cuda:0")
W, H, far = 1920, 1080, 1000.0
buf = torch.zeros(4 * W * H, dtype=torch.int32, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(buf.data_ptr())
import tthip
blas = tthip.Blas(tthip.Mesh.sponza()); am = tthip.AssetManager(); am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE)); sc = am.build()
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream); eng.upload(sc)
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
out = {}
for b in (0, 1):
    n = W * H
    if b == 1:
        n = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
    for _ in range(3):
        buf.zero_()
        s = eng.trace(rays, n, b, far, W, H, device=True)
    t = buf.cpu().numpy().view(np.uint32).reshape(-1, 4)[:n].astype(np.int64)
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, 1] - t0) / 100.0
    it, nv = t[:, 2], t[:, 3]
    dur = en - st
    kend = en.max()
    print(f"bounce {b}: rays {n} kernel {s.kernel_ms*1e3:.0f}us last end {kend:.0f}us last start {st.max():.0f}us")
    print("  iterations p50 %d p90 %d p99 %d p99.9 %d max %d; node visits p50 %d max %d" % (
        np.percentile(it, 50), np.percentile(it, 90), np.percentile(it, 99), np.percentile(it, 99.9), it.max(), np.percentile(nv, 50), nv.max()))
    print("  ray duration us p50 %.1f p90 %.1f p99 %.1f max %.1f; us/iteration median %.2f" % (
        np.percentile(dur, 50), np.percentile(dur, 90), np.percentile(dur, 99), dur.max(), np.median(dur / np.maximum(it, 1))))
    late = np.argsort(en)[-20:]
    print("  20 latest-finishing rays: start/end/iters:", [(round(float(st[i])), round(float(en[i])), int(it[i])) for i in late[-8:]])
    for frac in (0.5, 0.8, 0.9, 0.95, 0.99):
        print(f"   {frac:.2f} of rays started by {np.percentile(st, frac*100):.0f}us, finished by {np.percentile(en, frac*100):.0f}us")
    # rays still in flight when the last ray started, and their remaining durations
    ts = st.max()
    infl = (st <= ts) & (en > ts)
    print(f"  in flight at last start: {infl.sum()} rays; their iters p50 {np.percentile(it[infl],50):.0f} p99 {np.percentile(it[infl],99):.0f} max {it[infl].max()}")
    np.save(os.path.join(REPO, "gpurun_out", f"diag_rays_b{b}.npy"), t.astype(np.uint32))
