"""Per-wave timeline (TT_DIAG_TL build): iteration duration and active lanes over launch time."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch
dev = torch.device("cuda:0")
W, H, far = 1920, 1080, 1000.0
NW = 8192
buf = torch.zeros(NW * 64 * 2, dtype=torch.int32, device=dev)
os.environ["TT_DIAG_TIMES_PTR"] = str(buf.data_ptr())
import tthip
blas = tthip.Blas(tthip.Mesh.sponza()); am = tthip.AssetManager(); am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE)); sc = am.build()
eng = tthip.Engine(0, stream=torch.cuda.current_stream(dev).cuda_stream); eng.upload(sc)
rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
eng.generate(rays, c2w, ip, W, H, 0.3, far, jitter=1, frames=0, max_bounce=1, device=True)
for b in (0, 1):
    n = W * H
    if b == 1:
        n = eng.enqueue_bounce(rays, W * H, 0, far, W, H, device=True)
    for _ in range(3):
        buf.zero_()
        s = eng.trace(rays, n, b, far, W, H, device=True)
    t = buf.cpu().numpy().view(np.uint32).reshape(NW, 64, 2).astype(np.int64)
    used = t[:, 0, 0] > 0
    t = t[used]
    tm = t[:, :, 0]; act = t[:, :, 1] & 0xff; segl = (t[:, :, 1] >> 8) & 0xf; cyc = t[:, :, 1] >> 12
    valid = tm > 0
    t0 = tm[valid].min()
    print(f"bounce {b}: waves {used.sum()} kernel {s.kernel_ms*1e3:.0f}us")
    # per-sample interval: 4 iterations between consecutive samples of one wave
    dt = (tm[:, 1:] - tm[:, :-1]) / 100.0 / 4.0  # us per iteration
    dc = ((cyc[:, 1:] - cyc[:, :-1]) % (1 << 20)) / 4.0  # shader cycles per iteration
    ok = valid[:, 1:] & valid[:, :-1]
    tmid = (tm[:, :-1] - t0) / 100.0
    for lo in range(0, 700, 50):
        m = ok & (tmid >= lo) & (tmid < lo + 50)
        if m.sum() == 0:
            continue
        print(f"  t [{lo:3d},{lo+50:3d}) us: samples {m.sum():6d} us/iter {np.median(dt[m]):.2f} cycles/iter {np.median(dc[m]):.0f} "
              f"GHz {np.median(dc[m] / (dt[m] * 1e3)):.2f} active lanes mean {act[:, :-1][m].mean():.1f} segs_left>0 {np.mean(segl[:, :-1][m] > 0):.2f}")
