"""Randomized parity sweep (GPU box): many seeded scenes and cameras beyond the fixed test seeds,
each traced by the engine (closest hit at bounce 0 with _PrimaryTriangleInfo, the diffuse bounce-1
rays, any-hit NEE rays) and re-traced by the CPU oracle; prints one line per case and a summary.
Scenes: single-object soups (500-120k tris, random triangle sizes), two-level instanced scenes
(random props, rigid + uniform-scale instances), and glass / cutout soups for the any-hit tint.
The oracle is the checker only (test infrastructure)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402,F401  (binds the HIP runtime first)

import handbuilt as hb  # noqa: E402
import oracle_ctypes as O  # noqa: E402
import tthip  # noqa: E402
from parity_util import CPU_THREADS, FAR  # noqa: E402
from test_gpu_parity import glass_soup, instanced_scene  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
SEED0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
# "variants": every case also draws the compile-time trace variants of GlobalDefines.cginc:4,11 as
# launch flags (IgnoreGlassMain / IgnoreBackfacing, both, or neither) for its closest-hit traces
MODES = sys.argv[3].split(",") if len(sys.argv) > 3 else []
VARIANTS = "variants" in MODES
# "adaptive": every closest-hit launch runs twice with TT_TRACE_ADAPTIVE_ORDER (the second one dequeues
# in the order the first one's costs give) and the second one's records are compared
ADAPTIVE = "adaptive" in MODES
# "axis": degenerate directions -- every third case looks exactly down an axis (whole rows / columns of
# rays with a zero component), and 3% of every case's primary rays get one or two components replaced by
# +0.0 or -0.0 (inf / NaN slabs in the node test: the C5 bench frame's longest ray is one of these)
AXIS = "axis" in MODES
# "slots": every instanced case is also traced by a frame slot (tt_ctx_share_blas) whose instances were all
# moved (its own _MeshData rewrite + TLAS refit): primary + info, bounce 1 and NEE rays against the oracle on
# the scene as the slot holds it (its TLAS nodes read back, its _MeshData)
SLOTS = "slots" in MODES
# "group": every case is also traced through a multi-GPU group of the C ABI (tt_group_*): 1-5 members sharing
# device 0 (copy gather), a random tile edge and slot count, bounce 1 on; the gathered screen-order records
# against the oracle's jittered frame, and every member's bounce-1 rays and records against the oracle's
# enqueue + trace over that member's own rays (tt_group_tile_pixels order)
GROUP = "group" in MODES
FLAG_SETS = (0, tthip.TT_TRACE_IGNORE_GLASS, tthip.TT_TRACE_IGNORE_BACKFACING,
             tthip.TT_TRACE_IGNORE_GLASS | tthip.TT_TRACE_IGNORE_BACKFACING)
eng = tthip.Engine(0)
bad_total, rays_total = 0, 0


def device_rays(ptr, n):
    """n RayData records copied back from a device pointer the group hands out (torch's HIP runtime)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.zeros(n, tthip.RAY_DTYPE)
    assert hip.hipMemcpy(out.ctypes.data, ptr, 48 * n, 2) == 0  # hipMemcpyDeviceToHost
    return out


def compare(sc, rays, n, bounce, W, H, info=True, flags=0, e=None):
    e = eng if e is None else e
    rg, rc = rays.copy(), rays.copy()
    ig = np.zeros((W * H, 4), np.uint32) if info else None
    ic = np.zeros((W * H, 4), np.uint32) if info else None
    if ADAPTIVE:
        r0 = rays.copy()
        e.trace(r0, n, bounce, FAR, W, H, info=None, flags=flags | tthip.TT_TRACE_ADAPTIVE_ORDER)
        e.trace(rg, n, bounce, FAR, W, H, info=ig, flags=flags | tthip.TT_TRACE_ADAPTIVE_ORDER)
    else:
        e.trace(rg, n, bounce, FAR, W, H, info=ig, flags=flags)
    st, _ = O.trace(sc, rc, n, bounce, FAR, W, H, info=ic, nthreads=CPU_THREADS, flags=flags)
    assert st == 0
    off = W * H if bounce % 2 else 0
    bad = int((rg["hits"][off:off + n] != rc["hits"][off:off + n]).any(1).sum())
    if info:
        bad += int((ig != ic).any(1).sum())
    return bad, rg


def moved(sc, rng):
    """sc's _MeshData and instance boxes with every record but the first moved by a random offset."""
    md = sc.meshdata.copy()
    box = np.ascontiguousarray(sc.meta["mesh_aabbs"], np.float32).copy()
    for i in range(1, len(md)):
        d = rng.normal(0, 1.0, 3)
        w2l = md["W2L"][i].astype(np.float64).reshape(4, 4).T
        sh = np.eye(4)
        sh[:3, 3] = -d
        md["W2L"][i] = tthip.unity_colmajor(w2l @ sh)
        box[i, 0:3] += d.astype(np.float32)
        box[i, 3:6] += d.astype(np.float32)
    return md, box


def shadow_compare(sc, sr, W, H, e=None):
    e = eng if e is None else e
    n = len(sr)
    out = []
    for side in (0, 1):
        r = sr.copy()
        vis = np.zeros((n, 4), np.float32)
        if side == 0:
            e.trace_shadow(r, n, 0, W, H, visibility=vis)
        else:
            assert O.shadow(sc, r, n, 0, W, H, visibility=vis, nthreads=CPU_THREADS)[0] == 0
        out.append((r, vis))
    (rg, vg), (rc, vc) = out
    same_t = np.ascontiguousarray(rg).view(np.uint8).reshape(n, -1) == np.ascontiguousarray(rc).view(np.uint8).reshape(n, -1)
    same_v = (vg.view(np.uint32) == vc.view(np.uint32)) | (np.isnan(vg) & np.isnan(vc))
    return int((~same_t.all(1) | ~same_v.all(1)).sum())


t0 = time.time()
for k in range(N):
    seed = SEED0 + k
    rng = np.random.default_rng(seed)
    flags = FLAG_SETS[int(rng.integers(0, 4))] if VARIANTS else 0
    kind = ("soup", "instanced", "glass")[k % 3]
    if kind == "soup":
        sc = tthip.single_object_scene(tthip.Mesh.soup(seed, int(rng.integers(500, 120000)), 1.0,
                                                       float(rng.uniform(0.01, 0.3))))
        pos = rng.uniform(-2.5, 2.5, 3)
        look = -pos + rng.normal(0, 0.3, 3)
    elif kind == "instanced":
        sc = instanced_scene(seed, n_props=int(rng.integers(3, 12)), n_inst=int(rng.integers(20, 300)))
        pos = np.array([rng.uniform(-30, 30), rng.uniform(2, 12), rng.uniform(35, 55)])
        look = np.array([0.0, -0.2, -1.0]) + rng.normal(0, 0.1, 3)
    else:
        sc = glass_soup(seed)
        pos = np.array([0.3, 0.2, 3.0]) + rng.normal(0, 0.3, 3)
        look = np.array([0.0, 0.0, -1.0]) + rng.normal(0, 0.1, 3)
    W, H = int(rng.integers(40, 256)), int(rng.integers(24, 160))
    if AXIS and k % 3 == 1:
        look = np.zeros(3)
        look[int(rng.integers(0, 3))] = float(rng.choice([-1.0, 1.0]))
        if abs(look[1]) == 1.0:  # not parallel to the camera's up vector
            look = np.array([0.0, 0.0, -1.0])
    c2w, ip = tthip.unity_camera(pos, look, (0, 1, 0), float(rng.uniform(30, 90)), W, H, 0.05, FAR)
    rays = O.generate(c2w, ip, W, H, 0.05, FAR)
    if AXIS:
        pick = np.nonzero(rng.random(W * H) < 0.03)[0]
        for i in pick:
            for ax in rng.choice(3, size=int(rng.integers(1, 3)), replace=False):
                rays["direction"][i, ax] = np.float32(-0.0) if rng.random() < 0.5 else np.float32(0.0)
    eng.upload(sc)
    b0, rg = compare(sc, rays, W * H, 0, W, H, flags=flags)
    # bounce 1 from the GPU's primary hits (identical to the oracle's when b0 == 0)
    r1 = rg.copy()
    nb = eng.enqueue_bounce(r1, W * H, 0, FAR, W, H, frames=k, max_bounce=2)
    b1, _ = compare(sc, r1, nb, 1, W, H, info=False, flags=flags) if nb else (0, None)
    sr = hb.nee_rays_from_hits(rg, W * H, tuple(rng.uniform(-2, 2, 3) + [0, 3, 0]), seed)
    bs = shadow_compare(sc, sr, W, H) if len(sr) else 0
    n_rays = W * H + nb + len(sr)
    bsl = 0
    if SLOTS and kind == "instanced":
        slot = tthip.Engine(0)
        try:
            slot.share_blas(eng, sc.tlas_nodes)
            md, box = moved(sc, rng)
            slot.update_meshdata(0, md)
            slot.tlas_refit(sc.tlas_nodes, box)
            ss = tthip.Scene(slot.scene_nodes(0, len(sc.nodes)), sc.tris, sc.tlas, md, sc.materials,
                             tlas_nodes=sc.tlas_nodes)
            s0, sg = compare(ss, rays, W * H, 0, W, H, flags=flags, e=slot)
            s1r = sg.copy()
            snb = slot.enqueue_bounce(s1r, W * H, 0, FAR, W, H, frames=k, max_bounce=2)
            s1, _ = compare(ss, s1r, snb, 1, W, H, info=False, flags=flags, e=slot) if snb else (0, None)
            ssr = hb.nee_rays_from_hits(sg, W * H, tuple(rng.uniform(-2, 2, 3) + [0, 3, 0]), seed)
            ssh = shadow_compare(ss, ssr, W, H, e=slot) if len(ssr) else 0
            bsl = s0 + s1 + ssh
            n_rays += W * H + snb + len(ssr)
        finally:
            slot.close()
    bgr = 0
    if GROUP:
        members = int(rng.integers(1, 6))
        tile = int(rng.choice([8, 16, 32, 64]))
        g = tthip.Group(W, H, devices=[0] * members, tile=tile, slots=int(rng.integers(1, 4)), bounce=True, copy=True)
        try:
            g.upload(sc)
            hits = torch.full((W * H, 4), -1, dtype=torch.int32, device="cuda:0")
            g.trace_frame(hits, c2w, ip, 0.05, FAR, jitter=1, frames=k, max_bounce=2)
            full = O.generate(c2w, ip, W, H, 0.05, FAR, jitter=1, frames=k, max_bounce=2)
            assert O.trace(sc, full, W * H, 0, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
            bgr += int((hits.cpu().numpy().view(np.uint32) != full["hits"][:W * H]).any(1).sum())
            n_rays += W * H
            for m in range(members):
                n, nbm, ptr = g.frame_rays(m)
                pix = tthip.group_tile_pixels(W, H, members, m, tile).astype(np.int64)
                mr = np.zeros(W * H + n, tthip.RAY_DTYPE)
                mr[:n] = full[pix]
                nb_ref = O.enqueue_bounce(sc, mr, n, 0, FAR, W, H, frames=k, max_bounce=2)
                if nb_ref:
                    assert O.trace(sc, mr, nb_ref, 1, FAR, W, H, nthreads=CPU_THREADS)[0] == 0
                got = device_rays(ptr, W * H + n)
                if nbm != nb_ref:
                    bgr += max(nbm, nb_ref)
                else:
                    same = (np.ascontiguousarray(got[W * H:W * H + nbm]).view(np.uint8).reshape(nbm, 48) ==
                            np.ascontiguousarray(mr[W * H:W * H + nbm]).view(np.uint8).reshape(nbm, 48)).all(1)
                    bgr += int((~same).sum())
                n_rays += nbm
        finally:
            g.close()
    rays_total += n_rays
    bad_total += b0 + b1 + bs + bsl + bgr
    print(f"case {k:3d} {kind:9s} seed {seed} flags {flags:#04x} tris {len(sc.tris):6d} {W}x{H}: primary+info mismatches {b0}, "
          f"bounce-1 ({nb} rays) {b1}, shadow ({len(sr)} rays) {bs}" + (f", frame slot {bsl}" if SLOTS and kind == "instanced"
                                                                          else "")
          + (f", group {bgr}" if GROUP else ""), flush=True)
print(f"SUMMARY: {N} cases, {rays_total} rays traced on the GPU and the oracle, {bad_total} mismatching records, "
      f"{time.time() - t0:.0f} s", flush=True)
sys.exit(1 if bad_total else 0)
