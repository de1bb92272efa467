#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric: Mrays/s for primary + 1-bounce closest-hit CWBVH8 traversal
on a Sponza-shaped scene at 1920x1080, with the trace kernel's roofline fraction and a CPU
baseline (the scalar oracle on the host cores) on the same workload.

One "step" = one pass of the hot path over one batch: the kernel_trace replacement run on the
2,073,600 primary rays (bounce 0, with _PrimaryTriangleInfo) and then on the compacted bounce-1
rays (bounce 1, _PrimaryTriangleInfo written where GlobalColors.Data.w == 1), both already
resident in HBM in the reference's 2*W*H ping-pong RayData buffer. Ray generation and the
bounce enqueue run once during setup (they are the caller's kernels, not the trace).

Multi-GPU (``bench.py --gpus N``, self-launched, or under ``torchrun --nproc-per-node N``): one process
per GPU, scene replicated per GPU. Default layout ``--shard tiles`` (strong scaling, the north star's
layout): ONE 1080p frame's 64x64 screen tiles are dealt to the ranks -- round-robin
(``--deal rr``), or longest-processing-time first by a previous frame's tile costs (``--deal lpt``) -- each
rank traces its tiles' primary rays and their bounce-1 rays (1 part x 6 frame slots per rank, every slot
its own jittered sample), and the frame's primary hit records go to rank 0 in ONE RCCL gather over xGMI
-- inside the timed step (on a second stream, overlapped with the bounce-1 trace). ``value`` = all
ranks' rays / the slowest rank's time; the efficiency against the N = 1 frame is in
``config.aux_strong_tiles``. Beside it: ``config.aux_spp_weak`` (weak scaling: an N-sample frame's
(sample, tile) units round-robin, a frame's worth per rank, same gather; the headline with ``--shard
spp``) and, with ``--shard sample``, every rank tracing its own full-frame sample with no collective.

N = 1: the whole frame as one launch per bounce with 3 frames in flight, every frame slot its own jittered
sample; after the timed steps every slot's records (both bounces, both _PrimaryTriangleInfo forms) are
compared with the oracle traced from the same pre-state (``oracle_check``, ``oracle_identical``).

Streams: torch and the engine share ONE stream (a torch.cuda.Stream made current before any
allocation and passed to tt_ctx_create), so every torch copy / collective and every engine launch
is ordered, and every per-launch time comes from HIP events on that stream (the engine's own
timing ring, tt_timing_read). Only one context of a frame layout records them (tt_ctx_set_timing: the
markers cost ~5% of a strong-scaled rank's frame), and at N > 1 none inside the timed region: the launch
times then come from K more steps right after it.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))

METRIC = "Mrays/sec (primary+1-bounce) on Sponza CWBVH at 1080p; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


# frame slots of the N = 1 headline: the whole 1080p frame, one launch per bounce, 3 frames in flight
# (profiles/r04/ab/r04k_* / r04l_*: 1 part x 3 slots 6,259-6,273 Mrays/s vs 2 parts x 1 slot 5,538-5,550)
N1_SLOTS = 3


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def alg_bytes(stats, bounce: int, info_written: int) -> float:
    """Algorithmic bytes of one trace launch:
    B_ray = 48 (RayData) + 16 (hit) + 16*[info written] + 80*N_node + 36*N_tri + 8*N_accept + 68*N_blas."""
    return (48.0 * stats.rays + 16.0 * stats.rays + 16.0 * info_written + 80.0 * stats.node_visits
            + 36.0 * stats.tri_tests + 8.0 * stats.accepts + 68.0 * stats.blas_entries)


def nee_rays(torch, rays, n, far, light):
    """ShadowRayData (48 B) toward `light` from the hit points of the first n RayData records in the
    device buffer `rays` (uint8): origin backed off 1e-3 along the incoming ray, t = distance,
    illumination 1. Built on the GPU with torch (setup, not timed)."""
    r = rays[: n * 48].view(torch.float32).view(n, 12)
    t = r[:, 10]
    hit = t < far
    o, d = r[hit, 0:3], r[hit, 4:7]
    p = o + d * t[hit, None] - d * 1e-3
    to = torch.tensor(light, dtype=torch.float32, device=rays.device)[None, :] - p
    dist = torch.sqrt((to * to).sum(1))
    sr = torch.zeros((p.shape[0], 12), dtype=torch.float32, device=rays.device)
    sr[:, 0:3] = p
    sr[:, 4:7] = to / dist[:, None]
    sr[:, 7] = dist
    sr[:, 8:11] = 1.0
    sri = sr.view(torch.int32)
    sri[:, 11] = rays[: n * 48].view(torch.int32).view(n, 12)[hit, 3]  # PixelIndex, integer copy
    return sr.contiguous().view(torch.uint8).view(-1)


TIMING_RING = 256  # the engine's HIP-event ring (tt_api.hip TT_RING): tt_timing_read returns the last 256


def ring_tail(eng, per_step, steps):
    """The engine ring's per-call times (ms) of the last min(steps, 256 // per_step) steps, shape
    (rows, per_step): with more calls than the ring holds, the oldest are overwritten, so per-launch
    statistics cover the last rows steps (the wall-clock `value` always covers all of them)."""
    rows = min(steps, TIMING_RING // per_step)
    ms = np.asarray(eng.timing_read(), np.float64)
    assert len(ms) == rows * per_step, (len(ms), rows, per_step)
    return ms.reshape(rows, per_step)


def timed_launches(eng, launches, warmup, steps):
    """Runs the list of launch closures warmup + steps times; returns per-launch HIP-event times
    (ms) as an array of shape (rows, len(launches)) over the last rows <= steps repetitions."""
    import torch

    for _ in range(warmup):
        for f in launches:
            f()
    torch.cuda.synchronize()
    eng.timing_reset()
    for _ in range(steps):
        for f in launches:
            f()
    torch.cuda.synchronize()
    return ring_tail(eng, len(launches), steps)


def aux_configs(torch, tthip, eng, dev, args, which):
    """The other BASELINE.json configs, each traced by the same engine with
    inputs resident in HBM and timed per launch with HIP events (not the metric):
      c3  C2 geometry, primary + 3 diffuse bounces (each bounce's compacted rays kept in their own
          buffer so every repetition traces identical rays)
      c4  Bistro-shaped two-level instancing, 1920x1080 primary + bounce 1
      refit  per-frame GPU TLAS refit (C4 instances) and BLAS refit (C2 mesh as a deforming mesh)
      c5  San-Miguel-shaped 10M tris, 3840x2160 primary (single GPU; 8 GPUs shard it by tiles)"""
    import ttconfigs as T

    far = T.FAR
    out = {}

    def pack(name, n_rays_per_launch, ms, extra):
        mean = ms.mean(0)
        rec = {"rays": [int(n) for n in n_rays_per_launch], "trace_ms": [round(float(m), 4) for m in mean],
               "mrays_s": round(float(sum(n_rays_per_launch)) / float(mean.sum()) / 1e3, 1)}
        rec.update(extra)
        out[name] = rec
        log(f"aux {name}: {rec}")

    def rays_with_bounces(view, W, H, nb_max, frames):
        WH = W * H
        c2w, ip = view.camera(W, H)
        base = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(base, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=frames, max_bounce=max(nb_max, 1),
                     device=True)
        bufs, counts = [base.clone()], [WH]
        cur = base
        for b in range(nb_max):
            eng.trace(cur, counts[-1], b, far, W, H, device=True)
            n = eng.enqueue_bounce(cur, counts[-1], b, far, W, H, frames=frames, max_bounce=max(nb_max, 1),
                                   device=True)
            bufs.append(cur.clone())
            counts.append(n)
        torch.cuda.synchronize(dev)
        return bufs, counts

    def parts_layout(sc, view, W, H, nb, info, colors_t, P=2, adaptive=False):
        """The same frame as P tile-interleaved parts, each with its own engine context on its own
        stream and its own chain of bounce launches (bench.py's metric layout): wall
        ms per frame over all launches of all parts. adaptive: TT_TRACE_ADAPTIVE_ORDER on the primary launches,
        the frames alternating between two jittered samples (frames_accumulated 0 / 1), so each launch's
        order comes from the previous frame's costs, never from its own rays."""
        import ttdist

        WH = W * H
        c2w, ip = view.camera(W, H)
        n_frames = 2 if adaptive else 1
        flags = tthip.TT_TRACE_ADAPTIVE_ORDER if adaptive else 0
        extra_engs, streams = [], []
        try:
            for k in range(P - 1):
                streams.append(tthip.dedicated_stream(torch, dev, k))  # a HW queue of its own (ttlayout docstring)
                e1 = tthip.Engine(dev.index, stream=streams[-1].cuda_stream)
                extra_engs.append(e1)
                e1.share_scene(eng)  # one scene copy for all parts (tt_ctx_share_scene)
                e1.set_timing(False)  # (wall clock; no per-launch markers, tt_ctx_set_timing)
            chains = [[] for _ in range(n_frames)]  # chains[f]: per part (engine, bufs, counts)
            base = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
            for f in range(n_frames):
                eng.generate(base, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=f, max_bounce=max(nb, 1),
                             device=True)
                for e, pix_np in zip([eng] + extra_engs, ttdist.part_pixels(W, H, 1, 0, P)):
                    cur = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
                    n = int(pix_np.shape[0])
                    cur.view(2 * WH, 48)[:n] = base.view(WH, 48)[torch.from_numpy(pix_np).to(dev)]
                    torch.cuda.synchronize(dev)
                    bufs, counts = [cur.clone()], [n]
                    for b in range(nb):
                        e.trace(cur, counts[-1], b, far, W, H, device=True)
                        counts.append(e.enqueue_bounce(cur, counts[-1], b, far, W, H, frames=f,
                                                       max_bounce=max(nb, 1), device=True))
                        bufs.append(cur.clone())
                    torch.cuda.synchronize(dev)
                    chains[f].append((e, bufs, counts))
            del base
            k_frame = [0]

            def frame():
                ch = chains[k_frame[0] % n_frames]
                k_frame[0] += 1
                for b in range(nb + 1):
                    for e, bufs, counts in ch:
                        e.trace(bufs[b], counts[b], b, far, W, H, info=info, colors=colors_t if b > 0 else None,
                                device=True, asynchronous=True, flags=flags if b == 0 else 0)

            reps = max(4, args.steps // 2) // n_frames * n_frames
            for _ in range(max(2, args.warmup)):
                frame()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(reps):
                frame()
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) * 1e3 / reps
            rays = sum(sum(sum(c) for _, _, c in ch) for ch in chains) / n_frames
            return {"ms_per_frame": round(ms, 4), "mrays_s": round(rays / ms / 1e3, 1), "rays": int(rays)}
        finally:
            for e1 in extra_engs:
                e1.close()

    def slots_layout(view, W, H, nb, colors_t, adaptive=False):
        """The whole frame as one launch per bounce in the kernel's own order, N1_SLOTS frames in flight
        (bench.py's N = 1 layout): slot f has its own context (borrowing the scene), its own stream with a
        HW queue of its own, its own copies of the bounce chain's ray buffers and its own
        _PrimaryTriangleInfo; frame k runs its bounce chain on slot k mod N1_SLOTS. Wall ms per frame,
        frames back to back. adaptive: TT_TRACE_ADAPTIVE_ORDER on the primary launches, each slot's
        frames alternating between two jittered samples (frames_accumulated 0 / 1), so a launch's order
        comes from its context's previous frame, never from its own rays."""
        n_var = 2 if adaptive else 1
        flags = tthip.TT_TRACE_ADAPTIVE_ORDER if adaptive else 0
        fr = [rays_with_bounces(view, W, H, nb, v) for v in range(n_var)]
        engs, chains = [eng], []
        try:
            for f in range(1, N1_SLOTS):
                e1 = tthip.Engine(dev.index, stream=tthip.dedicated_stream(torch, dev, f - 1).cuda_stream)
                e1.share_scene(eng)
                e1.set_timing(False)  # (wall clock; no per-launch markers, tt_ctx_set_timing)
                engs.append(e1)
            for f, e in enumerate(engs):
                chains.append((e, [([b.clone() for b in bufs] if f else bufs, counts) for bufs, counts in fr],
                               torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)))
            torch.cuda.synchronize(dev)
            k_frame = [0]

            def frame():
                k = k_frame[0]
                e, var, inf = chains[k % N1_SLOTS]
                bf, counts = var[(k // N1_SLOTS) % n_var]
                k_frame[0] += 1
                for b in range(nb + 1):
                    e.trace(bf[b], counts[b], b, far, W, H, info=inf, colors=colors_t if b > 0 else None,
                            device=True, asynchronous=True, flags=flags if b == 0 else 0)

            for _ in range(max(2, args.warmup) * N1_SLOTS * n_var):
                frame()
            torch.cuda.synchronize(dev)
            reps = max(4, args.steps // 2) * N1_SLOTS * n_var
            t0 = time.perf_counter()
            for _ in range(reps):
                frame()
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) * 1e3 / reps
            rays = int(round(sum(sum(c) for _, c in fr) / n_var))
            return {"ms_per_frame": round(ms, 4), "mrays_s": round(rays / ms / 1e3, 1), "rays": rays}
        finally:
            for e1 in engs[1:]:
                e1.close()
            del chains, fr

    def adaptive_one_launch(view, W, H, nb, info, colors_t):
        """TT_TRACE_ADAPTIVE_ORDER with one launch per bounce: two jittered frames alternate (each launch
        ordered by the previous frame's costs; the primary launches flagged); per-bounce HIP-event ms (order
        kernel included)."""
        fr = [rays_with_bounces(view, W, H, nb, f) for f in range(2)]
        launches = [(lambda bufs=bufs, counts=counts, b=b: eng.trace(
            bufs[b], counts[b], b, far, W, H, info=info, colors=colors_t if b > 0 else None, device=True,
            asynchronous=True, flags=tthip.TT_TRACE_ADAPTIVE_ORDER if b == 0 else 0))
            for bufs, counts in fr for b in range(nb + 1)]
        ms = timed_launches(eng, launches, max(2, args.warmup), max(2, args.steps // 4))
        ms = ms.reshape(-1, nb + 1)  # rows: frames
        rays = [sum(c[b] for _, c in fr) / 2.0 for b in range(nb + 1)]
        mean = ms.mean(0)
        del fr
        return {"trace_ms": [round(float(m), 4) for m in mean],
                "mrays_s": round(float(sum(rays)) / float(mean.sum()) / 1e3, 1), "rays_mean": [int(r) for r in rays]}

    def run(name, scene_fn, view, W, H, nb, extra_fn, with_parts=False, adaptive=False):
        try:
            t0 = time.time()
            sc = scene_fn()
            build_s = time.time() - t0
            eng.upload(sc)
            bufs, counts = rays_with_bounces(view, W, H, nb, 0)
            info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
            colors = np.zeros(W * H, tthip.COL_DTYPE)
            colors["Data"][:, 3] = 1.0  # as the metric's step: info re-written at bounce 1 only
            colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
            launches = [(lambda b=b: eng.trace(bufs[b], counts[b], b, far, W, H, info=info,
                                               colors=colors_t if b > 0 else None, device=True,
                                               asynchronous=True)) for b in range(nb + 1)]
            ms = timed_launches(eng, launches, max(1, args.warmup), max(3, args.steps // 2))
            extra = dict(extra_fn(sc), width=W, height=H, build_s=round(build_s, 1))
            del bufs
            if with_parts:
                for P, key in ((2, "two_parts_two_streams"), (3, "three_parts_three_streams")):
                    try:
                        extra[key] = parts_layout(sc, view, W, H, nb, info, colors_t, P)
                    except Exception as e:  # noqa: BLE001
                        extra[key] = {"error": f"{type(e).__name__}: {e}"}
            if with_parts:  # the N = 1 headline's layout: one launch per bounce, N1_SLOTS frames in flight
                try:
                    extra[f"one_launch_{N1_SLOTS}_frame_slots"] = slots_layout(view, W, H, nb, colors_t)
                except Exception as e:  # noqa: BLE001
                    extra[f"one_launch_{N1_SLOTS}_frame_slots"] = {"error": f"{type(e).__name__}: {e}"}
            if adaptive:  # TT_TRACE_ADAPTIVE_ORDER (tt_order.hip), frames alternating
                try:
                    ad = {"one_launch_per_bounce": adaptive_one_launch(view, W, H, nb, info, colors_t)}
                    if with_parts:
                        ad["two_parts_two_streams"] = parts_layout(sc, view, W, H, nb, info, colors_t, 2, True)
                        ad[f"one_launch_{N1_SLOTS}_frame_slots"] = slots_layout(view, W, H, nb, colors_t, True)
                    ad["note"] = ("primary launches flagged (a compacted bounce list's chunks shift from frame to "
                                  "frame, DESIGN.md 3.1); two jittered frames (frames_accumulated 0 / 1) alternate, "
                                  "so a launch's order comes from the previous frame's costs; order kernel inside "
                                  "the per-launch HIP-event times")
                    extra["adaptive_order"] = ad
                except Exception as e:  # noqa: BLE001
                    extra["adaptive_order"] = {"error": f"{type(e).__name__}: {e}"}
            pack(name, counts, ms, extra)
            del info, colors_t
            return sc
        except Exception as e:  # auxiliary: record, never lose the metric line
            out[name] = {"error": f"{type(e).__name__}: {e}"}
            log(f"aux {name} failed: {e}")
            return None

    def time_calls(fn, warmup, steps):
        """Per-call GPU time (ms) of `fn` (one asynchronous engine call on the shared stream) from
        the engine's timing ring: HIP events around the call's device work on that stream."""
        for _ in range(warmup):
            fn()
        eng.timing_reset()
        for _ in range(steps):
            fn()
        return ring_tail(eng, 1, steps)[:, 0]

    if "c3" in which:
        run("c3_sponza_primary_plus_3_bounces_1080p", T.c2_sponza, T.C2_VIEW, 1920, 1080, 3,
            lambda sc: {"tris": int(len(sc.tris))}, with_parts=True)
    sc4 = None
    if "c4" in which:
        sc4 = run("c4_bistro_primary_plus_1_bounce_1080p", T.c4_bistro, T.C4_VIEW, 1920, 1080, 1,
            lambda sc: {"unique_tris": int(len(sc.tris)), "instanced_tris": sc.meta["instanced_tris"],
                        "unique_blas": 600, "instances": 2400, "cwbvh_nodes": int(len(sc.nodes))},
            with_parts=True, adaptive=True)
    if "dyn" in which:
        # the reference's per-frame dynamic-scene update on C4 (AssetManager.cs:1767-1826): every
        # frame rewrites all _MeshData records (MeshDataBuffer.SetData, :1825) and refits the TLAS
        # (RefitTLAS, :1821-1823, :1473-1606) before tracing. Here: tt_scene_update_meshdata of all
        # 2,401 records from a host array + tt_tlas_refit from device AABBs + Generate + primary
        # trace + diffuse enqueue + bounce-1 trace, the instances alternating between two poses (a
        # 5 cm shift of every instance). Wall time per frame and the host time of the update call.
        rec = {}
        try:
            if sc4 is None:
                sc4 = T.c4_bistro()
            eng.upload(sc4)
            W, H = 1920, 1080
            n_md = len(sc4.meshdata)
            md_a = sc4.meshdata.copy()
            md_b = sc4.meshdata.copy()
            box_a = np.ascontiguousarray(sc4.meta["mesh_aabbs"], np.float32).reshape(n_md, 6)
            box_b = box_a.copy()
            d = np.array([0.05, 0.0, 0.02])
            shift = np.eye(4)
            shift[:3, 3] = -d
            for i in range(1, n_md):  # record 0: the static street parent
                w2l = md_a["W2L"][i].astype(np.float64).reshape(4, 4).T
                md_b["W2L"][i] = tthip.unity_colmajor(w2l @ shift)
                box_b[i, 0:3] += d.astype(np.float32)
                box_b[i, 3:6] += d.astype(np.float32)
            boxes = [torch.from_numpy(box_a).to(dev), torch.from_numpy(box_b).to(dev)]
            mds = [md_a, md_b]
            c2w, ip = T.C4_VIEW.camera(W, H)
            rays = torch.zeros(2 * W * H * 48, dtype=torch.uint8, device=dev)
            info = torch.zeros(W * H * 16, dtype=torch.uint8, device=dev)
            colors = np.zeros(W * H, tthip.COL_DTYPE)
            colors["Data"][:, 3] = 1.0
            colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
            host_upd, host_refit, nbs = [], [], []

            def frame(k, record):
                t0 = time.perf_counter()
                eng.update_meshdata(0, mds[k])
                t1 = time.perf_counter()
                eng.tlas_refit(sc4.tlas_nodes, boxes[k], device=True, asynchronous=True)
                t2 = time.perf_counter()
                eng.generate(rays, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=0, max_bounce=1, device=True)
                eng.trace(rays, W * H, 0, far, W, H, info=info, device=True, asynchronous=True)
                nb_ = eng.enqueue_bounce(rays, W * H, 0, far, W, H, frames=0, max_bounce=1, device=True)
                eng.trace(rays, nb_, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)
                if record:
                    host_upd.append(t1 - t0)
                    host_refit.append(t2 - t1)
                    nbs.append(nb_)

            for k in range(max(2, args.warmup)):
                frame(k & 1, False)
            torch.cuda.synchronize(dev)
            reps = max(6, args.steps // 2)
            tf = time.perf_counter()
            for k in range(reps):
                frame(k & 1, True)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - tf) * 1e3 / reps
            # the update + refit alone on the stream (HIP events around the refit; the update's
            # device work is one H2D copy + one small kernel)
            eng.timing_reset()
            for k in range(reps):
                eng.update_meshdata(0, mds[k & 1])
                eng.tlas_refit(sc4.tlas_nodes, boxes[k & 1], device=True, asynchronous=True)
            refit_ms = ring_tail(eng, 1, reps)[:, 0]
            eng.upload(sc4)  # leave the scene as built
            # the frame-slot counts (--dyn-slots, a comma list): the first is `frame_slots`, the others go
            # under `frame_slots_more` (more frames in flight hide more of each frame's serial small work)
            slots_recs = []
            for S_ in [int(v) for v in str(args.dyn_slots).split(",") if v.strip()]:
                try:
                    slots_recs.append(dyn_frame_slots(torch, tthip, eng, dev, sc4, mds, boxes, args, W, H, S_))
                except Exception as e:  # noqa: BLE001
                    slots_recs.append({"slots": S_, "error": f"{type(e).__name__}: {e}"})
            slots_rec = slots_recs[0] if slots_recs else None
            eng.upload(sc4)
            rays_f = W * H + float(np.mean(nbs))
            rec = {"instances_updated": n_md, "tlas_nodes": int(sc4.tlas_nodes), "frames": reps,
                   "ms_per_frame": round(ms, 4), "mrays_s": round(rays_f / ms / 1e3, 1),
                   "update_meshdata_host_ms_median": round(float(np.median(host_upd)) * 1e3, 4),
                   "update_meshdata_host_ms_max": round(float(np.max(host_upd)) * 1e3, 4),
                   "tlas_refit_host_ms_median": round(float(np.median(host_refit)) * 1e3, 4),
                   "tlas_refit_gpu_ms_median": round(float(np.median(refit_ms)), 4),
                   "note": "frame = update_meshdata (all records, host array, async) + tlas_refit (device boxes) + "
                           "Generate + primary trace + enqueue (returns the count: one sync) + bounce-1 trace",
                   "frame_slots": slots_rec,
                   "frame_slots_more": {str(r_.get("slots")): r_ for r_ in slots_recs[1:]}}
        except Exception as e:  # auxiliary: record, never lose the metric line
            rec["error"] = f"{type(e).__name__}: {e}"
        out["c4_dynamic_frame"] = rec
        log(f"aux c4 dynamic frame: {rec}")
    if "refit" in which:
        # row f4 per frame: the GPU TLAS refit of the C4 scene (AssetManager.RefitTLAS, 2,400
        # instance boxes -> TLAS nodes) and the BLAS refit of the C2 mesh as a deforming mesh
        # (ParentObject.RefitMesh: 262k triangles re-derived + BLAS refit), device-resident inputs.
        rec = {}
        try:
            if sc4 is None:
                sc4 = T.c4_bistro()
            eng.upload(sc4)
            aabbs = torch.from_numpy(np.ascontiguousarray(sc4.meta["mesh_aabbs"], np.float32)).to(dev)
            ms = time_calls(lambda: eng.tlas_refit(sc4.tlas_nodes, aabbs, device=True, asynchronous=True),
                            3, max(5, args.steps))
            rec["tlas_refit_c4"] = {"instances": int(len(sc4.meshdata)), "tlas_nodes": int(sc4.tlas_nodes),
                                    "ms_median": round(float(np.median(ms)), 4), "ms_mean": round(float(ms.mean()), 4)}
            mesh = tthip.Mesh.sponza()
            blas = tthip.Blas(mesh)
            am = tthip.AssetManager()
            am.add_parent(blas, None, np.zeros(7, tthip.MAT_DTYPE))
            eng.upload(am.build())
            pos, nrm, idx = mesh.arrays()
            vtx = np.zeros((len(pos), 10), np.float32)  # Unity-like stride: position, normal, tangent
            vtx[:, 0:3], vtx[:, 3:6] = pos, nrm
            v_t = torch.from_numpy(vtx).to(dev)
            i_t = torch.from_numpy(np.ascontiguousarray(idx, np.int32)).to(dev)
            l_t = torch.from_numpy(blas.leaf_order()).to(dev)
            ms = time_calls(lambda: eng.blas_refit(0, v_t, i_t, l_t, None, device=True, asynchronous=True),
                            3, max(5, args.steps))
            n_tris = int(len(idx) // 3)
            rec["blas_refit_c2"] = {"tris": n_tris, "ms_median": round(float(np.median(ms)), 4),
                                    "ms_mean": round(float(ms.mean()), 4),
                                    "mtris_s": round(n_tris / float(np.median(ms)) / 1e3, 1)}
        except Exception as e:  # auxiliary: record, never lose the metric line
            rec["error"] = f"{type(e).__name__}: {e}"
        out["f4_refit_per_frame"] = rec
        log(f"aux refit: {rec}")
    if "c5" in which:
        run("c5_san_miguel_primary_4k", T.c5_san_miguel, T.C5_VIEW, 3840, 2160, 0,
            lambda sc: {"tris": int(len(sc.tris)), "cwbvh_nodes": int(len(sc.nodes))}, with_parts=True,
            adaptive=True)
    return out


def lpt_deal(torch, tthip, ttdist, eng, dev, W, H, c2w, ip, near, far, world, args):
    """The strong-scaling deal of 64x64 tiles to ranks: round-robin (--deal rr), or
    longest-processing-time first (--deal lpt, default) by the tile costs of a previous frame -- here sample
    0 traced once at setup on every rank's own GPU with TT_TRACE_ADAPTIVE_ORDER, whose per-8x8-chunk cost
    map (tt_trace_chunk_costs: the chunk's longest ray in node steps) is summed per tile. The trace is
    deterministic, so every rank computes the same deal without a collective. Returns (owner or None, info)."""
    if args.deal != "lpt" or world == 1:
        return None, {"deal": "round-robin"}
    full = torch.zeros(W * H * 48, dtype=torch.uint8, device=dev)
    eng.generate(full, c2w, ip, W, H, near, far, jitter=1, frames=0, max_bounce=1, device=True)
    eng.trace(full, W * H, 0, far, W, H, device=True, flags=tthip.TT_TRACE_ADAPTIVE_ORDER)
    cc = eng.chunk_costs(0)
    del full
    costs = ttdist.tile_costs_from_chunks(cc, W, H)
    owner = ttdist.lpt_owner(costs, world)
    loads = np.bincount(owner, weights=costs, minlength=world)
    rr = np.bincount(np.arange(len(costs)) % world, weights=costs, minlength=world)
    return owner, {"deal": "lpt", "cost_source": "sample 0, tt_trace_chunk_costs (per 8x8 chunk: longest ray's node steps,"
                                                 " floor 24) summed per 64x64 tile",
                   "max_over_mean_cost": round(float(loads.max() / loads.mean()), 4),
                   "round_robin_max_over_mean_cost": round(float(rr.max() / rr.mean()), 4)}


def split_batched_gather(blocks, sizes, B):
    """A gather of B-frame launches (FrameLayout batch B): every rank's block holds its parts back to back, each
    part's records the B frames' back to back. Returns per frame b: (blocks, sizes) as assemble_parts takes them."""
    # (the RCCL gather's blocks are device tensors: one copy to the host each, numpy from there on)
    blocks = [g.cpu().numpy() if hasattr(g, "cpu") else np.asarray(g) for g in blocks]
    out = []
    for b in range(B):
        fb, sb = [], []
        for g, n in zip(blocks, sizes):
            rows, ns, o = [], [], 0
            for n_p in n:
                m = n_p // B
                rows.append(g[o + b * m:o + (b + 1) * m])
                ns.append(m)
                o += n_p
            fb.append(np.concatenate(rows) if rows else g[:0])
            sb.append(ns)
        out.append((fb, sb))
    return out


def node_fetch_model(dom, s_prim, s_bnc, parts):
    """The dominant launch's node visits per second against the rate one MI355X sustains for scattered 80-B node
    fetches (tools/micro/coop_fetch.hip -> profiles/node_fetch_latest.json): from L2-resident tables and from a
    table the size of the scene's node set. A model of the memory path the node loads use (their texture-data
    busy, roofline.binding_unit), not a bound: the kernel's visits mix L1 / L2 hits of the hot top levels with
    misses."""
    try:
        nf = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                         "node_fetch_latest.json")))["scatter_gnodes_s"]
    except (OSError, ValueError, KeyError):
        return None
    if not dom:
        return None
    bounce = dom["kernel"].endswith("2>")
    st, n = (s_bnc, parts[0].nb) if bounce else (s_prim, parts[0].n)
    if not n:
        return None
    npr = st.node_visits / n
    g = dom["grays_s"] * npr
    l2 = max(nf.get("table_1MiB", 0.0), nf.get("table_2MiB", 0.0))
    return {"kernel": dom["kernel"], "nodes_per_ray": round(npr, 3), "launch_gnodes_s": round(g, 2),
            "scatter_l2_resident_gnodes_s": l2, "frac_l2_resident": round(g / l2, 4) if l2 else None,
            "scatter_40MiB_gnodes_s": nf.get("table_40MiB"),
            "note": "a model, not a bound: node visits per second of the dominant launch vs the scattered 80-B node "
                    "fetch rate of tools/micro/coop_fetch.hip (profiles/node_fetch_latest.json)"}


def dyn_frame_slots(torch, tthip, eng, dev, sc4, mds, boxes, args, W, H, S):
    """The reference's dynamic frame (AssetManager.cs:1767-1826: every _MeshData record rewritten and the TLAS
    refit, then the traces) with N1_SLOTS frames in flight: slot f is a context with a TLAS, TLASBVH8Indices and
    _MeshData of its own over `eng`'s BLASes and triangles (tt_ctx_share_blas; slot 0 is `eng` itself), on a
    stream with a HW queue of its own. Frame k runs on slot k % N1_SLOTS: update_meshdata (pose k & 1, all
    records) + tlas_refit + Generate (frames_accumulated = k) + primary trace + the diffuse enqueue with a
    device-resident count + the indirect bounce-1 trace, every call asynchronous -- no host synchronization and
    no wait on another slot. Afterwards each slot's last frame (hit records of both bounces, both
    _PrimaryTriangleInfo forms) is compared byte for byte with one context issuing the same frame serially."""
    import ttconfigs as T

    WH = W * H
    far = T.FAR
    T_ = int(sc4.tlas_nodes)
    c2w, ip = T.C4_VIEW.camera(W, H)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0
    colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    S = max(1, int(S))
    engs, streams = [eng], [torch.cuda.ExternalStream(eng.stream, device=dev)]
    for f in range(1, S):
        st = tthip.dedicated_stream(torch, dev, f - 1)
        e = tthip.Engine(dev.index, stream=st.cuda_stream)
        e.share_blas(eng, T_)
        e.set_timing(False)  # (wall clock; no per-launch markers, tt_ctx_set_timing)
        engs.append(e)
        streams.append(st)
    bufs = [dict(rays=torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev),
                 i0=torch.zeros(WH * 16, dtype=torch.uint8, device=dev),
                 i1=torch.zeros(WH * 16, dtype=torch.uint8, device=dev)) for _ in range(S)]
    n_frames = max(2, args.warmup) * S + max(6, args.steps // 2) * S
    counts = torch.zeros(n_frames, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    host_ms = []

    def frame(k):
        f = k % S
        e, b = engs[f], bufs[f]
        t0 = time.perf_counter()
        if "noupdate" not in args.dyn_diag:  # (diagnosis: which per-frame call costs what, --dyn-diag)
            e.update_meshdata(0, mds[k & 1])
            e.tlas_refit(T_, boxes[k & 1], device=True, asynchronous=True)
        if "nogen" not in args.dyn_diag or k < S:
            e.generate(b["rays"], c2w, ip, W, H, T.NEAR, far, jitter=1, frames=k, max_bounce=1, device=True,
                       asynchronous=True)
        # (the adaptive order on the primaries, INTEGRATION.md §5's advice for scenes beyond the L2s: each slot's
        # launch ordered by its own previous frame -- another pose and jitter)
        e.trace(b["rays"], WH, 0, far, W, H, info=b["i0"], device=True, asynchronous=True,
                flags=tthip.TT_TRACE_ADAPTIVE_ORDER if args.dyn_adaptive else 0)
        # BufferSizes[1].tracerays straight into this frame's entry of the count log (no copy on the stream)
        cnt = counts[k:k + 1]
        e.enqueue_bounce_indirect(b["rays"], None, WH, cnt, 0, far, W, H, frames=k, max_bounce=1)
        e.trace_indirect(b["rays"], cnt, WH, 1, far, W, H, info=b["i1"], colors=colors_t)
        host_ms.append((time.perf_counter() - t0) * 1e3)

    k = 0
    eng.set_timing(False)  # (wall clock: no per-launch timing markers on slot 0 either, tt_ctx_set_timing)
    try:
        for _ in range(max(2, args.warmup) * S):
            frame(k)
            k += 1
        torch.cuda.synchronize(dev)
        k0 = k
        reps = max(6, args.steps // 2) * S
        t0 = time.perf_counter()
        for _ in range(reps):
            frame(k)
            k += 1
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / reps
        nb = counts[k0:k].cpu().numpy().astype(np.int64)
        rays = reps * WH + int(nb.sum())
        got = [{key: bufs[f][key].cpu().numpy() for key in ("rays", "i0", "i1")} | {"k": kk, "nb": int(counts[kk].item())}
               for f, kk in ((kk % S, kk) for kk in range(k - S, k))]
    finally:
        eng.set_timing(True)
        for e in engs[1:]:
            e.close()
    # the serial reference: one context, the same calls for each slot's last frame, synchronously
    ref = tthip.Engine(dev.index)
    same = True
    diff = []
    try:
        ref.upload(sc4)
        rr = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        r0 = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
        r1 = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
        for g in got:
            kk = g["k"]
            ref.update_meshdata(0, mds[kk & 1])
            ref.tlas_refit(T_, boxes[kk & 1], device=True)
            ref.generate(rr, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=kk, max_bounce=1, device=True)
            ref.trace(rr, WH, 0, far, W, H, info=r0, device=True)
            nb_ref = ref.enqueue_bounce(rr, WH, 0, far, W, H, frames=kk, max_bounce=1, device=True)
            ref.trace(rr, nb_ref, 1, far, W, H, info=r1, colors=colors_t, device=True)
            torch.cuda.synchronize(dev)
            a = rr.view(-1, 48).cpu().numpy()
            gv = g["rays"].reshape(-1, 48)
            # the bounce-1 _PrimaryTriangleInfo texels this frame writes: the pixels of its bounce-1 rays (the
            # others keep an earlier frame's texel, on either side)
            pix = gv[WH:WH + g["nb"], 12:16].copy().view(np.uint32).reshape(-1).astype(np.int64)
            i1a, i1b = r1.cpu().numpy().reshape(-1, 16), g["i1"].reshape(-1, 16)
            d = {"frame": kk, "bounce_count": nb_ref == g["nb"], "primary_records": bool(np.array_equal(a[:WH], gv[:WH])),
                 "bounce_records": bool(np.array_equal(a[WH:WH + nb_ref], gv[WH:WH + nb_ref])),
                 "info_bounce0": bool(np.array_equal(r0.cpu().numpy(), g["i0"])),
                 "info_bounce1": bool(nb_ref == g["nb"] and np.array_equal(i1a[pix], i1b[pix]))}
            diff.append(d)
            same = same and all(v for k_, v in d.items() if k_ != "frame")
    finally:
        ref.close()
    return {"slots": S, "frames": reps, "ms_per_frame": round(ms, 4), "mrays_s": round(rays / reps / ms / 1e3, 1),
            "adaptive_order_primary": bool(args.dyn_adaptive), "diagnosis": args.dyn_diag or None,
            "rays_per_frame_mean": int(round(rays / reps)), "host_ms_per_frame_median": round(float(np.median(host_ms)), 4),
            "identical_to_serial": bool(same), "checks": diff,
            "note": f"frame k on slot k % {S}, each slot a context with its own TLAS / _MeshData over the shared BLASes "
                    "(tt_ctx_share_blas): update_meshdata (all records) + tlas_refit + Generate (frames_accumulated = k) + "
                    "primary + enqueue (device count) + indirect bounce-1, all asynchronous; each slot's last frame "
                    "compared with one context issuing the same calls serially"}


def c5_tiles(torch, dist, tthip, eng, dev, red_dev, args, rank, world):
    """BASELINE configs[4] as the north star lays it out, run after the metric when
    N > 1: the San-Miguel-shaped scene (10 M tris) replicated on every rank, the 3840x2160 frame's
    64x64 tiles dealt round-robin, each rank tracing its tiles' primary rays as P parts x F frame slots
    (ttlayout.FrameLayout: frame k + 1 overlaps frame k's drain), one RCCL gather of the frame's 16-B hit
    records to rank 0 per frame, which reassembles the frame and compares it with one GPU tracing the
    whole frame. Strong scaling: frame time = slowest rank; efficiency against the N = 1 frame (the whole
    4K frame, 2 parts, 1 slot) traced on every rank's own GPU at once in the same run (fastest).
    Failures are agreed on collectively before the gather, so one rank's error cannot hang the rest."""
    import ttconfigs as T
    import ttdist
    import ttlayout

    rec, ok = {}, 1
    W, H, far = 3840, 2160, T.FAR
    WH = W * H
    F = max(1, args.strong_slots)
    P = max(1, args.strong_parts)
    el1 = el_n = 0.0
    lay = None
    try:
        t0 = time.time()
        sc = T.c5_san_miguel()
        build_s = time.time() - t0
        eng.upload(sc)
        c2w, ip = T.C5_VIEW.camera(W, H)
        make_full = ttlayout.full_frame_maker(torch, eng, dev, W, H, c2w, ip, T.NEAR, far)

        def timed_layout(plan, slots=F, batch=1):
            # every frame slot its own jittered samples, cycling through args.cycle of them (ttlayout docstring);
            # batch: frames per launch (the rank's shards at N > 1, bench.py --batch)
            lay_ = ttlayout.FrameLayout(torch, tthip, eng, dev, W, H, far, plan, make_full, slots=slots, bounce=False,
                                        info=False, slot_stride=batch, cycle=args.cycle, batch=batch)
            for _ in range(max(2, args.warmup)):
                lay_.step()
            torch.cuda.synchronize(dev)
            lay_.timing_reset()
            reps = max(4, args.steps // 2)
            tp = time.perf_counter()
            for _ in range(reps):
                lay_.step()
            torch.cuda.synchronize(dev)
            el = (time.perf_counter() - tp) * 1e3 / reps / batch  # per frame
            lay_.launch_ms()
            return lay_, el

        # the N = 1 frame on every rank's GPU at once (no collective), in both single-GPU layouts (2 parts x 1
        # slot; one launch in the kernel's own order with N1_SLOTS frames in flight); t(1) = the faster
        solo, el1a = timed_layout([[(0, pix)] for pix in ttdist.part_pixels(W, H, 1, 0, 2)], slots=1)
        solo.close()
        solo, el1b = timed_layout([[(0, np.arange(WH, dtype=np.int64))]], slots=N1_SLOTS)
        solo.close()
        del solo
        el1 = min(el1a, el1b)
        rec["n1_ms_per_frame_by_layout_rank"] = {"2x1": round(el1a, 4), f"1x{N1_SLOTS}": round(el1b, 4)}
        owner, deal = lpt_deal(torch, tthip, ttdist, eng, dev, W, H, c2w, ip, T.NEAR, far, world, args)
        B5 = max(1, args.batch)
        lay, el_n = timed_layout([[(b, pix) for b in range(B5)]
                                  for pix in ttdist.part_pixels(W, H, world, rank, P, owner=owner)], batch=B5)
        rec.update(rays_this_rank=lay.n_prim(), build_s=round(build_s, 1), tile_deal=deal)
    except Exception as e:  # noqa: BLE001 — auxiliary; agreed on below
        ok = 0
        rec["error"] = f"rank {rank}: {type(e).__name__}: {e}"
        log(f"c5 tiles failed: {rec['error']}")
    flags = torch.tensor([float(ok)], dtype=torch.float64, device=red_dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if flags[0].item() < 1.0:
        if lay is not None:
            lay.close()
        return rec if rank == 0 else None
    t1 = torch.tensor([el1], dtype=torch.float64, device=red_dev)
    dist.all_reduce(t1, op=dist.ReduceOp.MIN)
    tn = torch.tensor([el_n], dtype=torch.float64, device=red_dev)
    dist.all_reduce(tn, op=dist.ReduceOp.MAX)
    # the frame again, with the per-frame gather inside the timed frames (on the comm stream)
    lay.attach_gather(dist, world, rank, red_dev)
    for _ in range(max(2, args.warmup)):
        lay.step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    reps = max(4, args.steps // 2)
    tg = time.perf_counter()
    for _ in range(reps):
        lay.step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    el_g = (time.perf_counter() - tg) * 1e3 / reps / lay.B  # per frame
    lay.launch_ms()
    tgm = torch.tensor([el_g], dtype=torch.float64, device=red_dev)
    dist.all_reduce(tgm, op=dist.ReduceOp.MAX)
    sizes, gl = lay.last_gathered() if rank == 0 else (None, None)
    B5 = lay.B
    last_samples = [lay.last_sample(b) for b in range(B5)]
    lay.close()
    if rank != 0:
        return None
    identical = True
    for b, (fb, sb) in enumerate(split_batched_gather([g[:sum(n)] for g, n in zip(gl, sizes)], sizes, B5)):
        frame = ttdist.assemble_parts(fb, sb, W, H, world, P, owner=owner)
        full = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(full, c2w, ip, W, H, T.NEAR, far, jitter=1, frames=last_samples[b], max_bounce=1, device=True)
        eng.trace(full, WH, 0, far, W, H, device=True)
        ref = full.view(WH, 48)[:, 32:48].contiguous().view(torch.int32).cpu().numpy().view(np.uint32)
        identical = identical and bool(np.array_equal(frame, ref))
    ms1, msn, msg = float(t1.item()), float(tn.item()), float(tgm.item())
    rec.update(config="c5_san_miguel_4k_tiles", ranks=world, tile=64, parts_per_rank=P, frame_slots=F,
               frame_rays=WH, n1_ms_per_frame=round(ms1, 4), ms_per_frame_slowest_rank=round(msn, 4),
               efficiency=round(ms1 / (world * msn), 4), mrays_s_frame=round(WH / msn / 1e3, 1),
               with_gather=dict(ms_per_frame_slowest_rank=round(msg, 4), efficiency=round(ms1 / (world * msg), 4),
                                mrays_s_frame=round(WH / msg / 1e3, 1)),
               identical_to_1gpu=identical, frames_per_launch=B5,
               note="efficiency = t(N = 1: the whole 4K frame in the faster single-GPU layout, on every rank's GPU "
                    "at once, fastest) / (N x t(N), slowest rank); with_gather: the per-frame RCCL gather of the hit "
                    "records to rank 0 inside the timed frames")
    log(f"c5 tiles: {rec}")
    return rec


def group_tiles(torch, dist, args, rank, world, backend, red_dev, gpu, W, H):
    """aux_group_tiles: the LIBRARY's multi-GPU path (tt_group_*, csrc/tt_group.hip) -- what a C# host calls --
    on this job's ranks: every rank starts tools/group_leg.py as a child process on its GPU; the children form
    one group (tt_group_unique_id on rank 0, tt_group_create_rank everywhere), replicate the scene
    (tt_group_scene_upload) and time K frames of tt_group_trace_frame: every rank generates and traces its
    64x64 tiles (round-robin) and their bounce-1 rays, and the primary hit records reach rank 0 in one RCCL
    gather per frame (inside the library), scattered back to screen order. Frames are asynchronous over
    --group-slots slots. value = all ranks' rays (primary + bounce 1) / the slowest rank's time; strong scaling
    (one 1080p frame per frame whatever N). At N = 1 the group has one member tracing the whole frame straight
    into the output (a one-rank group has nothing to gather).
    The child isolates the leg: its communicator and gathers can never stall the bench's own ranks -- a child
    that fails or exceeds the time limit is killed and the leg reports the failure."""
    import subprocess
    import tempfile

    if backend != "nccl":
        return {"skipped": "needs RCCL: one process per GPU"}
    d = tempfile.mkdtemp(prefix="tt_group_leg_") if rank == 0 else None
    if world > 1:
        box = [d]
        dist.broadcast_object_list(box, src=0)
        d = box[0]
    S = max(1, args.group_slots)
    R = max(1, args.cycle) if world > 1 else S
    # frames per call: as the torch layouts (--batch at N > 1, --n1-batch at N = 1): each call traces B samples of
    # the still view as one B-frames-tall screen (tt_group_config.batch)
    Bg = max(1, args.batch if world > 1 else args.n1_batch)
    cmd = [sys.executable, os.path.join(REPO, "tools", "group_leg.py"), "--rank", str(rank), "--world", str(world),
           "--device", str(gpu), "--dir", d, "--steps", str(args.group_frames), "--warmup", str(max(args.warmup, 10)),
           "--slots", str(S), "--cycle", str(R), "--batch", str(Bg), "--width", str(W), "--height", str(H),
           "--tris", str(args.tris),
           "--seed", hex(args.seed)]
    res, err = None, None
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.group_timeout)
        if r.returncode == 0 and r.stdout.strip():
            res = json.loads(r.stdout.strip().splitlines()[-1])
        else:
            err = f"rank {rank}: exit {r.returncode}: {r.stderr[-300:]}"
    except subprocess.TimeoutExpired:
        err = f"rank {rank}: the group leg exceeded {args.group_timeout} s (killed)"
    except Exception as e:  # noqa: BLE001
        err = f"rank {rank}: {type(e).__name__}: {e}"
    ok = torch.tensor([0.0 if res is None else 1.0], dtype=torch.float64, device=red_dev)
    el = torch.tensor([0.0 if res is None else res["elapsed_s"]], dtype=torch.float64, device=red_dev)
    per = torch.tensor([0.0] * R if res is None else [float(x) for x in res["rays_per_sample"]], dtype=torch.float64,
                       device=red_dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(per, op=dist.ReduceOp.SUM)
    if rank == 0:
        shutil.rmtree(d, ignore_errors=True)
    if float(ok.item()) < 1.0:
        return {"error": err or "another rank's group leg failed"}
    el = float(el.item())
    per = per.cpu().numpy()
    K = args.group_frames  # calls, Bg frames each
    rays = float(sum(per[k % R] for k in range(K)))
    out = {"value": round(rays / el / 1e6, 2), "unit": "Mrays/s", "scaling": "strong", "ranks": world,
           "ms_per_frame": round(el * 1e3 / (K * Bg), 4), "calls": K, "frames_per_call": Bg, "frame_slots": S,
           "samples_cycled": R * Bg, "rays_per_frame_all_ranks": int(round(rays / (K * Bg))),
           "gather_identical_to_1gpu": None if res is None else res.get("parity"),
           "api": "tt_group_unique_id + tt_group_create_rank + tt_group_scene_upload + tt_group_trace_frame "
                  "(TT_TRACE_ASYNC) + tt_group_sync, one child process per rank (tools/group_leg.py)",
           "layout": "one 1080p frame per step: 64x64 tiles round-robin over the ranks, each rank's Generate + "
                     "primary trace + bounce-1 enqueue/trace on its own device, one RCCL gather of the primary hit "
                     "records to rank 0 per frame inside the library (world 1: the whole frame traced straight into "
                     "the output, nothing to gather)"}
    if world > 1 and getattr(args, "_solo_ms", None):
        out["efficiency_vs_n1_frame"] = round(args._solo_ms / (world * el * 1e3 / (K * Bg)), 4)
    return out


def oracle_records_check(scene, layout, pre, post, colors, far, W, H):
    """The records the bench's timed launches wrote, against the oracle (oracle/tt_oracle.c through
    tests/oracle_ctypes.py -- the checker, never the measured path). `pre`: every slot's host state after
    FrameLayout.poison_records() (hit records and _PrimaryTriangleInfo filled with a poison byte); `post`:
    the same buffers after the timed steps. The oracle traces each slot's primary rays (bounce 0, with
    _PrimaryTriangleInfo) and bounce-1 rays (the GlobalColors-gated form) in place on `pre`; every 48-B
    RayData record and every 16-B _PrimaryTriangleInfo texel must then equal `post` byte for byte (a record
    neither side writes -- the Reps bound -- keeps the poison on both)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O

    t0 = time.perf_counter()
    hw, aff, quota = cpu_share()
    nthreads = max(1, min(aff, 64))
    H = layout.Hs  # a batch of B frames is one B-tall screen (FrameLayout batch): offsets, texels, colors
    if layout.B > 1:
        colors = np.tile(colors, layout.B)
    bad_rec = bad_info0 = bad_info1 = 0
    rays = 0
    samples = []
    for f, row in enumerate(layout.slots):
        samples.append(sorted({layout.sample_of(f, k) for lst in layout.plan for k, _ in lst}))
        for s_, p in enumerate(row):
            r = pre[f]["rays"][s_]
            O.trace(scene, r, p.n, 0, far, W, H, info=pre[f]["info0"], nthreads=nthreads)
            if layout.bounce and p.nb:
                O.trace(scene, r, p.nb, 1, far, W, H, info=pre[f]["info1"], colors=colors, nthreads=nthreads)
            rays += p.n + p.nb
            bad_rec += int(np.any(r.reshape(-1, 48) != post[f]["rays"][s_].reshape(-1, 48), axis=1).sum())
        for key in ("info0", "info1"):
            if pre[f][key] is not None:
                n_bad = int(np.any(pre[f][key].reshape(-1, 16) != post[f][key].reshape(-1, 16), axis=1).sum())
                if key == "info0":
                    bad_info0 += n_bad
                else:
                    bad_info1 += n_bad
    unwritten = sum(int(np.all(post[f]["rays"][s_].reshape(-1, 48)[:p.n, 32:48] == layout.POISON, axis=1).sum())
                    for f, row in enumerate(layout.slots) for s_, p in enumerate(row))
    return {"identical": bad_rec == 0 and bad_info0 == 0 and bad_info1 == 0,
            "mismatching_ray_records": bad_rec, "mismatching_info_bounce0": bad_info0,
            "mismatching_info_bounce1": bad_info1, "rays_checked": rays, "slots": layout.F,
            "samples_per_slot": samples, "primary_records_left_unwritten": unwritten,
            "kernels": "tt_trace_kernel<false,false,1> (primary) and <false,false,2> (bounce 1): the timed launches",
            "oracle": f"oracle/tt_oracle.c ({os.path.basename(O.lib()._path)}), {nthreads} threads",
            "seconds": round(time.perf_counter() - t0, 2)}


def cpu_share():
    """(hardware threads, CPUs this process may run on, cgroup CPU quota or None)."""
    hw = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = hw
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return hw, aff, quota


def cpu_baseline(scene, rays, info_n, n_prim, nb, colors, far, W, H, seconds):
    """The scalar oracle (oracle/tt_oracle.c, -O3, no intrinsics) on the host cores over the same
    step workload (primary + bounce-1 rays), repeated for ~`seconds`. Primary figure: every CPU the
    process may run on (sched_getaffinity); a 16-thread run is kept as a secondary field (the
    per-GPU CPU share the GPU box grants)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O  # the oracle is only the CPU baseline here, never the measured path
    import tthip

    host_rays = rays.cpu().numpy().view(tthip.RAY_DTYPE).copy()
    host_info = np.zeros((info_n, 4), np.uint32)
    hw, aff, quota = cpu_share()

    def run(nthreads, budget):
        done, reps, tc0 = 0, 0, time.perf_counter()
        while True:
            O.trace(scene, host_rays, n_prim, 0, far, W, H, info=host_info, nthreads=nthreads)
            O.trace(scene, host_rays, nb, 1, far, W, H, info=host_info, colors=colors, nthreads=nthreads)
            done += n_prim + nb
            reps += 1
            if time.perf_counter() - tc0 >= budget:
                break
        t = time.perf_counter() - tc0
        return done / t / 1e6, reps, t

    # thread counts tried: 16 (the per-GPU CPU share the GPU box grants), the cgroup quota rounded up
    # (capped at the affinity mask), and every CPU of the affinity mask; the baseline is the best
    # of them (an oversubscribed quota runs slower than the threads it can actually use)
    cands = sorted({min(16, aff), min(aff, math.ceil(quota)) if quota else aff, aff})
    runs = {}
    for nt in cands:
        runs[nt] = run(nt, seconds / len(cands))
        log(f"cpu baseline candidate: {nt} threads -> {runs[nt][0]:.3f} Mrays/s ({runs[nt][1]} reps)")
    best = max(runs, key=lambda k: runs[k][0])
    v_best, reps, tcpu = runs[best]
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    cpu = {"value": round(v_best, 3), "unit": "Mrays/s", "cores": best, "kind": "port",
           "host_cpu": model, "hardware_threads": hw, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
           "candidates": {str(k): round(v[0], 3) for k, v in runs.items()},
           "sample": f"full step workload ({n_prim} primary + {nb} bounce-1 rays) x {reps} in {tcpu:.1f}s, "
                     f"oracle/tt_oracle.c scalar C ({os.path.basename(O.lib()._path)}), {best} threads "
                     f"(the best of {cands} threads: 16, the cgroup quota {quota} rounded up, the affinity mask's "
                     f"{aff}); C# scalar baseline (bindings/csharp/ScalarTraversal.cs) "
                     + ("not run: no .NET runtime (dotnet) on the box" if shutil.which("dotnet") is None
                        else "not run by bench.py: see tools/dump_scene_raw.py")}
    log(f"cpu baseline {cpu['value']} Mrays/s on {best} threads ({reps} reps, {tcpu:.1f}s); all: {cpu['candidates']}")
    return cpu


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_ranks(n: int, argv, timeout=None) -> int:
    """`bench.py --gpus N` without a launcher: starts N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, as torchrun would),
    before this process touches the GPU. Rank 0 prints the JSON line. Returns the first failing rank's
    exit code (a rank killed by a signal counts as 128 + signal), 0 when all succeed; once one rank
    fails the others get a few seconds to finish, then are terminated so none is left blocked in a
    collective (the ranks terminated that way do not mask the first failure's code)."""
    import signal
    import subprocess

    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TT_BENCH_SELF_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      start_new_session=False))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}), master 127.0.0.1:{port}")
    t0 = time.time()
    rcs = [None] * n
    first_fail = None
    t_fail = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and first_fail is None:
                    first_fail, t_fail = rcs[i], time.time()
        failed = first_fail is not None and time.time() - t_fail > 5.0  # (a grace period to finish)
        late = timeout is not None and time.time() - t0 > timeout
        if (failed or late) and any(rc is None for rc in rcs):
            log(f"rank exit codes {rcs}{' (timeout)' if late else ''}: terminating the remaining ranks")
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            if late and not failed:
                rcs = [rc if rc else 124 for rc in rcs]
            break
        time.sleep(0.2)
    code = lambda rc: (128 - rc) if rc < 0 else rc  # Popen: -signal for a killed child
    codes = [code(rc) for rc in rcs]
    log(f"rank exit codes {codes}")
    return code(first_fail) if first_fail is not None else max(codes)


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU). Under a launcher (torchrun: WORLD_SIZE set) it must equal "
                         "WORLD_SIZE; without one, N > 1 starts N rank processes of this script itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tris", type=int, default=262267)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x53504F4E)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-oracle-check", action="store_true",
                    help="N = 1: skip the oracle check of the records the timed launches wrote (oracle_check)")
    ap.add_argument("--shard", choices=["spp", "tiles", "sample"], default="tiles",
                    help="N > 1 layout. tiles (default, strong scaling: the north star's layout, SURVEY.md §8(e)): ONE "
                         "1080p frame's 64x64 screen tiles dealt round-robin to the ranks, each rank tracing its tiles' "
                         "primary and bounce-1 rays, and the frame's primary hit records RCCL-gathered to rank 0 inside "
                         "every timed step; its efficiency against the N = 1 frame is in config.aux_strong_tiles. spp "
                         "(weak scaling, also reported as config.aux_spp_weak): the job at N ranks is an N-sample frame "
                         "whose (sample, tile) units are dealt round-robin (ttdist.spp_part_pixels), same gather. "
                         "sample: every rank traces its own full-frame sample, no collective (weak scaling)")
    ap.add_argument("--parts", type=int, default=0,
                    help="a rank's pixels (N = 1: the frame; N > 1: its tiles) are traced as this many tile-interleaved "
                         "parts, each by its own engine on its own stream (each part's bounce-1 after its own primary), "
                         "so one part's launch drain overlaps the other parts' work (tools/exp_streams.py). 1: one "
                         "launch per bounce; 0 (default): 2 for a full frame's worth per rank (N = 1, the spp "
                         "headline); the strong-scaling shards use --strong-parts")
    ap.add_argument("--slots", type=int, default=0,
                    help="frame slots F of the headline layout (ttlayout.FrameLayout): frame k runs on slot k %% F with "
                         "its own buffers and streams on HW queues of their own, so frames k + 1 .. k + F - 1 run while "
                         "frame k drains. 0 (default): N = 1 the whole frame as one launch per bounce with "
                         f"{N1_SLOTS} slots; 1 for the spp headline's frame's worth per rank; --strong-slots for the "
                         "strong-scaling shards (--shard tiles)")
    ap.add_argument("--strong-slots", type=int, default=6,
                    help="frame slots of the strong-scaling tile layouts (N > 1: aux_strong_tiles, aux_c5_tiles, "
                         "--shard tiles): frames k .. k + 5 of a rank in flight at once, each slot on its own HW "
                         "queue. 1 part x 6 slots is the best layout measured for the <= 1/2-frame shards "
                         "(tools/strong_replay.py, profiles/r04/replay/: C2 N = 8 0.135 ms per frame vs 0.155 / "
                         "0.150 with 4 / 3 slots and 0.223-0.271 with 2x2 / 2x1 / 3x1; C5 4K N = 8 0.241 vs 0.270 / "
                         "0.312)")
    ap.add_argument("--deal", choices=["lpt", "rr"], default="rr",
                    help="strong-scaling tile deal (N > 1): rr (default) = round-robin; lpt = longest-processing-time "
                         "first by a previous frame's tile costs (tt_trace_chunk_costs of sample 0, computed identically "
                         "on every rank). The one-GPU replay of every rank's N = 8 shard measured lpt no better "
                         "(profiles/r05/replay/: C2 0.616 vs 0.626, C5 4K 0.552 vs 0.576): C2's ranks are within noise "
                         "either way and C5's slowest rank is set by one degenerate ray's chain, not by its tile load")
    ap.add_argument("--strong-parts", type=int, default=1,
                    help="tile-interleaved parts per rank of the strong-scaling tile layouts (see --strong-slots)")
    ap.add_argument("--no-spp-aux", action="store_true",
                    help="N > 1, --shard tiles: skip the weak-scaling spp layout beside the headline (aux_spp_weak)")
    ap.add_argument("--no-strong", action="store_true",
                    help="N > 1: skip the strong-scaling 1080p tile layout and its N = 1 reference frame")
    ap.add_argument("--no-shadow", action="store_true", help="skip the auxiliary any-hit NEE measurement")
    ap.add_argument("--steady-steps", type=int, default=200,
                    help="N = 1: steps of the secondary steady-state leg after the timed region (0 = skip)")
    ap.add_argument("--no-single", action="store_true",
                    help="N = 1, parts > 1: skip the single-stream leg (one launch at a time; roofline.single_stream)")
    ap.add_argument("--no-recur", action="store_true",
                    help="skip the auxiliary unjittered (UseReCur) primary + bounce launches (profiling runs: they "
                         "use the metric's kernel instantiation and would mix into its rocprof average)")
    ap.add_argument("--no-c5-tiles", action="store_true",
                    help="N > 1: skip the tile-sharded San-Miguel 4K frame + hit gather run after the metric")
    ap.add_argument("--dyn-slots", default=f"{N1_SLOTS},6",
                    help="aux dyn: frame-slot counts (contexts with TLASes of their own) of the dynamic-frame leg, a "
                         "comma list: the first is the record's frame_slots, the others frame_slots_more")
    ap.add_argument("--n1-batch", type=int, default=4,
                    help="N = 1: frames each launch traces at once (the whole frame B times on a B-tall screen, each "
                         "frame its own sample; the in-run oracle check covers every record; 1 = one frame per launch, "
                         "rounds 1-5's headline layout)")
    ap.add_argument("--batch", type=int, default=4,
                    help="N > 1 strong-scaling headline: frames each launch traces at once (FrameLayout batch; 1 = one "
                         "frame per launch); N = 1 always 1")
    ap.add_argument("--cycle", type=int, default=6,
                    help="samples each frame slot cycles through in the N > 1 layouts (and aux_c5_tiles); 1 at N = 1")
    ap.add_argument("--dyn-diag", default="",
                    help="aux dyn frame slots, diagnosis only (the record check then fails by design): comma list of "
                         "noupdate (no _MeshData rewrite / TLAS refit), nogen (Generate only in each slot's first frame)")
    ap.add_argument("--dyn-adaptive", type=int, default=1,
                    help="aux dyn frame slots: TT_TRACE_ADAPTIVE_ORDER on each slot's primary launch (1, default) or not")
    ap.add_argument("--group-slots", type=int, default=4,
                    help="frames in flight of the library's multi-GPU group leg (aux_group_tiles)")
    ap.add_argument("--no-group", action="store_true", help="skip aux_group_tiles (the tt_group_* library path)")
    ap.add_argument("--group-frames", type=int, default=100,
                    help="timed calls of the group leg (aux_group_tiles; each --batch / --n1-batch frames): many, so "
                         "the children's start skew "
                         "(a file barrier) stays small against the leg's time at N = 8")
    ap.add_argument("--group-timeout", type=float, default=240.0,
                    help="seconds each rank's group-leg child may take before it is killed (aux_group_tiles)")
    ap.add_argument("--aux", default="c3,c4,dyn,refit,c5",
                    help="other BASELINE configs to measure after the metric at N=1 (comma list of c3,c4,dyn,refit,c5;"
                         " '' = none)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            # no launcher: become one (nothing has touched the GPU in this process)
            raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
        if args.gpus is not None and args.gpus < 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus} must be >= 1")
    elif args.gpus is not None and args.gpus != int(env_world):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks; "
                         "refusing to report a measurement for a different GPU count")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("TT_BENCH_LAUNCH_CHECK") == "1":
        # launcher rehearsal (tests/test_bench_launch.py): the rank wiring and a gloo world, no GPU work
        import torch.distributed as dist

        dist.init_process_group(backend="gloo")
        rec = {"rank": rank, "world": world, "dist_world_size": dist.get_world_size(),
               "dist_rank": dist.get_rank(), "local_rank": local_rank,
               "self_launched": os.environ.get("TT_BENCH_SELF_LAUNCHED") == "1"}
        dist.barrier()
        dist.destroy_process_group()
        print(json.dumps(rec), flush=True)
        fail = os.environ.get("TT_BENCH_LAUNCH_CHECK_FAIL_RANK")
        raise SystemExit(3 if fail is not None and int(fail) == rank else 0)
    import torch  # first: tthip must bind to torch's HIP runtime (see tthip.hip_lib)
    import torch.distributed as dist
    import tthip
    import ttdist
    import ttlayout

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (the HIP engine has no CPU fallback)")
    # RCCL ("nccl") over xGMI, one process per GPU. TT_BENCH_DIST_BACKEND=gloo is a rehearsal mode for
    # boxes with fewer GPUs than ranks (ranks share devices, host-side collectives); not a bench mode.
    backend = os.environ.get("TT_BENCH_DIST_BACKEND", "nccl")
    if backend == "nccl" and local_rank >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} (local {local_rank}) needs GPU {local_rank}, but "
                         f"{torch.cuda.device_count()} are visible: one process per GPU")
    gpu = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # ONE stream for torch and the engine, current before anything is allocated or launched
    # the base stream (part 0 / slot 0 of every layout, the aux legs, the N = 1 reference) gets a HW queue of
    # its own too: a pool stream can share its queue with any other stream of the process (RCCL's included)
    stream = tthip.dedicated_stream(torch, dev, -1)
    torch.cuda.set_stream(stream)
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    # TT_BENCH_RCCL_WORLD1=1 (rehearsal, not a bench mode): one rank runs the N > 1 tile path with a
    # real RCCL communicator of size 1 -- the gather on RCCL's own stream beside the part streams
    rccl1 = world == 1 and os.environ.get("TT_BENCH_RCCL_WORLD1") == "1"
    if world > 1 or rccl1:
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend=backend)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: the process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    dist_world = dist.get_world_size() if (world > 1 or rccl1) else None
    tiles = (world > 1 or rccl1) and args.shard in ("tiles", "spp")
    spp = tiles and args.shard == "spp"  # the N-sample frame (weak scaling); "tiles": one frame (strong)
    # frames per launch: --batch for the N > 1 strong-scaling shards, --n1-batch (default 4: a still view accumulating samples; `interactive` reports 1) for the N = 1 frame
    B_batch = max(1, args.batch) if (world > 1 and tiles and not spp) else (max(1, args.n1_batch) if world == 1 else 1)
    W, H = args.width, args.height
    WH = W * H
    far = 1000.0

    # ------------------------------------------------------------------ scene (replicated)
    t0 = time.time()
    blas = tthip.Blas(tthip.Mesh.sponza(args.seed, args.tris))
    am = tthip.AssetManager()
    mats = np.zeros(7, tthip.MAT_DTYPE)
    am.add_parent(blas, None, mats)
    scene = am.build()
    log(f"rank {rank}: scene {len(scene.tris)} tris, {len(scene.nodes)} nodes, build {time.time() - t0:.2f}s")
    eng = tthip.Engine(gpu, stream=stream.cuda_stream)
    assert eng.stream == stream.cuda_stream == torch.cuda.current_stream(dev).cuda_stream != 0, \
        "engine and torch must share one (non-NULL) stream"
    eng.upload(scene)
    # the BASELINE meshes of >= 100k triangles built later (aux configs, C5 tiles) use the GPU BLAS
    # builder (tt_blas_build_device, byte-identical to the host build; tests/test_gpu_builder.py)
    tthip.set_build_engine(eng, min_tris=100_000)

    # ------------------------------------------------------------------ resident rays
    info = torch.zeros(WH * 16, dtype=torch.uint8, device=dev)
    colors = np.zeros(WH, tthip.COL_DTYPE)
    colors["Data"][:, 3] = 1.0  # shade set Data.w = CurBounce + 1 = 1 at bounce 0
    colors_t = torch.from_numpy(colors.view(np.uint8)).to(dev)
    c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, 0.3, far)
    # Primary rays come from the reference's default Generate (RayGenKernels.compute:46-47 with
    # UseReCur = false, RayTracingMaster.cs:189): sub-pixel jitter random(0, pixel_index) - 0.5. The
    # UseReCur variant (no jitter, SURVEY 8(d)'s determinism choice) is measured as aux_recur_unjittered:
    # its screen column x = W/2 has direction.z == -0.0 exactly, whose NaN z slabs make ~1,000 rays
    # walk ~900 nodes each (tools/long_rays.py). The sample layout jitters with frames = rank.
    jitter, frames = 1, (rank if (world > 1 and not tiles) else 0)
    # a rank's pixels (the whole frame at N = 1) as P tile-interleaved parts x F frame slots, each part of
    # each slot traced by its own engine context on its own stream (ttlayout.FrameLayout): a part's launches
    # overlap the other parts' launch drains, and with F >= 2 frame k + 1's primaries overlap frame k's
    # bounce-1 launches. Parts per rank: a full frame's worth of rays (N = 1, and every rank of the spp
    # headline) as 2 parts; the strong-scaling shards (one frame's tiles over N ranks) as --strong-parts x
    # --strong-slots, default 1 x 6 (profiles/r04/replay/r04j_slots46.json).
    P_strong = max(1, args.strong_parts)
    F_strong = max(1, args.strong_slots)
    if args.parts <= 0:
        # N = 1: the whole frame as ONE launch per bounce in the kernel's own tile order, N1_SLOTS frames in
        # flight; the spp headline at N > 1 (a frame's worth of tile units per rank) the same way, so its
        # per-rank work runs in the N = 1 layout and the driver's 1 -> N curve compares like with like
        args.parts = P_strong if (world > 1 and tiles and not spp) else 1
    P = max(1, args.parts) if (tiles or world == 1) else 1
    F = max(1, args.slots if args.slots > 0 else (F_strong if (world > 1 and tiles and not spp) else
                                                  (N1_SLOTS if P == 1 else 1)))
    split = tiles or P > 1
    make_full = ttlayout.full_frame_maker(torch, eng, dev, W, H, c2w, ip, 0.3, far, jitter=jitter)

    def layout_of(plan, slots, batch=1):
        # every frame slot traces its own jittered sample (slot f: sample k + f * S where the plan names
        # sample k, S = the plan's samples), as a renderer's frames in flight do (RayGenKernels.compute:45-46)
        # At N > 1 each slot also cycles through args.cycle samples over its frames (a rare costly ray then recurs
        # in one frame of `cycle` on its slot, not in every frame of it); N = 1 keeps one sample per slot, whose
        # records the oracle check compares.
        n_samples = 1 + max(k for lst in plan for k, _ in lst)
        return ttlayout.FrameLayout(torch, tthip, eng, dev, W, H, far, plan, make_full, slots=slots,
                                    bounce=True, info=True, colors=colors_t, frames=frames, slot_stride=n_samples,
                                    cycle=args.cycle if world > 1 else 1, batch=batch)

    def timed(lay):
        """W untimed steps, then exactly K steps between barrier + synchronize pairs: this rank's seconds."""
        for _ in range(args.warmup):
            lay.step()
        torch.cuda.synchronize(dev)
        lay.timing_reset()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        k0 = lay.k
        t0_ = time.perf_counter()
        for _ in range(args.steps):
            lay.step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el_ = time.perf_counter() - t0_
        lay.timed_rays = lay.rays_in_frames(k0, lay.k)  # the K frames' rays (slots differ with their jitter)
        return el_

    # the strong-scaling deal of tiles to ranks (--deal: LPT by a previous frame's tile costs, or round-robin)
    owner, deal_info = lpt_deal(torch, tthip, ttdist, eng, dev, W, H, c2w, ip, 0.3, far, world, args) \
        if (tiles or args.deal == "lpt") and world > 1 else (None, {"deal": "none (one rank)"})
    if spp:  # this rank's (sample, tile) units of the N-sample frame (ttdist.spp_part_pixels)
        plan = ttdist.spp_part_pixels(W, H, world, rank, P)
    elif split:  # this rank's pixels of the one frame, compacted in tile order, split into P parts
        # (at N > 1 each launch traces `batch` frames of the rank's tiles at once: FrameLayout batch)
        plan = [[(frames + b, pix) for b in range(B_batch)]
                for pix in ttdist.part_pixels(W, H, world, rank, P, owner=owner)]
    else:  # the whole frame, one launch per bounce in the kernel's own tile order
        plan = [[(frames + b, np.arange(WH, dtype=np.int64)) for b in range(B_batch)]]
    layout = layout_of(plan, F, batch=B_batch if ((split and not spp) or world == 1) else 1)
    parts = layout.parts
    n_prim, nb = layout.n_prim(), layout.n_bounce()
    rays_per_step = n_prim + nb
    s_prim, s_bnc = parts[0].s_prim, parts[0].s_bnc
    B_prim = alg_bytes(s_prim, 0, parts[0].n)  # part 0's launches (the engine ring below)
    B_bnc = alg_bytes(s_bnc, 1, parts[0].nb)
    # all parts' launches of a step, averaged over the frame slots (each traces its own jittered sample)
    B_step = sum(alg_bytes(p.s_prim_r[r], 0, p.n) + alg_bytes(p.s_bnc_r[r], 1, p.nb_r[r]) for row in layout.slots
                 for p in row for r in range(layout.R)) / (layout.F * layout.R)
    log(f"rank {rank}: primary {n_prim} rays nodes/ray {s_prim.node_visits / max(parts[0].n, 1):.2f} "
        f"tris/ray {s_prim.tri_tests / max(parts[0].n, 1):.2f} "
        f"hits {s_prim.hits}; bounce {nb} rays nodes/ray {s_bnc.node_visits / max(parts[0].nb, 1):.2f} "
        f"tris/ray {s_bnc.tri_tests / max(parts[0].nb, 1):.2f}; reps_exhausted {s_prim.reps_exhausted + s_bnc.reps_exhausted}"
        f"; parts {P}, frame slots {F}" + (f"; {world}-sample frame (spp)" if spp else ""))

    # N = 1: the records the timed launches write are checked against the oracle afterwards (oracle_check):
    # every slot's hit records and _PrimaryTriangleInfo are poisoned now and the host state kept as the oracle's
    # input -- before the legs below, whose GPU work brings the clocks back up after these host copies
    pre_state = layout.poison_records() if (world == 1 and not args.no_oracle_check) else None

    # The two auxiliary legs that trace the metric's own scene -- the single-stream leg (N = 1) and the
    # sample-sharded layout (N > 1) -- run BEFORE the timed region: they are sustained GPU work, so the
    # timed steps start with the engine clocks settled instead of ramping through the first ~30 ms
    # (profiles/r03/warm/: the same 20-step window reads 0.805-0.816 ms per step straight after setup
    # and 0.783-0.787 once ~40 ms of work has run; the steady-state leg after the region, 0.779).
    # the kernel alone, one launch at a time (N = 1, P > 1): the full frame in the kernel's own tile
    # order on the shared stream, per-launch HIP events -- the per-launch roofline and the launch
    # times rocprofv3 reports for this command's trace kernels
    single = None
    frame_rays, frame_nb = (parts[0].rays, nb) if (P == 1 and world == 1 and layout.B == 1) else (None, None)
    if world == 1 and (P > 1 or F > 1 or frame_rays is None):
        one = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(one, c2w, ip, W, H, 0.3, far, jitter=jitter, frames=frames, max_bounce=1, device=True)
        o_prim = eng.trace(one, WH, 0, far, W, H, info=info, device=True, stats=True)
        onb = eng.enqueue_bounce(one, WH, 0, far, W, H, frames=frames, max_bounce=1, device=True)
        o_bnc = eng.trace(one, onb, 1, far, W, H, info=info, colors=colors_t, device=True, stats=True)
        frame_rays, frame_nb = one, onb
        if not args.no_single:
            launches = [lambda: eng.trace(one, WH, 0, far, W, H, info=info, device=True, asynchronous=True),
                        lambda: eng.trace(one, onb, 1, far, W, H, info=info, colors=colors_t, device=True,
                                          asynchronous=True)]
            oms = timed_launches(eng, launches, args.warmup, args.steps)
            o_avg = float(oms.mean())
            o_ach = ((alg_bytes(o_prim, 0, WH) + alg_bytes(o_bnc, 1, onb)) / 2.0) / (o_avg * 1e-3) / 1e9
            single = {"achieved": round(o_ach, 1), "frac": round(o_ach / HBM_PEAK_GBS, 4),
                      "avg_launch_ms": round(o_avg, 4), "trace_ms_primary": round(float(oms[:, 0].mean()), 4),
                      "trace_ms_bounce": round(float(oms[:, 1].mean()), 4),
                      "mrays_s": round((WH + onb) / float(oms.sum(1).mean()) / 1e3, 2)}
            log(f"single-stream leg (the kernel alone, one launch at a time): {single}")

    # secondary N > 1 layout: every rank traces its own full-frame jittered sample (weak scaling)
    sample_sharded = None
    if tiles:
        srays = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(srays, c2w, ip, W, H, 0.3, far, jitter=1, frames=rank, max_bounce=1, device=True)
        eng.trace(srays, WH, 0, far, W, H, device=True)
        snb = eng.enqueue_bounce(srays, WH, 0, far, W, H, frames=rank, max_bounce=1, device=True)

        def sstep():
            eng.trace(srays, WH, 0, far, W, H, info=info, device=True, asynchronous=True)
            eng.trace(srays, snb, 1, far, W, H, info=info, colors=colors_t, device=True, asynchronous=True)

        for _ in range(args.warmup):
            sstep()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        ts = time.perf_counter()
        for _ in range(args.steps):
            sstep()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        st = torch.tensor([time.perf_counter() - ts, float((WH + snb) * args.steps)], dtype=torch.float64,
                          device=red_dev)
        tmax = st[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        rsum = st[1:].clone()
        dist.all_reduce(rsum, op=dist.ReduceOp.SUM)
        sample_sharded = {"value": round(float(rsum.item()) / float(tmax.item()) / 1e6, 2), "unit": "Mrays/s",
                          "scaling": "weak", "ranks": world,
                          "ms_per_step": round(float(tmax.item()) * 1e3 / args.steps, 4)}
        del srays
        log(f"sample-sharded (weak) layout: {sample_sharded}")

    # N > 1: the N = 1 frame (the whole 1080p frame in the single-GPU headline layout: 2 parts, 1 slot) on
    # every rank's own GPU at once, no collective -- the T(1) of the strong-scaling efficiency below,
    # measured in the same run on the same kind of GPU (the fastest rank's, conservative)
    solo_ms = None
    solo_layouts = {}
    if world > 1 and not args.no_strong:
        # both single-GPU layouts (the whole frame as 2 parts x 1 slot, and as one launch per bounce in the
        # kernel's own order with N1_SLOTS frames in flight -- the N = 1 headline's); t(1) = the faster
        for name, plan_1, slots_1 in (("2x1", [[(0, pix)] for pix in ttdist.part_pixels(W, H, 1, 0, 2)], 1),
                                      (f"1x{N1_SLOTS}", [[(0, np.arange(WH, dtype=np.int64))]], N1_SLOTS)):
            solo = layout_of(plan_1, slots_1)
            el_solo = timed(solo)
            solo.launch_ms()
            solo.close()
            t = torch.tensor([el_solo], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            solo_layouts[name] = round(float(t.item()) * 1e3 / args.steps, 4)
            solo_rays = solo.rays_per_frame()
            del solo
        solo_ms = min(solo_layouts.values())
        log(f"N = 1 frame on each rank's GPU: {solo_layouts} ms per frame (fastest rank)")

    G = layout.attach_gather(dist, world, rank, red_dev) if tiles else None
    # (the gloo rehearsal's host-side collective blocks the host in the copy, so there it serialises)
    gather_overlapped = tiles and red_dev.type == "cuda"
    # N > 1: no per-launch timing markers inside the timed region (at a rank's 1/N shard they cost ~5% of
    # the frame, profiles/r05/events/); the launch times below come from K more steps right after it
    layout.time_none = world > 1
    elapsed = timed(layout)
    if world > 1:
        layout.time_none = False
        layout.timing_reset()
        for _ in range(args.steps):
            layout.step()
        torch.cuda.synchronize(dev)
    lm = layout.launch_ms()  # part 0's launches, the last <= 128 frames of its slot
    launch_ms = lm.reshape(-1)
    total_rays = float(layout.timed_rays)
    rays_per_step = layout.timed_rays / args.steps  # mean over the slots' frames
    trace_ms_rank = float(np.sum(launch_ms)) / (len(launch_ms) // 2)  # part 0's two launches per step
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([total_rays], dtype=torch.float64, device=red_dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        total_rays = float(r.item())
        tr = torch.tensor([trace_ms_rank], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tr, op=dist.ReduceOp.MAX)
        trace_ms_slowest = float(tr.item())
    else:
        trace_ms_slowest = trace_ms_rank

    prim_ms = launch_ms[0::2]
    bnc_ms = launch_ms[1::2]
    avg_ms = float(np.mean(launch_ms))
    if P == 1 and F == 1:  # GB/s per launch, averaged over both launches
        achieved = ((B_prim + B_bnc) / 2.0) / (avg_ms * 1e-3) / 1e9
    else:  # the parts' launches overlap: all of a step's algorithmic bytes over the step's wall time
        achieved = B_step / (elapsed / args.steps) / 1e9

    # the same step for longer, right after the timed region (N = 1): the rate once clocks and caches
    # have settled -- with W = 5, K = 20 the first post-warmup steps run ~2% slower.
    # A secondary field; `value` is always the W/K protocol's measurement above.
    steady = None
    if world == 1 and args.steady_steps > 0:
        torch.cuda.synchronize(dev)
        ks = layout.k
        ts = time.perf_counter()
        for _ in range(args.steady_steps):
            layout.step()
        torch.cuda.synchronize(dev)
        es = time.perf_counter() - ts
        steady = {"steps": args.steady_steps, "ms_per_step": round(es * 1e3 / args.steady_steps, 4),
                  "mrays_s": round(layout.rays_in_frames(ks, layout.k) / es / 1e6, 2),
                  "note": "untimed-for-value: the same step repeated after the timed region"}
        log(f"steady state: {steady}")
    layout.timing_reset()  # drain the rings of the steady steps

    # SURVEY 8(e) parity -- the gathered (N > 1) or the parts' (N = 1) frame(s) must equal one launch
    # tracing each whole frame
    def one_gpu_frame(k):
        one = torch.zeros(WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(one, c2w, ip, W, H, 0.3, far, jitter=jitter, frames=k, max_bounce=1, device=True)
        eng.trace(one, WH, 0, far, W, H, device=True)
        return one.view(WH, 48)[:, 32:48].contiguous().view(torch.int32).cpu().numpy().view(np.uint32)

    gather_parity = None
    if G is not None:
        sizes, gather_list = layout.last_gathered()  # the last step's gather (steady-state steps included)
    if (split or F > 1) and rank == 0:
        last = layout.last_slot()  # the last frame's slot; its samples are layout.last_sample(k)
        r_last = layout.cycle_of(layout.k - 1)
        if spp:
            fr = ttdist.assemble_spp([g[:sum(n)] for g, n in zip(gather_list, sizes)], W, H, world, P)
            gather_parity = all(bool(np.array_equal(fr[k], one_gpu_frame(layout.last_sample(k))))
                                for k in range(world))
            frame = fr[0]
        else:
            if tiles and layout.B > 1:  # every frame of the last batched launch, each against one GPU
                per_frame = split_batched_gather([g[:sum(n)] for g, n in zip(gather_list, sizes)], sizes, layout.B)
                frames_b = [ttdist.assemble_parts(fb, sb, W, H, world, P, owner=owner) for fb, sb in per_frame]
                batch_parity = all(bool(np.array_equal(frames_b[b], one_gpu_frame(layout.last_sample(frames + b))))
                                   for b in range(layout.B))
                frame = frames_b[0]
            elif tiles:
                frame = ttdist.assemble_parts([g[:sum(n)] for g, n in zip(gather_list, sizes)], sizes, W, H, world, P,
                                              owner=owner)
            elif split:
                own = torch.cat([p.prim_hits_r[r_last] for p in layout.slots[last]]).cpu()
                frame = ttdist.assemble_parts([own], [[p.n for p in parts]], W, H, 1, P)
            else:  # one part per slot in the kernel's own order: the last frame's records are in screen order
                # (a batched N = 1 launch: its first frame, the plan's sample `frames`)
                frame = layout.slots[last][0].prim_hits_r[r_last][:WH].contiguous().cpu().numpy().view(np.uint32).reshape(WH, 4)
            gather_parity = bool(np.array_equal(frame, one_gpu_frame(layout.last_sample(frames))))
            if tiles and layout.B > 1:
                gather_parity = gather_parity and batch_parity
        log(f"gathered frame(s): {int((frame[:, 1] != 0xFFFFFFFF).sum())} primary hits of {WH} pixels in sample 0, "
            f"{world if spp else 1} sample(s) identical to single-GPU traces: {gather_parity}")

    # N = 1: every slot's records as the timed (and steady-state) launches left them -- the non-stats
    # tt_trace_kernel<false,false,1|2> instantiations on each slot's own jittered frame -- against the oracle
    # traced from the same poisoned pre-state (tests/oracle_ctypes.py: checker only, never the measured path)
    oracle_check = None
    if pre_state is not None:
        post_state = layout.snapshot()
        oracle_check = oracle_records_check(scene, layout, pre_state, post_state, colors, far, W, H)
        del pre_state, post_state
        log(f"oracle check of the timed records: {oracle_check}")

    # N > 1: the strong-scaling layout -- ONE 1-sample frame's tiles dealt round-robin (P_strong parts x
    # F_strong frame slots per rank), the same per-frame gather; frame time = the slowest rank's; its
    # efficiency against the N = 1 frame measured above on every rank's GPU
    strong = None
    if world > 1 and not args.no_strong:
        if spp:
            lay_s = layout_of([[(0, pix)] for pix in ttdist.part_pixels(W, H, world, rank, P_strong, owner=owner)],
                              F_strong)
            lay_s.attach_gather(dist, world, rank, red_dev)
        else:
            lay_s = layout  # the headline already is the strong-scaling layout
        el_s = timed(lay_s) if lay_s is not layout else elapsed
        if lay_s is not layout:
            lay_s.launch_ms()
        st_ = torch.tensor([el_s, float(lay_s.timed_rays)], dtype=torch.float64, device=red_dev)
        tmax = st_[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        rsum = st_[1:].clone()
        dist.all_reduce(rsum, op=dist.ReduceOp.SUM)
        par = None
        if rank == 0:
            sz_s, gl_s = lay_s.last_gathered()
            per_frame = split_batched_gather([g[:sum(n)] for g, n in zip(gl_s, sz_s)], sz_s, lay_s.B)
            par = all(bool(np.array_equal(ttdist.assemble_parts(fb, sb, W, H, world, lay_s.P, owner=owner),
                                          one_gpu_frame(lay_s.last_sample(b))))
                      for b, (fb, sb) in enumerate(per_frame))
        ms_n = float(tmax.item()) * 1e3 / args.steps / lay_s.B  # per frame (a step traces B frames)
        strong = {"value": round(float(rsum.item()) / float(tmax.item()) / 1e6, 2), "unit": "Mrays/s",
                  "scaling": "strong", "ranks": world, "parts_per_rank": lay_s.P, "frame_slots": lay_s.F,
                  "ms_per_frame": round(ms_n, 4),
                  "rays_per_frame_all_ranks": int(round(float(rsum.item()) / args.steps / lay_s.B)),
                  "frames_per_launch": lay_s.B,
                  "n1_ms_per_frame": round(solo_ms, 4), "n1_rays_per_frame": int(solo_rays),
                  "n1_ms_per_frame_by_layout": solo_layouts,
                  "efficiency": round(solo_ms / (world * ms_n), 4),
                  "gather_identical_to_1gpu": par, "tile_deal": deal_info,
                  "layout": "one 1080p frame (1 sample): 64x64 tiles dealt over the ranks (tile_deal), each rank's tiles "
                            f"as {lay_s.P} parts x {lay_s.F} frame slots (each launch tracing {lay_s.B} frame(s)), + "
                            "one RCCL gather of the frames' primary hit records per step; efficiency = t(N = 1 frame in the faster single-GPU layout, "
                            "every rank's GPU at once, fastest) / (N x t(N))"}
        if lay_s is not layout:
            lay_s.close()
            del lay_s
        log(f"strong-scaling tile layout: {strong}")
    # N = 1 with batched launches: the interactive layout beside the headline -- one frame per launch (any
    # camera: each frame's Generate may take a new pose, RayGenKernels.compute:40-57) x N1_SLOTS frames in flight.
    # The headline's B frames per launch need the next B cameras up front, i.e. a still view accumulating samples.
    interactive = None
    if world == 1 and layout.B > 1:
        lay_i = layout_of([[(frames, np.arange(WH, dtype=np.int64))]], N1_SLOTS)
        el_i = timed(lay_i)
        lay_i.launch_ms()
        ms_i = el_i * 1e3 / args.steps
        interactive = {"value": round(lay_i.timed_rays / el_i / 1e6, 2), "unit": "Mrays/s", "ms_per_frame": round(ms_i, 4),
                       "frames_per_launch": 1, "frame_slots": lay_i.F, "frames_in_flight": lay_i.F,
                       "frame_latency_ms": round(lay_i.F * ms_i, 4), "camera": "per frame (any pose)",
                       "layout": f"the whole 1080p frame, one launch per bounce, {lay_i.F} frames in flight (bench.py "
                                 "--n1-batch 1)"}
        lay_i.close()
        del lay_i
        log(f"interactive layout (1 frame per launch): {interactive}")
    layout.close()  # the borrowing contexts go before any aux leg re-uploads `eng`'s scene

    # N > 1 with the strong-scaling headline: the weak-scaling spp layout beside it (an N-sample frame's
    # (sample, tile) units round-robin, a frame's worth per rank in the N = 1 layout: 1 part x N1_SLOTS
    # slots, the same per-frame gather); value = all ranks' rays / the slowest rank's time
    spp_aux = None
    if world > 1 and tiles and not spp and not args.no_spp_aux:
        lay_w = layout_of(ttdist.spp_part_pixels(W, H, world, rank, 1), N1_SLOTS)
        lay_w.attach_gather(dist, world, rank, red_dev)
        el_w = timed(lay_w)
        lay_w.launch_ms()
        st_w = torch.tensor([el_w, float(lay_w.timed_rays)], dtype=torch.float64, device=red_dev)
        tmax = st_w[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        rsum = st_w[1:].clone()
        dist.all_reduce(rsum, op=dist.ReduceOp.SUM)
        par_w = None
        if rank == 0:
            sz_w, gl_w = lay_w.last_gathered()
            fr_w = ttdist.assemble_spp([g[:sum(n)] for g, n in zip(gl_w, sz_w)], W, H, world, 1)
            par_w = all(bool(np.array_equal(fr_w[k], one_gpu_frame(lay_w.last_sample(k)))) for k in range(world))
        spp_aux = {"value": round(float(rsum.item()) / float(tmax.item()) / 1e6, 2), "unit": "Mrays/s",
                   "scaling": "weak", "ranks": world, "parts_per_rank": lay_w.P, "frame_slots": lay_w.F,
                   "ms_per_step": round(float(tmax.item()) * 1e3 / args.steps, 4),
                   "samples_per_frame": world, "gather_identical_to_1gpu": par_w,
                   "layout": f"{world}-sample 1080p frame (sample k = Generate with frames_accumulated = k), its "
                             f"(sample, 64x64 tile) units round-robin over {world} ranks (a frame's worth each), each "
                             f"rank's units as 1 part x {lay_w.F} frame slots, + one RCCL gather of the primary hit "
                             "records per step"}
        lay_w.close()
        del lay_w
        log(f"spp (weak-scaling) layout: {spp_aux}")

    # ---- auxiliary: the UseReCur ray generation (no jitter), primary + bounce 1, N=1
    recur = None
    if world == 1 and not args.no_recur:
        rr = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)
        eng.generate(rr, c2w, ip, W, H, 0.3, far, jitter=0, frames=0, max_bounce=1, device=True)
        rs = eng.trace(rr, WH, 0, far, W, H, info=info, device=True, stats=True)
        rnb = eng.enqueue_bounce(rr, WH, 0, far, W, H, frames=0, max_bounce=1, device=True)
        launches = [lambda: eng.trace(rr, WH, 0, far, W, H, info=info, device=True, asynchronous=True),
                    lambda: eng.trace(rr, rnb, 1, far, W, H, info=info, colors=colors_t, device=True,
                                      asynchronous=True)]
        rms = timed_launches(eng, launches, args.warmup, args.steps)
        rmean = rms.mean(0)
        recur = {"primary_rays": WH, "bounce_rays": rnb, "trace_ms": [round(float(m), 4) for m in rmean],
                 "mrays_s": round((WH + rnb) / float(rmean.sum()) / 1e3, 1),
                 "primary_nodes_per_ray": round(rs.node_visits / WH, 2), "reps_exhausted": int(rs.reps_exhausted),
                 "note": "RayGenKernels.compute:47 with UseReCur: column x=W/2 has direction.z == -0.0 (NaN z slabs)"}
        # UseReCur's camera rays are the same every frame, so TT_TRACE_ADAPTIVE_ORDER on the primary
        # launch is ordered by exactly its previous frame's costs: the Reps-exhausting chain starts first
        launches[0] = lambda: eng.trace(rr, WH, 0, far, W, H, info=info, device=True, asynchronous=True,
                                        flags=tthip.TT_TRACE_ADAPTIVE_ORDER)
        ams = timed_launches(eng, launches, max(2, args.warmup), args.steps).mean(0)
        recur["adaptive_order"] = {"trace_ms": [round(float(m), 4) for m in ams],
                                   "mrays_s": round((WH + rnb) / float(ams.sum()) / 1e3, 1),
                                   "note": "primary launch flagged (identical camera rays every UseReCur frame)"}
        del rr
        log(f"recur (unjittered) primary + bounce: {recur}")

    # ---- auxiliary (not the metric): any-hit NEE visibility rays (tt_trace_shadow)
    # from this rank's primary hit points toward a point light. Every launch first restores the
    # pristine rays (occluded rays get t = 0 in place) on the shared stream; only the kernel is timed.
    shadow = None
    if not args.no_shadow:
        # the frame's primary hits at N = 1, part 0's at N > 1
        sr = (nee_rays(torch, frame_rays, WH, far, light=(0.0, 9.0, 0.5)) if frame_rays is not None else
              nee_rays(torch, parts[0].rays, parts[0].n, far, light=(0.0, 9.0, 0.5)))
        ns = int(sr.shape[0]) // 48
        work = torch.empty_like(sr)
        work.copy_(sr)
        s_sh = eng.trace_shadow(work, ns, 0, W, H, device=True, stats=True)
        for k in range(args.warmup + args.steps):
            if k == args.warmup:
                eng.timing_reset()
            work.copy_(sr)
            eng.trace_shadow(work, ns, 0, W, H, device=True, asynchronous=True)
        sh_ms = ring_tail(eng, 1, args.steps)[:, 0]
        shadow = {"rays": ns, "trace_ms": round(float(np.mean(sh_ms)), 4),
                  "trace_ms_median": round(float(np.median(sh_ms)), 4),
                  "mrays_s": round(ns / float(np.mean(sh_ms)) / 1e3, 1),
                  "occluded": int(s_sh.hits), "nodes_per_ray": round(s_sh.node_visits / max(ns, 1), 2)}
        log(f"shadow: {ns} NEE rays {shadow['trace_ms']} ms/launch = {shadow['mrays_s']} Mrays/s, "
            f"{shadow['occluded']} occluded")

    # ---- auxiliary: the ray producers around the trace (excluded from the metric):
    # Generate (1080p primary rays) and the diffuse-bounce enqueue with wave-ballot compaction (counter
    # reset + kernel), on a scratch copy of the traced rays restored before every call; engine timing ring.
    producers = None
    if world == 1:  # on the full-frame buffer in the kernel's own order (the parts hold compacted tiles)
        scratch = frame_rays.clone()
        eng.timing_reset()
        for k in range(args.steps):
            eng.generate(scratch, c2w, ip, W, H, 0.3, far, jitter=jitter, frames=frames, max_bounce=1, device=True)
        gen_ms = eng.timing_read()
        eng.timing_reset()
        for k in range(args.steps):
            scratch.copy_(frame_rays)
            eng.enqueue_bounce(scratch, WH, 0, far, W, H, frames=frames, max_bounce=1, device=True)
        enq_ms = eng.timing_read()
        producers = {"generate_ms": round(float(np.median(gen_ms)), 4), "primary_rays": n_prim,
                     "enqueue_compact_ms": round(float(np.median(enq_ms)), 4), "bounce_rays": nb}
        del scratch
        log(f"ray producers: {producers}")

    group = None
    if not args.no_group:
        # every rank takes part (RCCL's init is collective); a failure is reported, never the metric lost
        args._solo_ms = solo_ms
        try:
            group = group_tiles(torch, dist, args, rank, world, backend, red_dev, gpu, W, H)
        except Exception as e:  # noqa: BLE001 — auxiliary
            group = {"error": f"{type(e).__name__}: {e}"}
        log(f"library group path (tt_group_*): {group}")

    aux = None
    if world == 1 and args.aux:
        aux = aux_configs(torch, tthip, eng, dev, args, set(args.aux.split(",")))

    c5t = None
    if world > 1 and not args.no_c5_tiles:
        try:  # failures before the gather are agreed on inside; this catches rank 0's reassembly
            c5t = c5_tiles(torch, dist, tthip, eng, dev, red_dev, args, rank, world)
        except Exception as e:  # noqa: BLE001 — auxiliary, never lose the metric line
            c5t = {"error": f"{type(e).__name__}: {e}"}
            log(f"c5 tiles failed: {e}")


    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ------------------------------------------------------------------ CPU baseline (rank 0, N=1)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the same step workload on the full-frame buffer (the parts' buffers hold compacted tiles)
        if frame_nb != nb:
            log(f"note: full-frame bounce batch {frame_nb} rays, the parts' {nb}")
        cpu = cpu_baseline(scene, frame_rays, WH, WH, frame_nb, colors, far, W, H, args.cpu_seconds)

    # fabric traffic per launch from the round's separate rocprofv3 --pmc pass of this same command
    # (tools/profile_round.sh -> profiles/traffic_latest.json); null when no such pass was committed
    traffic, traffic_src = None, None
    tpath = os.path.join(REPO, "profiles", "traffic_latest.json")
    if os.path.exists(tpath) and (W, H, args.tris) == (1920, 1080, 262267):
        with open(tpath) as f:
            tj = json.load(f)
        traffic = round(float(tj["mean_bytes_per_launch"]))
        traffic_src = "profiles/traffic_latest.json <- " + tj.get("source", "?").split(" ")[0]
        traffic_k = {k.rstrip(">").split(",")[-1].strip(): v["bytes"] for k, v in tj.get("per_kernel", {}).items()
                     if k.startswith("void tt_trace_kernel<false, false,")}
    else:
        traffic_k = {}

    # unit utilisation of the same kernels from the round's separate PMC passes (tools/pmc_units.sh
    # -> profiles/units_latest.json): the binding units, since the scene is cache-resident
    units, units_k, units_src = None, {}, None
    upath = os.path.join(REPO, "profiles", "units_latest.json")
    if os.path.exists(upath) and (W, H, args.tris) == (1920, 1080, 262267):
        with open(upath) as f:
            uj = json.load(f)
        units, units_src = uj.get("mean"), uj.get("source")
        units_k = {k.rstrip(">").split(",")[-1].strip(): v for k, v in uj.get("per_kernel", {}).items()}

    # roofline: the dominant launch (the longer of the primary / bounce-1 launches, one launch at
    # a time: P = F = 1, or the single-stream leg) against the HARD VALU issue bound: every wave64 VALU
    # instruction at its 2-cycle minimum (MI355X_MICROARCH.md, per-instruction constants) on 1024 SIMDs at the
    # 2.4 GHz peak clock, i.e. 1024 x 2.4e9 / (2 x VALU instructions per ray) rays/s -- frac <= 1 by
    # construction. VALU instructions per ray and the unit busy fractions come from the round's PMC passes of
    # the same kernels (tools/pmc_units.sh -> profiles/units_latest.json). Two labelled models sit beside it:
    # the instruction-mix model (each instruction priced at its measured class cost, tools/valu_mix.py) and the
    # quad-cycle model of rounds 1-4 (every instruction at 4 cycles); neither is a bound.
    if P == 1 and F == 1:
        per_launch = {"1": (n_prim, float(np.mean(prim_ms))), "2": (nb, float(np.mean(bnc_ms)))}
    elif single is not None:
        per_launch = {"1": (WH, single["trace_ms_primary"]), "2": (frame_nb, single["trace_ms_bounce"])}
    else:
        per_launch = {}
    CLK, SIMDS = 2.4e9, 1024
    valu = {}
    for info, (n, ms) in per_launch.items():
        u = units_k.get(info, {})
        rate = n / (ms * 1e-3) / 1e9
        ipr = u.get("valu_instr_per_ray")
        hard = SIMDS * CLK / (2.0 * ipr) / 1e9 if ipr else None
        mix_cpi = u.get("mix_cycles_per_instr")
        mix = SIMDS * CLK / (mix_cpi * ipr) / 1e9 if (ipr and mix_cpi) else None
        quad = u.get("valu_ceiling_grays_s")
        # the PMC run's busy fractions of the same kernel: VALU against the 2-cycle issue bound (instructions x 2
        # cycles over 1024 SIMDs x the run's GPU cycles), the texture-data return path (TD) and address path (TA)
        hard_busy = (ipr * u["rays"] * 2.0 / (SIMDS * u["cycles"])) if (ipr and u.get("rays") and u.get("cycles")) else None
        busy = {"valu_2cyc_issue": None if hard_busy is None else round(hard_busy, 3),
                "td": u.get("td_busy"), "ta": u.get("ta_busy"), "valu_quad_cycle_model": u.get("valu_issue_busy")}
        names = {"valu_2cyc_issue": "VALU issue (2-cycle bound)", "td": "TD (texture-data return path)",
                 "ta": "TA (texture-address path)"}
        cand = {k: v for k, v in busy.items() if k in names and v is not None}
        bind = max(cand, key=cand.get) if cand else None
        valu[info] = {"kernel": f"tt_trace_kernel<false,false,{info}>", "rays": int(n), "launch_ms": round(ms, 4),
                      "grays_s": round(rate, 4), "valu_instr_per_ray": ipr,
                      "issue_bound_2cyc_grays_s": None if hard is None else round(hard, 4),
                      "frac": round(rate / hard, 4) if hard else None,
                      "mix_model_grays_s": None if mix is None else round(mix, 4),
                      "frac_mix_model": round(rate / mix, 4) if mix else None,
                      "mix_cycles_per_instr": mix_cpi,
                      "quad_cycle_model_grays_s": quad, "frac_quad_cycle_model": round(rate / quad, 4) if quad else None,
                      "units_busy_pmc": busy,
                      "binding_unit": None if bind is None else {"unit": names[bind], "busy": cand[bind]}}
    dom = max(valu.values(), key=lambda v: v["launch_ms"]) if valu else None
    # the DRAM-side fraction (SURVEY §8(d) consistency warning): the PMC pass's fabric bytes of each launch
    # (2 x FETCH_SIZE + WRITE_SIZE, per the gfx950 correction) over the same launch's HIP-event duration
    dram = {}
    for k, v in valu.items():
        if k in traffic_k:
            gbs = traffic_k[k] / (v["launch_ms"] * 1e-3) / 1e9
            dram[k] = {"kernel": v["kernel"], "traffic_bytes": round(traffic_k[k]), "launch_ms": v["launch_ms"],
                       "gbs": round(gbs, 1), "frac_dram": round(gbs / HBM_PEAK_GBS, 4)}
    dom_dram = dram.get(max(valu, key=lambda k: valu[k]["launch_ms"])) if valu and dram else None

    ms_per_step = elapsed * 1e3 / args.steps
    # the whole step (all parts' / frame slots' launches, overlapped) against the same hard bound: the step's
    # wave64 VALU instructions (rank 0's rays x SQ_INSTS_VALU per ray) at 2 cycles on 1024 SIMDs at 2.4 GHz
    step_valu = None
    i1 = units_k.get("1", {}).get("valu_instr_per_ray")
    i2 = units_k.get("2", {}).get("valu_instr_per_ray")
    if i1 and i2:
        rays1 = sum(p.n for row in layout.slots for p in row) / layout.F
        rays2 = sum(p.nb_r[r] for row in layout.slots for p in row for r in range(layout.R)) / (layout.F * layout.R)
        instr = rays1 * i1 + rays2 * i2
        hard_ms = instr * 2.0 / (SIMDS * CLK) * 1e3
        step_valu = {"issue_bound_2cyc_ms": round(hard_ms, 4), "ms_per_step": round(ms_per_step, 4),
                     "frac": round(hard_ms / ms_per_step, 4), "rays": [round(rays1), round(rays2)],
                     "valu_instr_per_step": round(instr),
                     "achieved_cycles_per_valu_instr": round(CLK * ms_per_step * 1e-3 * SIMDS / instr, 3),
                     "note": "rank 0's step against the hard VALU issue bound (every wave64 VALU instruction at 2 "
                             "cycles, 1024 SIMDs, 2.4 GHz); includes launch gaps and drains"
                             + ("" if world == 1 else " and the gather")}
        m1 = units_k.get("1", {}).get("mix_cycles_per_instr")
        m2 = units_k.get("2", {}).get("mix_cycles_per_instr")
        if m1 and m2:
            mix_ms = (rays1 * i1 * m1 + rays2 * i2 * m2) / (SIMDS * CLK) * 1e3
            step_valu["mix_model"] = {"ms": round(mix_ms, 4), "frac": round(mix_ms / ms_per_step, 4),
                                      "note": "a model, not a bound: each VALU instruction at its class's measured "
                                              "cost (tools/valu_mix.py)"}
    result = {
        "metric": METRIC,
        "value": round(total_rays / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        # the job's scaling mode, the same at every N: spp / sample keep per-GPU work fixed as N grows
        "scaling": "strong" if args.shard == "tiles" else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded Sponza-shaped hall, tools: tt_synth_sponza); primary rays from the reference's "
                "default Generate (jittered, UseReCur=false)",
        "config": {"workload": "sponza_primary_plus_1_bounce_1080p", "scene": "Sponza-shaped CWBVH8 (C2)",
                   "tris": int(len(scene.tris)), "cwbvh_nodes": int(len(scene.nodes)), "width": W, "height": H,
                   "primary_rays": int(n_prim), "bounce_rays": int(nb), "rays_per_step_rank0": int(rays_per_step),
                   "rays_per_step_all_ranks": int(round(total_rays / args.steps)), "frames_per_step": layout.B,
                   # a frame is issued frames_in_flight frames before it completes: its latency is that many frame times
                   "frames_in_flight": layout.B * F,
                   "frame_latency_ms": round(F * ms_per_step, 4),
                   "camera": ("static (progressive accumulation): each launch traces frames_per_step frames of one "
                              "pose, so the next poses must be known ahead; the per-frame layout is `interactive`"
                              if layout.B > 1 else "per frame (any pose)"),
                   "jitter": jitter,
                   "seed": hex(args.seed),
                   "parallelism": ((f"single GPU, full frame as {P} tile-interleaved parts on {P} streams"
                                    if P > 1 else "single GPU, full frame as one launch per bounce in the kernel's "
                                    "own 8x8 tile order")
                                   + (f", {F} frame slots (frames k .. k + {F - 1} in flight on streams with HW queues "
                                      "of their own: each launch's drain overlaps the next frames' launches)"
                                      if F > 1 else "")
                                   + (f"; each launch traces {layout.B} consecutive frames (each its own jittered "
                                      f"sample) as one {W}x{H * layout.B} screen, frame j's PixelIndex + j*W*H "
                                      "(bench.py --n1-batch)" if layout.B > 1 else "") if world == 1 else
                                   ((f"{world}-sample 1080p frame (sample k = Generate with frames_accumulated = k), "
                                     f"its (sample, 64x64 tile) units round-robin over {world} ranks (one frame's "
                                     f"worth each: weak scaling), " if spp else
                                     f"one 1080p frame's 64x64 screen tiles round-robin over {world} ranks, ")
                                    + f"each rank's tiles as {P} "
                                    f"tile-interleaved parts x {F} frame slots on {P * F} streams, + one RCCL gather of the "
                                    f"primary hit records to rank 0 per step (inside the timed step"
                                    + (", overlapped with the bounce-1 trace on a second stream)" if gather_overlapped
                                       else ")") if tiles
                                    else f"sample-sharded x{world} (frames_accumulated=rank), no collective")),
                   "stream": "torch and engine share one stream (a torch ExternalStream on a HW queue of its own); "
                             "per-launch times are HIP events on it"
                             + (f" (part 0 / slot 0 of {P} x {F}: its launches overlap the others')"
                                if P * F > 1 else ""),
                   "parts_per_rank": P, "frame_slots": F, "samples_cycled_per_slot": layout.R,
                   "parts_share_one_scene_copy": P * F > 1,
                   "samples_per_frame": world if spp else 1,
                   "dist_world_size": dist_world, "dist_backend": backend if dist_world else None,
                   "launcher": ("bench.py self-launch" if os.environ.get("TT_BENCH_SELF_LAUNCHED") == "1"
                                else "external (WORLD_SIZE set)" if env_world is not None else "none (1 rank)"),
                   "trace_ms_primary": round(float(np.mean(prim_ms)), 4),
                   "trace_ms_bounce": round(float(np.mean(bnc_ms)), 4),
                   "trace_ms_primary_median": round(float(np.median(prim_ms)), 4),
                   "trace_ms_bounce_median": round(float(np.median(bnc_ms)), 4),
                   "trace_ms_per_step_slowest_rank": round(trace_ms_slowest, 4),
                   "kernel_mrays_s_trace_only": round((parts[0].n + parts[0].nb) / trace_ms_rank / 1e3, 2),
                   "gather_identical_to_1gpu": gather_parity,
                   "steady_state": steady,
                   "aux_strong_tiles": strong, "aux_spp_weak": spp_aux,
                   "aux_sample_sharded": sample_sharded, "aux_recur_unjittered": recur,
                   "aux_shadow_nee": shadow, "aux_ray_producers": producers, "aux_configs": aux,
                   "aux_c5_tiles": c5t, "aux_group_tiles": group},
        "roofline": {"bound": "valu_issue", "unit": "Grays/s",
                     "achieved": dom["grays_s"] if dom else None,
                     "peak": dom["issue_bound_2cyc_grays_s"] if dom else None,
                     "frac": dom["frac"] if dom else None,
                     "kernel": dom["kernel"] if dom else None,
                     "binding_unit": dom["binding_unit"] if dom else None,
                     "units_busy_pmc": dom["units_busy_pmc"] if dom else None,
                     "traffic": traffic,
                     "per_launch": valu,
                     "models": {"node_fetch": node_fetch_model(dom, s_prim, s_bnc, parts),
                                "mix_grays_s": dom["mix_model_grays_s"] if dom else None,
                                "frac_mix": dom["frac_mix_model"] if dom else None,
                                "quad_cycle_grays_s": dom["quad_cycle_model_grays_s"] if dom else None,
                                "frac_quad_cycle": dom["frac_quad_cycle_model"] if dom else None,
                                "note": "models, not bounds: mix = every VALU instruction at its class's measured cost "
                                        "(tools/valu_mix.py: the kernel's ISA x per-block execution counts x "
                                        "profiles/r01_micro_valu_ops.txt); quad_cycle = every instruction at 4 cycles "
                                        "(rounds 1-4's 'ceiling')"},
                     "hbm": {"achieved_alg_gbs": round(achieved, 1), "peak_gbs": HBM_PEAK_GBS,
                             "frac_alg": round(achieved / HBM_PEAK_GBS, 4),
                             "traffic_bytes_per_launch": traffic,
                             "frac_dram": dom_dram["frac_dram"] if dom_dram else None,
                             "dram_per_launch": dram or None,
                             "alg_bytes_per_launch": round((B_prim + B_bnc) / 2.0) if P == 1 else round(B_step / (2 * P)),
                             "alg_bytes_per_step": round(B_step),
                             "note": ("achieved_alg_gbs = algorithmic bytes per trace launch (B_ray, SURVEY §8d) / mean "
                                      "HIP-event launch time" if P == 1 and F == 1 else
                                      f"achieved_alg_gbs = algorithmic bytes (B_ray, SURVEY §8d) of all 2 x {P} trace "
                                      "launches of a step / the step's wall time") + "; the bytes are served mostly "
                                     "from L2 / MALL: traffic = fabric bytes per launch from " + (traffic_src or "no PMC pass")
                                     + " (2 x FETCH_SIZE + WRITE_SIZE, includes Infinity-Cache hits), so HBM does not "
                                     "bind this loop"},
                     "single_stream": single, "step": step_valu,
                     "note": "bound = VALU issue: achieved = rays/s of the dominant launch (one launch at a time, HIP "
                             "events on its stream); peak = the hard issue bound of the same instruction stream = 1024 "
                             "SIMDs x 2.4 GHz / (2 cycles x wave64 VALU instructions per ray), the instructions per ray "
                             "from the PMC pass " + (units_src or "(none)") + " (tools/pmc_units.sh -> "
                             "tools/pmc_units_summary.py -> profiles/units_latest.json); frac <= 1 by construction. "
                             "binding_unit = the busiest of VALU (against the same 2-cycle bound), TD and TA in that PMC "
                             "run"},
        "interactive": interactive,
        "cpu_baseline": cpu,
        "oracle_identical": None if oracle_check is None else oracle_check["identical"],
        "oracle_check": oracle_check,
    }
    print(json.dumps(result), flush=True)
    if world > 1 or rccl1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
