#!/usr/bin/env python3
"""Strong-scaling prediction on ONE GPU (VERDICT r3 "Next 1"): replays, one rank at a
time, exactly the launches every rank of an N-GPU strong-scaling run issues -- its 64x64 round-robin
tiles (dealt round-robin, or longest-processing-time first by sample 0's tile costs with --deal lpt) as P
tile-interleaved parts x F frame slots, every slot its own jittered sample (ttlayout.FrameLayout, the layout
bench.py runs for the N > 1 headline / aux_c5_tiles) -- and predicts

    t(N)   = max over ranks r of rank r's frame time (ms per frame, frames back to back)
    eff(N) = t(1) / (N * t(N)),   t(1) = the whole frame in the N = 1 layout (2 parts, 1 slot)

The per-frame RCCL gather of the hit records is not replayed (it runs on its own stream beside the
traces; bench.py measures it on a real node). Configs: C2 (Sponza-shaped 1080p, primary + bounce 1)
and C5 (San-Miguel-shaped 4K, primary only). Output: one JSON document on stdout (commit it under
profiles/). Usage: tools/strong_replay.py [--configs c2,c5] [--parts 1] [--slots 6] [--layouts PxF,...] [--steps 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c5")
    ap.add_argument("--slots", type=int, default=6, help="frame slots per rank (bench.py --strong-slots)")
    ap.add_argument("--parts", type=int, default=1, help="parts per rank at N > 1 (bench.py --strong-parts)")
    ap.add_argument("--layouts", default=None,
                    help="comma list of PxF layouts to replay at every N > 1 instead of (parts, --slots), e.g. 3x1,1x3")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--ranks", default="all", help="'all' or a comma list of ranks to replay per N")
    ap.add_argument("--tile", type=int, default=64, help="screen tile edge of the round-robin sharding")
    ap.add_argument("--n1-slots", type=int, default=3, help="frame slots of the N = 1 one-launch reference")
    ap.add_argument("--deal", choices=["rr", "lpt"], default="rr",
                    help="tile deal at N > 1: rr (round-robin, bench.py's default) or lpt (longest-processing-time first "
                         "by sample 0's tile costs, tt_trace_chunk_costs)")
    ap.add_argument("--batch", type=int, default=4,
                    help="B frames of a rank's shard in each launch, as bench.py --batch (N > 1 rows; "
                         "ms per frame = ms per step / B; FrameLayout batch: each frame its own texels)")
    ap.add_argument("--n1-batched", action="store_true",
                    help="also replay the N > 1 rows' layout (--parts x --slots, --batch frames per launch) at N = 1, the "
                         "whole frame as one rank's shard, as a candidate for t(1): efficiency then credits batching "
                         "only with what it gains over batching one GPU")
    ap.add_argument("--cycle", type=int, default=6,
                    help="samples each slot cycles through (bench.py --cycle, its N > 1 layouts); 1: one per slot")
    ap.add_argument("--slot-stride", type=int, default=1,
                    help="slot f traces sample f * stride (bench.py: 1, every frame in flight its own jitter; 0: one "
                         "sample replicated in every slot, rounds 1-4)")
    args = ap.parse_args()
    import torch
    import tthip
    import ttconfigs as T
    import ttdist
    import ttlayout

    dev = torch.device("cuda", 0)
    stream = tthip.dedicated_stream(torch, dev, -1)  # the base stream: a HW queue of its own, as bench.py's
    torch.cuda.set_stream(stream)
    eng = tthip.Engine(0, stream=stream.cuda_stream)
    tthip.set_build_engine(eng, min_tris=100_000)
    out = {"tool": "tools/strong_replay.py", "device": torch.cuda.get_device_name(0), "slots": args.slots,
           "cycle": args.cycle,
           "tile": args.tile, "steps": args.steps, "deal": args.deal, "slot_stride": args.slot_stride, "configs": {}}

    def frame_ms(lay):
        # as bench.py at N > 1: no per-launch timing markers in the timed frames (tt_ctx_set_timing)
        lay.time_none = not os.environ.get("TT_REPLAY_TIMED_SLOT")
        for _ in range(args.warmup):
            lay.step()
        torch.cuda.synchronize(dev)
        lay.timing_reset()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lay.step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        lay.launch_ms()
        return ms

    def run(name, scene, view, W, H, bounce):
        eng.upload(scene)
        c2w, ip = view.camera(W, H)
        make_full = ttlayout.full_frame_maker(torch, eng, dev, W, H, c2w, ip, T.NEAR, T.FAR)
        colors = None
        if bounce:
            col = np.zeros(W * H, tthip.COL_DTYPE)
            col["Data"][:, 3] = 1.0
            colors = torch.from_numpy(col.view(np.uint8)).to(dev)
        rows = []
        t1 = None
        chunk = None
        if args.deal == "lpt":  # sample 0's per-8x8-chunk costs (the bench's deal input), once per config
            full = make_full(0)
            eng.trace(full, W * H, 0, T.FAR, W, H, device=True, flags=tthip.TT_TRACE_ADAPTIVE_ORDER)
            chunk = eng.chunk_costs(0)
            del full
        for n in [int(x) for x in args.ns.split(",")]:
            if n == 1:  # the reference: both single-GPU layouts (2 parts x 1 slot; the whole frame as one launch in
                # the kernel's own order with --n1-slots frames in flight, bench.py's N = 1 headline); t(1) = the faster
                layouts = [(2, 1, 1), (0, args.n1_slots, 1)]
                if args.n1_batched:
                    layouts.append((args.parts, args.slots, max(1, args.batch)))
            elif args.layouts:
                layouts = [tuple(int(v) for v in l.split("x")) + (max(1, args.batch),) for l in args.layouts.split(",")]
            else:
                layouts = [(args.parts, args.slots, max(1, args.batch))]
            ranks = range(n) if args.ranks == "all" else [int(r) for r in args.ranks.split(",") if int(r) < n]
            owner = ttdist.lpt_owner(ttdist.tile_costs_from_chunks(chunk, W, H, args.tile), n) \
                if (chunk is not None and n > 1) else None
            for P, F, B in layouts:
                per = []
                B = B if P > 0 else 1  # frames per launch (N > 1 rows, and the --n1-batched N = 1 row)
                for r in ranks:
                    plan = ([[(0, np.arange(W * H, dtype=np.int64))]] if P == 0 else  # P = 0: native whole frame
                            [[(b, pix) for b in range(B)]
                             for pix in ttdist.part_pixels(W, H, n, r, P, args.tile, owner=owner)])
                    lay = ttlayout.FrameLayout(torch, tthip, eng, dev, W, H, T.FAR, plan, make_full,
                                               slots=F, bounce=bounce, info=True, colors=colors,
                                               slot_stride=args.slot_stride * B, cycle=args.cycle, batch=B)
                    ms = frame_ms(lay) / B
                    per.append({"rank": r, "rays": lay.rays_per_frame(), "ms_per_frame": round(ms, 4)})
                    lay.close()
                    del lay
                    print(f"[replay] {name} N={n} {P}x{F} rank {r}: {per[-1]}", file=sys.stderr, flush=True)
                t_n = max(p["ms_per_frame"] for p in per)
                if n == 1:
                    t1 = t_n if t1 is None else min(t1, t_n)
                rows.append({"n_gpus": n, "parts_per_rank": P, "frame_slots": F, "frames_per_launch": B, "ranks": per,
                             "deal": "lpt" if owner is not None else "round-robin",
                             "t_frame_ms_slowest_rank": t_n,
                             "predicted_efficiency": round(t1 / (n * t_n), 3) if t1 else None,
                             "predicted_frame_mrays_s": round(sum(p["rays"] for p in per) / t_n / 1e3, 1)
                             if args.ranks == "all" else None})
        out["configs"][name] = {"width": W, "height": H, "tris": int(len(scene.tris)), "rows": rows}

    which = set(args.configs.split(","))
    if "c2" in which:
        run("c2_sponza_1080p_primary_plus_bounce1", T.c2_sponza(), T.C2_VIEW, 1920, 1080, True)
    if "c5" in which:
        t0 = time.time()
        sc = T.c5_san_miguel()
        print(f"[replay] c5 build {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        run("c5_san_miguel_4k_primary", sc, T.C5_VIEW, 3840, 2160, False)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
