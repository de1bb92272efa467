"""ttlayout — how one rank issues its share of a frame's trace launches (bench.py, tools/strong_replay.py).

The reference dispatches kernel_trace once per bounce over the whole screen
(RayTracingMaster.cs:954-1007). A rank here traces its pixels (the whole frame at N = 1, its 64x64
tiles under tile sharding) as

  * P tile-interleaved **parts** (ttdist.part_pixels), each traced by its own engine context on its
    own HIP stream, so one part's launch drain overlaps the other parts' work; and
  * F **frame slots**: frame k runs on slot k % F. Each slot has its own ray, _PrimaryTriangleInfo
    and hit-record buffers and its own streams, so frame k + 1's primary launches (which depend on
    nothing of frame k) run while frame k's bounce-1 launches drain. Inside a frame the order is the
    reference's: a part's bounce-1 launch follows its primary launch on the same stream. With
    ``slot_stride`` s > 0 slot f traces sample k + f s wherever the plan names sample k, so the frames in
    flight carry their own jitter, as a renderer's consecutive frames do (Generate's random(0,
    pixel_index) depends on frames_accumulated, RayGenKernels.compute:45-46); s = 0 replicates one
    sample in every slot. With ``cycle`` R > 1 each slot also cycles through R samples over its
    successive frames (slot f's r-th frame traces sample k + s (f + F (r mod R))), so a rare costly
    ray -- C5's degenerate one -- recurs in one frame of R on its slot instead of in every frame of it.
    With ``batch`` B > 1 each part's plan holds B samples of the same pixels back to back and every launch
    traces all B frames at once: frame b's rays carry PixelIndex + b W H and the launches are issued for a
    screen B times as tall (W x B H), so each frame writes its own _PrimaryTriangleInfo texels (info buffers
    and the GlobalColors copy are B W H) -- fewer, larger launches for the small shards of strong scaling.
    Plan entry b names sample frames + b (with bounce) and every context keys the bounce enqueue's random
    numbers on the frame-local pixel at frames + b (tt_ctx_set_frame_pixels(W H)), so frame b's bounce rays
    are those of its pixels traced alone at its own sample.

All P x F contexts trace ONE scene copy (tt_ctx_share_scene, the base engine lends). Every stream the
layout creates (parts, slots, the gather) sits on a hardware queue of its own (tthip.dedicated_stream:
process-wide streams made with tt_stream_create, reused by every later layout): plain torch streams are dealt round-robin over a process's few HW queues, and two
persistent trace grids on one queue run back to back -- measured on the strong-scaling replay, the
ranks whose second part landed on the base stream's queue took 0.45 instead of 0.25 ms per frame
(profiles/r04/streams/queue_map.txt). TT_LAYOUT_POOL_STREAMS=1 restores torch pool streams (A/B). A step is one
frame: every part's primary launch (writing its 16-B hit records straight into the gather's send
buffer when there is one, tt_trace_closest_hits), the optional gather of those records to rank 0 on a
communication stream, then every part's bounce-1 launch. Bounce-1 rays are the primary hits'
diffuse continuations (tt_enqueue_diffuse_bounce), built once at setup -- the enqueue is the
caller's kernel, not the trace -- and re-traced every frame (the kernel resets every ray's state).
_PrimaryTriangleInfo is written at bounce 0; the bounce-1 form goes to a second buffer (the
reference rebinds the texture to GIWorldPosA at bounce > 0, RayTracingMaster.cs:884).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import numpy as np


class Part:
    """One launch stream of a rank: engine context, stream, its compacted rays and counts."""

    eng = None
    stream = None
    rays = None
    n = 0
    nb = 0
    s_prim = None
    s_bnc = None
    prim_hits = None
    hit_slices: List = []


class FrameLayout:
    """A rank's frame as ``len(plan)`` parts x ``slots`` frame slots (module docstring).

    plan: per part, [(sample k, pixel indices)] -- the rays of sample k (``make_full(k)``: a W*H
    RayData buffer of that sample's Generate) at those pixels, back to back in the part's buffer.
    bounce: trace bounce 1 too (False: primary only, the C5 config).
    lend: the engine whose scene every context traces (slot 0 / part 0 reuses it, on lend's own stream).
    slot_stride: slot f traces sample k + f * slot_stride where the plan names sample k (module docstring)."""

    def __init__(self, torch, tthip, lend, dev, W: int, H: int, far: float, plan, make_full: Callable,
                 slots: int = 1, bounce: bool = True, info: bool = True, colors=None, frames: int = 0,
                 slot_stride: int = 0, cycle: int = 1, batch: int = 1):
        self.torch, self.tthip, self.dev = torch, tthip, dev
        self.W, self.H, self.far = W, H, far
        self.P, self.F = len(plan), max(1, int(slots))
        self.bounce, self.colors, self.frames = bounce, colors, frames
        self.stride = max(0, int(slot_stride))
        self.R = max(1, int(cycle))
        self.B = max(1, int(batch))
        if self.B > 1:
            assert all(len(lst) == self.B for lst in plan), "batch B: every part's plan holds B (sample, pixels) entries"
            # the bounce enqueue draws frame b's random numbers at frames + b (tt_ctx_set_frame_pixels)
            assert not bounce or all(int(k) == frames + b for lst in plan for b, (k, _) in enumerate(lst)), \
                "batch B with bounce: part entry b names sample frames + b"
        self.Hs = H * self.B  # the screen height the launches are issued for (W x B H)
        self.lend = lend
        self.plan = plan
        WH = W * H
        WHs = WH * self.B
        if colors is not None and self.B > 1:
            colors = torch.cat([colors] * self.B)  # GlobalColors of the B-frames-tall screen
            self.colors = colors
        self.engines = []  # (engine, stream) per context, lend's first; contexts created here are closed by close()
        self.own = []
        self.n_streams = 0  # process-wide dedicated streams taken so far (tthip.dedicated_stream)
        self.pool_streams = os.environ.get("TT_LAYOUT_POOL_STREAMS", "0") == "1"
        # per-launch timing (two HIP-event markers around every kernel) only where it is read: part 0 of the
        # slot that traces the first frame after timing_reset (launch_ms), and lend's context (slot 0 / part
        # 0, whose timing the caller owns). On every other context it is off (tt_ctx_set_timing): at a
        # strong-scaled rank's launch sizes the markers cost 15-20% of the frame (profiles/r05/events/).
        # A/B knob: TT_LAYOUT_TIME_ALL=1 keeps it on everywhere.
        self.time_all = os.environ.get("TT_LAYOUT_TIME_ALL", "0") == "1"
        # time_none: no context times anything from the next timing_reset on, lend's included (a caller that
        # keeps the markers out of a timed region and samples launch times afterwards, bench.py at N > 1)
        self.time_none = False
        self.lend_off = False
        self.slots: List[List[Part]] = []
        # slot 0 / part 0 issues on lend's own stream: the gather orders against p.stream, so it must be
        # the stream lend's launches actually go to (not whatever stream torch has current)
        cur = torch.cuda.current_stream(dev)
        base_stream = cur if cur.cuda_stream == lend.stream else torch.cuda.ExternalStream(lend.stream, device=dev)
        self.info0 = [torch.zeros(WHs * 16, dtype=torch.uint8, device=dev) if info else None for _ in range(self.F)]
        self.info1 = [torch.zeros(WHs * 16, dtype=torch.uint8, device=dev) if (info and bounce) else None
                      for _ in range(self.F)]
        for f in range(self.F):
            row = []
            for s, lst in enumerate(plan):
                p = Part()
                if f == 0 and s == 0:
                    p.eng, p.stream = lend, base_stream
                else:
                    st = self.new_stream()
                    e = tthip.Engine(dev.index, stream=st.cuda_stream)
                    e.share_scene(lend)  # ONE scene copy: one cache footprint for all contexts
                    if not self.time_all:
                        e.set_timing(False)
                    self.own.append(e)
                    p.eng, p.stream = e, st
                if self.B > 1:  # frame b's bounce random numbers: its own pixel at frames + b
                    p.eng.set_frame_pixels(WH)
                p.n = int(sum(len(pix) for _, pix in lst))
                # GlobalRays ping-pong: bounce-1 rays live at [W*H, W*H + nb) (odd bounces, the API's offset);
                # one buffer per sample the slot cycles through
                p.rays_r = [torch.zeros(((WHs + p.n) if bounce else max(p.n, 1)) * 48, dtype=torch.uint8, device=dev)
                            for _ in range(self.R)]
                p.rays = p.rays_r[0]
                row.append(p)
            self.slots.append(row)
        # fill the parts' primary rays, sample by sample (slot f, cycle r: the plan's sample k is
        # sample_of(f, k, r))
        fr = [(f, r) for f in range(self.F) for r in range(self.R)]
        for k in sorted({self.sample_of(f, kk, r) for f, r in fr for lst in plan for kk, _ in lst}):
            full = make_full(k)
            for f, r in fr:
                for p, lst in zip(self.slots[f], plan):
                    o = 0
                    for j, (kk, pix) in enumerate(lst):
                        if self.sample_of(f, kk, r) == k and len(pix):
                            seg = p.rays_r[r].view(-1, 48)[o:o + len(pix)]
                            seg[:] = full.view(WH, 48)[torch.from_numpy(pix).to(dev)]
                            if self.B > 1 and j:  # frame j of the batch: PixelIndex + j W H
                                pi = seg[:, 12:16].contiguous().view(torch.int32).view(-1) + j * WH
                                seg[:, 12:16] = pi.view(torch.uint8).view(-1, 4)
                        o += len(pix)
            del full
        torch.cuda.synchronize(dev)
        # setup: one stats trace per bounce (part counters) and the bounce-1 enqueue, per slot and cycle sample
        for f, row in enumerate(self.slots):
            for p in row:
                p.s_prim_r, p.nb_r, p.s_bnc_r, p.prim_hits_r = [], [], [], []
                for r in range(self.R):
                    rays = p.rays_r[r]
                    Hs = self.Hs
                    p.s_prim_r.append(p.eng.trace(rays, p.n, 0, far, W, Hs, info=self.info0[f], device=True,
                                                  stats=True))
                    if bounce:  # (the bounce direction's hash seed: the slot's sample, as Generate's)
                        p.nb_r.append(p.eng.enqueue_bounce(rays, p.n, 0, far, W, Hs, frames=self.sample_of(f, frames, r),
                                                           max_bounce=1, device=True))
                        p.s_bnc_r.append(p.eng.trace(rays, p.nb_r[-1], 1, far, W, Hs, info=self.info1[f], colors=colors,
                                                     device=True, stats=True))
                    else:
                        p.nb_r.append(0)
                        p.s_bnc_r.append(None)
                    p.prim_hits_r.append(rays[: p.n * 48].view(p.n, 48)[:, 32:48].view(torch.int32))
                p.s_prim, p.nb, p.s_bnc, p.prim_hits = p.s_prim_r[0], p.nb_r[0], p.s_bnc_r[0], p.prim_hits_r[0]
                p.hit_slices = []
        torch.cuda.synchronize(dev)
        self.gather = None
        self.k = 0
        self.k_reset = 0

    def new_stream(self):
        """A launch stream on its own HW queue (module docstring); a torch pool stream under the A/B knob."""
        if self.pool_streams:
            return self.torch.cuda.Stream(self.dev)
        st = self.tthip.dedicated_stream(self.torch, self.dev, self.n_streams)
        self.n_streams += 1
        return st

    # ---------------------------------------------------------------- sizes
    def sample_of(self, f: int, k: int, r: int = 0) -> int:
        """The sample slot f traces in its cycle position r where the plan names sample k."""
        return int(k) + self.stride * (int(f) + self.F * (int(r) % self.R))

    def cycle_of(self, k: int) -> int:
        """The cycle position of frame k (its slot's (k // F)-th frame)."""
        return (int(k) // self.F) % self.R

    def frame_sample(self, k: int, kk: int) -> int:
        """The sample frame k traces where the plan names sample kk."""
        return self.sample_of(int(k) % self.F, kk, self.cycle_of(k))

    def last_sample(self, kk: int) -> int:
        """The sample the most recent frame traced where the plan names sample kk."""
        return self.frame_sample(self.k - 1, kk)

    @property
    def parts(self) -> List[Part]:
        """Slot 0's parts (with slot_stride > 0 the other slots trace other samples: rays_in_frames)."""
        return self.slots[0]

    def rays_per_frame(self) -> int:
        """Slot 0's rays per frame (primary + bounce 1)."""
        return int(sum(p.n + p.nb for p in self.parts))

    def rays_of_slot(self, f: int, r: int = 0) -> int:
        return int(sum(p.n + p.nb_r[r] for p in self.slots[f]))

    def rays_in_frames(self, k0: int, k1: int) -> int:
        """Rays traced by frames k0 .. k1 - 1 (frame k on slot k % F, cycle position cycle_of(k))."""
        return int(sum(self.rays_of_slot(k % self.F, self.cycle_of(k)) for k in range(k0, k1)))

    def last_slot(self) -> int:
        """The slot of the most recent frame."""
        return (self.k - 1) % self.F

    def n_prim(self) -> int:
        return int(sum(p.n for p in self.parts))

    def n_bounce(self) -> int:
        return int(sum(p.nb for p in self.parts))

    # ---------------------------------------------------------------- gather
    def attach_gather(self, dist, world: int, rank: int, red_dev):
        """The per-frame gather of the primary hit records to rank 0 (RCCL on the GPU, gloo rehearsals on
        the host). Shards are padded to the largest so every rank sends one equal-size message; a rank's
        parts back to back. On the GPU the primary traces write their records straight into the slot's
        send buffer (tt_trace_closest_hits); two send buffers per slot alternate, so a slot's next frame
        waits only for the gather two frames back. The gloo form copies the records to a host buffer."""
        torch = self.torch
        g = _Gather()
        n_t = torch.tensor([p.n for p in self.parts], dtype=torch.int64, device=red_dev)
        sz = [torch.zeros_like(n_t) for _ in range(world)]
        dist.all_gather(sz, n_t)
        g.dist, g.world, g.rank = dist, world, rank
        g.sizes = [[int(v) for v in x.tolist()] for x in sz]
        g.stream_hits = red_dev.type == "cuda"
        g.nbuf = 2 * self.F if g.stream_hits else 1
        m = max(sum(x) for x in g.sizes)
        g.bufs = [torch.zeros((m, 4), dtype=torch.int32, device=red_dev) for _ in range(g.nbuf)]
        g.lists = [[torch.empty_like(bf) for _ in range(world)] if rank == 0 else None for bf in g.bufs]
        g.comm = self.new_stream()
        g.done = [torch.cuda.Event() for _ in range(g.nbuf)]
        g.used = [False] * g.nbuf
        g.copied = torch.cuda.Event()
        g.last = None
        o = 0
        for s in range(self.P):
            n = self.parts[s].n
            for row in self.slots:
                row[s].hit_slices = [bf[o:o + n] for bf in g.bufs]
            o += n
        self.gather = g
        return g

    def last_gathered(self):
        """(sizes, per-rank gathered blocks) of the most recent frame's gather (rank 0)."""
        g = self.gather
        return g.sizes, g.lists[g.last]

    # ---------------------------------------------------------------- one frame
    def step(self):
        k = self.k
        self.k += 1
        f = k % self.F
        r = self.cycle_of(k)
        row = self.slots[f]
        g = self.gather
        W, H, far = self.W, self.Hs, self.far
        b = (f + self.F * ((k // self.F) % 2)) % g.nbuf if g is not None else 0
        for p in row:
            if g is not None and g.stream_hits:
                if g.used[b]:
                    p.stream.wait_event(g.done[b])  # the gather that last read send buffer b is done
                p.eng.trace(p.rays_r[r], p.n, 0, far, W, H, info=self.info0[f], device=True, asynchronous=True,
                            hits_out=p.hit_slices[b])
            else:
                p.eng.trace(p.rays_r[r], p.n, 0, far, W, H, info=self.info0[f], device=True, asynchronous=True)
        if g is not None:
            torch = self.torch
            for p in row:
                g.comm.wait_stream(p.stream)  # this frame's primary hit records are final
            with torch.cuda.stream(g.comm):
                if not g.stream_hits:
                    for p in row:
                        p.hit_slices[0].copy_(p.prim_hits_r[r])
                    g.copied.record(g.comm)
                g.dist.gather(g.bufs[b], g.lists[b], dst=0)
                if g.stream_hits:
                    g.done[b].record(g.comm)
                    g.used[b] = True
            g.last = b
        if self.bounce:
            for p in row:
                p.eng.trace(p.rays_r[r], p.nb_r[r], 1, far, W, H, info=self.info1[f], colors=self.colors, device=True,
                            asynchronous=True)
        if g is not None and not g.stream_hits:
            for p in row:
                # the next primary trace rewrites the records copied out above: it waits for the copy
                p.stream.wait_event(g.copied)

    def streams(self):
        return [p.stream for row in self.slots for p in row]

    # ---------------------------------------------------------------- record checks (bench.py's oracle leg)
    POISON = 0xA5

    def poison_records(self):
        """Fills every slot's hit records (RayData.hits of its primary and bounce-1 rays) and its
        _PrimaryTriangleInfo buffers with the byte POISON, so that a record the following launches do not
        write stays visible, and returns host copies of that state (snapshot()). (cycle 1 layouts only; a
        batch's bounce-1 rays sit at W x B H, the ping-pong offset of its B-tall screen)"""
        assert self.R == 1, "record checks need cycle 1"
        WH = self.W * self.Hs
        for f, row in enumerate(self.slots):
            for p in row:
                v = p.rays.view(-1, 48)
                v[: p.n, 32:48] = self.POISON
                if self.bounce and p.nb:
                    v[WH: WH + p.nb, 32:48] = self.POISON
            for b in (self.info0[f], self.info1[f]):
                if b is not None:
                    b.fill_(self.POISON)
        self.torch.cuda.synchronize(self.dev)
        return self.snapshot()

    def snapshot(self):
        """Host copies per slot: {"rays": [per part uint8 array], "info0": array or None, "info1": ...}."""
        self.torch.cuda.synchronize(self.dev)
        return [{"rays": [p.rays.cpu().numpy() for p in row],
                 "info0": None if self.info0[f] is None else self.info0[f].cpu().numpy(),
                 "info1": None if self.info1[f] is None else self.info1[f].cpu().numpy()}
                for f, row in enumerate(self.slots)]

    def timed(self, f: int, s: int) -> bool:
        """Whether slot f / part s records per-launch times (see __init__)."""
        if self.time_none:
            return False
        return self.time_all or (f, s) in ((0, 0), (self.k_reset % self.F, 0))

    def timing_reset(self):
        self.k_reset = self.k
        for f, row in enumerate(self.slots):
            for s, p in enumerate(row):
                if not (f == 0 and s == 0) or self.time_none or self.lend_off:
                    # (lend's own setting is the caller's, except while time_none turned it off)
                    p.eng.set_timing(self.timed(f, s))
                p.eng.timing_reset()
        self.lend_off = self.time_none

    def launch_ms(self, ring: int = 256) -> Optional[np.ndarray]:
        """Part 0's per-launch HIP-event times of the last frames its slot traced since timing_reset
        (rows: frames, columns: primary[, bounce-1]) -- the slot of the first frame after timing_reset
        (under TT_LAYOUT_TIME_ALL=1: the first slot that traced one); every timed context's ring is drained."""
        per = 2 if self.bounce else 1
        out = None
        first = self.k_reset % self.F
        for f in [first] + [g for g in range(self.F) if g != first]:
            row = self.slots[f]
            mine = sum(1 for k in range(self.k_reset, self.k) if k % self.F == f)
            for s, p in enumerate(row):
                if not self.timed(f, s):
                    continue
                ms = np.asarray(p.eng.timing_read(), np.float64)
                rows = min(mine, ring // per)
                assert len(ms) == rows * per, (len(ms), rows, per)
                if s == 0 and out is None and rows > 0:
                    out = ms.reshape(rows, per)
        return out

    def close(self):
        for e in self.own:
            e.close()
        self.own = []
        if self.B > 1 and self.lend is not None:
            self.lend.set_frame_pixels(0)  # lend's context back to the reference's form
            self.lend = None
        if self.gather is not None:
            self.gather.comm = None


class _Gather:
    pass


def full_frame_maker(torch, eng, dev, W: int, H: int, c2w, ip, near: float, far: float, jitter: int = 1,
                     max_bounce: int = 1):
    """make_full for FrameLayout: sample k's primary rays (the reference's Generate with
    frames_accumulated = k) in a fresh W*H RayData buffer."""

    def make(k: int):
        full = torch.zeros(W * H * 48, dtype=torch.uint8, device=dev)
        eng.generate(full, c2w, ip, W, H, near, far, jitter=jitter, frames=k, max_bounce=max_bounce, device=True)
        return full

    return make
