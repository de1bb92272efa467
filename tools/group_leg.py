#!/usr/bin/env python3
"""One rank of bench.py's `aux_group_tiles` leg: the library's multi-GPU group (tt_group_*, csrc/tt_group.hip)
measured in a CHILD process of each bench rank, so that nothing this leg does -- its own RCCL communicator
(ncclCommInitRank inside the library), its gathers -- can stall the bench's own ranks: each parent waits for
its child with a time limit and reports a failure instead of hanging (bench.py group_tiles).

The children meet through files in --dir (all ranks run on one node): rank 0 writes the 128-byte RCCL id
(tt_group_unique_id) to dir/uid, the others read it; `dir/ready_<rank>` files form the barrier before the timed
frames. Each child: builds the bench scene (the same seeded Sponza-shaped C2 buffers), creates its group member
(tt_group_create_rank on --device), uploads, traces one synchronous frame per cycled sample to learn its ray
counts (the bounce-1 count lives on the device), runs --warmup frames, waits at the barrier, times --steps
asynchronous frames (frame k = sample k mod --cycle, --slots frames in flight), and prints ONE JSON line:
{"elapsed_s", "host_s": the enqueue loop alone, "rays_per_sample": this rank's primary + bounce-1 rays per sample, "parity": rank 0 only -- the
last frame's gathered screen-order records against one context tracing that whole frame}."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def wait_for(path, seconds):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > seconds:
            raise TimeoutError(f"{path} did not appear within {seconds} s")
        time.sleep(0.0002)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--dir", required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--cycle", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1, help="frames per call (tt_group_config.batch)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tris", type=int, default=262267)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x53504F4E)
    a = ap.parse_args()

    import numpy as np
    import torch  # (tthip binds to torch's HIP runtime)
    import tthip

    torch.cuda.set_device(a.device)
    dev = torch.device("cuda", a.device)
    W, H, far, near = a.width, a.height, 1000.0, 0.3
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.sponza(a.seed, a.tris)), None, np.zeros(7, tthip.MAT_DTYPE))
    scene = am.build()
    c2w, ip = tthip.unity_camera((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H, near, far)

    uid_path = os.path.join(a.dir, "uid")
    if a.rank == 0:
        uid = tthip.group_unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(uid_path + ".tmp", uid_path)
    else:
        wait_for(uid_path, 60)
        uid = open(uid_path, "rb").read()
    S, R, B = max(1, a.slots), max(1, a.cycle), max(1, a.batch)
    g = tthip.Group(W, H, rank=a.rank, world=a.world, uid=uid, device=a.device, slots=S, bounce=True, batch=B)
    try:
        g.upload(scene)
        outs = [torch.zeros((B * W * H, 4), dtype=torch.int32, device=dev) for _ in range(S)] if a.rank == 0 else [None] * S
        torch.cuda.synchronize(dev)
        mine = []
        # call k traces samples B (k mod R) .. B (k mod R) + B - 1
        for k in range(R):
            g.trace_frame(outs[0], c2w, ip, near, far, jitter=1, frames=B * k, max_bounce=1)
            n_p, n_b, _ = g.frame_rays(0)
            mine.append(int(n_p + n_b))
        for k in range(a.warmup):
            g.trace_frame(outs[k % S], c2w, ip, near, far, jitter=1, frames=B * (k % R), max_bounce=1, asynchronous=True)
        g.sync()
        open(os.path.join(a.dir, f"ready_{a.rank}"), "w").close()
        for r in range(a.world):
            wait_for(os.path.join(a.dir, f"ready_{r}"), 120)
        t0 = time.perf_counter()
        for k in range(a.steps):
            g.trace_frame(outs[k % S], c2w, ip, near, far, jitter=1, frames=B * (k % R), max_bounce=1, asynchronous=True)
        host = time.perf_counter() - t0  # the host's enqueue time of all calls (the device may still be busy)
        g.sync()
        el = time.perf_counter() - t0
        parity = None
        if a.rank == 0:
            k = a.steps - 1  # the last call's last frame: sample B (k mod R) + B - 1
            got = outs[k % S][(B - 1) * W * H:].cpu().numpy().view(np.uint32)
            eng = tthip.Engine(a.device)
            try:
                eng.upload(scene)
                one = torch.zeros(W * H * 48, dtype=torch.uint8, device=dev)
                eng.generate(one, c2w, ip, W, H, near, far, jitter=1, frames=B * (k % R) + B - 1, max_bounce=1,
                             device=True)
                eng.trace(one, W * H, 0, far, W, H, device=True)
                ref = one.view(W * H, 48)[:, 32:48].contiguous().view(torch.int32).cpu().numpy().view(np.uint32)
                parity = bool(np.array_equal(got, ref))
            finally:
                eng.close()
        print(json.dumps({"elapsed_s": el, "host_s": host, "rays_per_sample": mine, "parity": parity}), flush=True)
    finally:
        g.close()


if __name__ == "__main__":
    main()
