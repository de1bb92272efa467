#!/usr/bin/env python3
"""How the library group (tt_group_*) behaves as a rank's shard shrinks, on one GPU: tools/group_leg.py at world 1
(whole frames through the RCCL self-gather) for screens of 1, 1/4 and 1/8 of 1080p, one or four frames per call (tt_group_config.batch) -- the pixels one rank of an
N = 1 / 4 / 8 node traces -- and per frame-slot count. A rank at N = 8 also receives nothing but its own share, so
this isolates the per-frame fixed costs (host_ms_per_call: the enqueue alone) (launches, the host's enqueue of a frame, the RCCL group call) that decide
the group's strong scaling. Prints one JSON line per configuration: ms per frame, Mrays/s."""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 200
configs = [tuple(int(x) for x in c.split("x")) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
    [(h, b, sl) for h in (1080, 272, 136) for b in (1, 4) for sl in (2, 4)]
for height, batch, slots in configs:
    d = tempfile.mkdtemp(prefix="tt_group_scale_")
    # TT_GROUP_FORCE_GATHER: keep the RCCL self-gather + scatter a one-rank group would skip, as an N-GPU rank has them
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "group_leg.py"), "--rank", "0", "--world", "1",
                        "--device", "0", "--dir", d, "--steps", str(frames), "--warmup", "10", "--slots", str(slots),
                        "--cycle", "4", "--batch", str(batch), "--height", str(height)], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, TT_GROUP_FORCE_GATHER="1"))
    if r.returncode != 0:
        print(json.dumps({"height": height, "batch": batch, "slots": slots, "error": r.stderr[-400:]}), flush=True)
        sys.exit(r.returncode)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    rays = sum(res["rays_per_sample"][k % 4] for k in range(frames))
    print(json.dumps({"width": 1920, "height": height, "batch": batch, "slots": slots, "calls": frames,
                      "ms_per_frame": round(res["elapsed_s"] * 1e3 / (frames * batch), 4),
                      "host_ms_per_call": round(res["host_s"] * 1e3 / frames, 4),
                      "mrays_s": round(rays / res["elapsed_s"] / 1e6, 1), "parity": res["parity"]}), flush=True)
