"""Per-launch fabric traffic of the trace kernel from a rocprofv3 --pmc FETCH_SIZE WRITE_SIZE pass
of bench.py (tools/profile_round.sh). Writes a JSON that bench.py reports as roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half of the bytes
of 16-B-per-lane reads (128-B requests tallied at 64 B), so read bytes = 2 x FETCH_SIZE; WRITE_SIZE
is exact for 16-B-per-lane stores. Both count L2 misses served by the Infinity Cache too, so this is
an upper bound on HBM bytes (the C2 scene, ~15 MB, is Infinity-Cache resident)."""
import collections
import csv
import glob
import json
import sys

src, out = sys.argv[1], sys.argv[2]
# one pass per counter (FETCH_SIZE and WRITE_SIZE cannot be collected together on gfx950): average
# each counter per kernel instantiation over its dispatches, then combine per instantiation
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "tt_trace_kernel" not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            vals[k][c].append(v)
if not vals:
    sys.exit("no tt_trace_kernel dispatches found under " + src)
per_kernel = {}
for k, cs in vals.items():
    fetch = sum(cs.get("FETCH_SIZE", [0.0])) / max(1, len(cs.get("FETCH_SIZE", [0.0])))
    write = sum(cs.get("WRITE_SIZE", [0.0])) / max(1, len(cs.get("WRITE_SIZE", [0.0])))
    per_kernel[k] = {"read_bytes": 2.0 * fetch * 1024.0, "write_bytes": write * 1024.0,
                     "bytes": 2.0 * fetch * 1024.0 + write * 1024.0, "dispatches": len(cs.get("FETCH_SIZE", []))}
# bench.py launches the primary and the bounce instantiation equally often
# (the timed launches are the non-STATS closest-hit instantiations; STATS launches run once in setup)
# (<false, false, 1>: primary with _PrimaryTriangleInfo, <false, false, 2>: bounce-1 with the Data.w-gated
# info; the parity check's full-frame <false, false, 0> launch and the aux configs are not the metric's)
timed = {k: v for k, v in per_kernel.items()
         if k.replace(" ", "") in ("voidtt_trace_kernel<false,false,1>", "voidtt_trace_kernel<false,false,2>")}
res = {"file": out.split("/")[-1], "source": src,
       "correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; includes Infinity-Cache hits",
       "per_kernel": per_kernel, "timed_kernels": sorted(timed),
       "mean_bytes_per_launch": sum(v["bytes"] for v in timed.values()) / max(1, len(timed))}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
