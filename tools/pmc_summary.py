"""Summarizes rocprofv3 counter CSVs (one dir per pass) for the trace kernel dispatches:
per-kernel-instantiation mean of each counter over dispatches, plus derived per-wave ratios."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcq"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/*/*_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "tt_trace" not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(m):
        print(f"  {c:24s} {m[c]:16.0f}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"):
            if c in m:
                print(f"  {c}/WAVE_CYCLES = {m[c] / wc:.3f}")
