"""Per-ray SQ instruction counts of the bench's trace kernels from rocprofv3 --pmc passes of
`bench.py --parts 1` (one directory per variant): VALU / LDS / SALU / VMEM-read instructions and
VALU issue cycles per ray, per kernel instantiation. Usage:
  python tools/pmc_compare.py NAME=DIR [NAME=DIR ...]  -> JSON on stdout"""
import collections
import csv
import glob
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_units_summary import bench_rays  # noqa: E402

out = {}
for spec in sys.argv[1:]:
    name, root = spec.split("=", 1)
    rays = bench_rays(root)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "tt_trace_kernel<false" not in r["Kernel_Name"]:
                continue
            per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
    rec = {}
    for k, cs in agg.items():
        info = k.rstrip(">").split(",")[-1].strip()
        n = rays[0] if info == "1" else rays[1]
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rec[k] = {c.replace("SQ_", "").lower() + "_per_ray": round(v / n, 2) for c, v in m.items() if c.startswith("SQ_")}
        if "SQ_ACTIVE_INST_VALU" in m:
            rec[k]["valu_issue_cycles_per_ray"] = round(4 * m["SQ_ACTIVE_INST_VALU"] / n, 1)
        if "GRBM_GUI_ACTIVE" in m:
            rec[k]["gpu_cycles"] = round(m["GRBM_GUI_ACTIVE"] / 8)
    out[name] = rec
print(json.dumps(out, indent=1))
