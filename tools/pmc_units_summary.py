"""Unit-utilisation summary of the timed closest-hit kernels from tools/pmc_units.sh passes:
VALU issue (SQ_ACTIVE_INST_VALU quad-cycles over SIMD quad-cycles), texture-data path
(TD_TD_BUSY over TD-cycles) and texture-address path (TA_TA_BUSY), per kernel and averaged over
the bench's two launches. Writes the JSON bench.py reads (profiles/units_latest.json).
Usage: python tools/pmc_units_summary.py gpurun_out/pmcu profiles/units_latest.json"""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
N_CU, SIMD_PER_CU, N_XCD = 256, 4, 8
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/*/*_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "tt_trace_kernel<false" not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
res = {}
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    cyc = m["GRBM_GUI_ACTIVE"] / N_XCD  # GRBM sums the 8 XCDs
    res[k] = {"cycles": round(cyc),
              "valu_issue_busy": round(m["SQ_ACTIVE_INST_VALU"] / (cyc / 4 * N_CU * SIMD_PER_CU), 3),
              "td_busy": round(m["TD_TD_BUSY"] / (cyc * N_CU), 3),
              "ta_busy": round(m["TA_TA_BUSY"] / (cyc * N_CU), 3)}
mean = {f: round(sum(r[f] for r in res.values()) / len(res), 3) for f in ("valu_issue_busy", "td_busy", "ta_busy")}
json.dump({"source": root, "per_kernel": res, "mean": mean,
           "note": "SQ_ACTIVE_INST_VALU / SQ quad-cycles of 1024 SIMDs; TD/TA busy over 256 CUs; cycles = GRBM_GUI_ACTIVE / 8"},
          open(out, "w"), indent=1)
print(json.dumps(mean))
