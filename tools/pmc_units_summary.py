"""Unit-utilisation summary and VALU-issue ceiling of the timed closest-hit kernels, from the
tools/pmc_units.sh passes (one rocprofv3 --pmc run per counter group on
`bench.py --parts 1`, so every dispatch of a kernel traces the same full-frame batch):

  valu_issue_busy  SQ_ACTIVE_INST_VALU quad-cycles / SIMD quad-cycles (1024 SIMDs)
  td_busy/ta_busy  TD_TD_BUSY / TA_TA_BUSY over TD/TA cycles (256 CUs)
  valu_issue_cycles_per_ray = 4 * SQ_ACTIVE_INST_VALU / rays of the dispatch
  valu_ceiling_grays_s      = 1024 SIMDs * 2.4 GHz / valu_issue_cycles_per_ray
                              (the rate with VALU issue 100% busy at the MI355X peak engine clock,
                               for the instruction stream the kernel runs)

Rays per dispatch come from the bench JSON line each pass printed (config.primary_rays /
config.bounce_rays): tt_trace_kernel<..., 1> is the primary launch (INFO = 1), <..., 2> the
bounce-1 launch. Writes the JSON bench.py reads for `roofline` (profiles/units_latest.json).
Usage: python tools/pmc_units_summary.py gpurun_out/pmcu profiles/units_latest.json"""
import collections
import csv
import glob
import json
import os
import sys

N_CU, SIMD_PER_CU, N_XCD = 256, 4, 8
PEAK_CLOCK_HZ = 2.4e9


def bench_rays(root):
    """(primary rays, bounce rays) from the bench line of the pass logs."""
    for log in sorted(glob.glob(os.path.join(root, "*.log"))):
        for ln in open(log, errors="replace"):
            if ln.startswith("{") and '"metric"' in ln:
                c = json.loads(ln)["config"]
                assert c.get("parts_per_rank", 1) == 1, "the VALU model needs full-frame launches (--parts 1)"
                return int(c["primary_rays"]), int(c["bounce_rays"])
    return None


def main():
    root, out = sys.argv[1], sys.argv[2]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/*/*_counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "tt_trace_kernel<false" not in r["Kernel_Name"] and "tt_trace_kernel_ord<" not in r["Kernel_Name"]:
                continue
            per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        # an adaptive-order kernel's first dispatch has no order yet (it only records costs): skip it
        first_ord = {}
        for (k, d) in per:
            if "_ord<" in k:
                first_ord[k] = min(first_ord.get(k, int(d)), int(d))
        for (k, d), cs in per.items():
            if k in first_ord and int(d) == first_ord[k] and sum(1 for kk, _ in per if kk == k) > 1:
                continue
            for c, v in cs.items():
                agg[k][c].append(v)
    rays = bench_rays(root)
    res = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        cyc = m["GRBM_GUI_ACTIVE"] / N_XCD  # GRBM sums the 8 XCDs
        rec = {"cycles": round(cyc),
               "valu_issue_busy": round(m["SQ_ACTIVE_INST_VALU"] / (cyc / 4 * N_CU * SIMD_PER_CU), 3),
               "td_busy": round(m["TD_TD_BUSY"] / (cyc * N_CU), 3),
               "ta_busy": round(m["TA_TA_BUSY"] / (cyc * N_CU), 3)}
        info = k.rstrip(">").split(",")[-1].strip()
        if rays is not None and info in ("1", "2"):
            n = rays[0] if info == "1" else rays[1]
            c_ray = 4.0 * m["SQ_ACTIVE_INST_VALU"] / n
            rec.update(rays=n, valu_instr_per_ray=round(m["SQ_INSTS_VALU"] / n, 2),
                       valu_issue_cycles_per_ray=round(c_ray, 2),
                       valu_ceiling_grays_s=round(N_CU * SIMD_PER_CU * PEAK_CLOCK_HZ / c_ray / 1e9, 4))
        res[k] = rec
    mean = {f: round(sum(r[f] for r in res.values()) / len(res), 3) for f in ("valu_issue_busy", "td_busy", "ta_busy")}
    json.dump({"source": root, "per_kernel": res, "mean": mean,
               "note": "SQ_ACTIVE_INST_VALU / SQ quad-cycles of 1024 SIMDs; TD/TA busy over 256 CUs; cycles = "
                       "GRBM_GUI_ACTIVE / 8; valu_ceiling_grays_s = 1024 SIMDs x 2.4 GHz / (4 x SQ_ACTIVE_INST_VALU "
                       "per ray)"},
              open(out, "w"), indent=1)
    print(json.dumps({k: {f: v.get(f) for f in ("valu_issue_busy", "valu_issue_cycles_per_ray", "valu_ceiling_grays_s")}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
