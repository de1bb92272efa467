#!/usr/bin/env python3
"""Issue-bound ceiling of the closest-hit kernel.

From rocprofv3 --pmc unit passes (tools/pmc_units.sh / pmc_units_config.sh: SQ_ACTIVE_INST_VALU,
SQ_INSTS_VALU, GRBM_GUI_ACTIVE) and the rays per launch, per timed kernel:

  VALU issue cycles per ray  c = 4 * SQ_ACTIVE_INST_VALU / rays     (quad-cycles -> SIMD cycles)
  VALU-issue ceiling         R = 1024 SIMDs * 2.4 GHz / c            (rays/s with VALU 100% busy at the
                                                                     MI355X peak engine clock)

i.e. the throughput the kernel would reach if nothing but VALU issue bounded it, with the
instruction stream it runs today. Usage:
  valu_ceiling.py UNITS_DIR KERNEL_SUBSTRING:RAYS[:MS] ...
(MS: the launch's product-kernel time, for the measured rate and the implied clock).
"""
import collections
import csv
import glob
import json
import sys

N_SIMD, N_XCD = 1024, 8


def load(root):
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
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    root = sys.argv[1]
    m = load(root)
    out = {}
    for spec in sys.argv[2:]:
        parts = spec.split(":")
        key, rays = parts[0], float(parts[1])
        k = next(kk for kk in m if key in kk)
        c = m[k]
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
        ms = float(parts[2]) if len(parts) > 2 else None
        f = 2.4e9
        valu_cyc_ray = 4.0 * c["SQ_ACTIVE_INST_VALU"] / rays
        busy = c["SQ_ACTIVE_INST_VALU"] / (cyc / 4.0 * N_SIMD)
        out[spec] = {"kernel": k, "rays": rays,
                     "pmc_run_clock_ghz": round(cyc / (ms * 1e-3) / 1e9, 3) if ms else None,
                     "valu_instr_per_ray": round(c["SQ_INSTS_VALU"] / rays, 1),
                     "valu_issue_cycles_per_ray": round(valu_cyc_ray, 1),
                     "valu_busy": round(busy, 3),
                     "ceiling_grays_s": round(N_SIMD * f / valu_cyc_ray / 1e9, 3),
                     "measured_grays_s": round(rays / (ms * 1e-3) / 1e9, 3) if ms else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
