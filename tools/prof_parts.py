#!/usr/bin/env python3
"""Cross-checks bench.py's roofline against a rocprofv3 --kernel-trace of the same command when the
N = 1 frame is traced as P parts on P streams (bench.py --parts P, the default 2).

The parts' launches overlap, so rocprofv3's per-kernel average duration is not the kernel's time per
frame: this tool takes the timed steps' dispatches from the kernel trace (the first 2P x (warmup +
steps) non-STATS closest-hit launches, <false, false, 1> primary and <false, false, 2> bounce-1, on
the part streams), drops the warmup, and reports the wall span per step (first start to last end of
the timed steps / steps), the per-stream launch averages, and the single-stream leg that follows (one
launch at a time on stream 0; its averages are bench.py's roofline.single_stream.avg_launch_ms).
With --bench the bench JSON line, it also recomputes roofline.achieved from the trace span.

Usage: prof_parts.py <run_kernel_trace.csv> [--parts 2 --warmup 3 --steps 20] [--bench bench.json]"""
import argparse
import csv
import json

TIMED = ("voidtt_trace_kernel<false,false,1>", "voidtt_trace_kernel<false,false,2>")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--parts", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--bench", default="")
    ap.add_argument("--single-last", action="store_true",
                    help="round-2 bench order (the single-stream leg after the timed region)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))
            if r["Kernel_Name"].split("(")[0].replace(" ", "") in TIMED]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    lead = []
    if not a.single_last:  # round 3: bench.py runs the single-stream leg BEFORE the timed parts
        lead, rows = rows[:2 * (a.warmup + a.steps)], rows[2 * (a.warmup + a.steps):]
    n_parts = 2 * a.parts * (a.warmup + a.steps)
    parts, rest = rows[:n_parts], rows[n_parts:]
    timed = parts[2 * a.parts * a.warmup:]
    t0 = min(int(r["Start_Timestamp"]) for r in timed)
    t1 = max(int(r["End_Timestamp"]) for r in timed)
    per_stream = {}
    for r in timed:
        k = (r["Stream_Id"], r["Kernel_Name"].split("(")[0])
        per_stream.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {"tool": "tools/prof_parts.py", "trace": a.trace, "parts": a.parts, "steps": a.steps,
           "step_span_ms": round((t1 - t0) / 1e6 / a.steps, 4),
           "per_stream_launch_ms": {f"stream {s} {k}": round(sum(v) / len(v), 4)
                                    for (s, k), v in sorted(per_stream.items())}}
    if a.single_last:
        # the single-stream leg: the launches after the last one on a part stream other than the first's
        # (bench.py runs its steady-state steps, still in parts, in between)
        part_streams = {r["Stream_Id"] for r in timed}
        others = part_streams - {timed[0]["Stream_Id"]} if timed else set()
        last_other = max((i for i, r in enumerate(rest) if r["Stream_Id"] in others), default=-1)
        leg = rest[last_other + 1:]
    else:
        leg = lead
    single = leg[2 * a.warmup: 2 * (a.warmup + a.steps)]
    if single:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in single]
        out["single_stream_avg_launch_ms"] = round(sum(d) / len(d), 4)
        out["single_stream_streams"] = sorted({r["Stream_Id"] for r in single})
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        rf = b["roofline"]
        out["bench_ms_per_step"] = b["ms_per_step"]
        hb = rf.get("hbm", rf)  # round 3: the algorithmic-bytes view moved to roofline.hbm
        out["bench_achieved_alg_GBs"] = hb.get("achieved_alg_gbs", rf.get("achieved"))
        out["trace_achieved_alg_GBs"] = round(hb["alg_bytes_per_step"] / (out["step_span_ms"] * 1e-3) / 1e9, 1)
        if rf.get("single_stream"):
            out["bench_single_stream_avg_launch_ms"] = rf["single_stream"]["avg_launch_ms"]
        pl = rf.get("per_launch", {})
        if pl:  # roofline.per_launch: HIP-event launch times of the single-stream leg, per kernel
            out["bench_per_launch_ms"] = {v["kernel"]: v["launch_ms"] for v in pl.values()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
