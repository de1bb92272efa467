#!/usr/bin/env python3
"""Static VALU / SALU / memory instruction counts of one kernel's ISA, per basic block, attributed to
source regions through the line table (hipcc -S --cuda-device-only -gline-tables-only dump).

A basic block's region is decided by the source lines of its instructions: the first rule (in the
order given) that matches any of the block's lines of the kernel's own file wins. Regions are given
as NAME=FILE:LO-HI[,FILE:LO-HI...]. Prints per region: blocks, VALU, SALU, memory instructions, and a
per-block listing with --blocks. Usage:
  isa_blocks.py dump.s KERNEL_SYMBOL [--regions spec ...] [--blocks]"""
import argparse
import collections
import re


def parse(path, sym):
    lines = open(path).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
    a = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, loc = [], None, None
    for l in lines[a + 1:b]:
        s = l.strip()
        m = re.match(r"^(\.LBB\w+):", s)
        if m or cur is None:
            cur = {"label": m.group(1) if m else "entry", "valu": 0, "salu": 0, "mem": 0, "lines": collections.Counter(),
                   "ops": collections.Counter()}
            blocks.append(cur)
            if m:
                continue
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cur["valu"] += 1
            cur["ops"][op] += 1
            if loc:
                cur["lines"][loc] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        elif op.startswith(("buffer_", "global_", "flat_", "ds_", "scratch_")):
            cur["mem"] += 1
            if loc:
                cur["lines"][loc] += 0
    return blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("sym")
    ap.add_argument("--regions", nargs="*", default=[])
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("--inherit", action="store_true",
                    help="a block none of whose lines matches a rule takes the region of the block before it")
    ap.add_argument("--json", default=None, help="write {region: {blocks, valu, salu, mem}} here")
    a = ap.parse_args()
    rules = []
    for spec in a.regions:
        name, rng = spec.split("=", 1)
        rs = []
        for part in rng.split(","):
            f, lohi = part.split(":")
            lo, hi = (int(x) for x in lohi.split("-"))
            rs.append((f, lo, hi))
        rules.append((name, rs))
    blocks = parse(a.dump, a.sym)
    agg = collections.defaultdict(lambda: [0, 0, 0, 0])
    prev = "other"
    for bl in blocks:
        reg = None
        for name, rs in rules:
            if any(f == fl and lo <= ln <= hi for (fl, ln) in bl["lines"] for f, lo, hi in rs):
                reg = name
                break
        if reg is None:
            reg = prev if a.inherit else "other"
        prev = reg
        bl["region"] = reg
        g = agg[reg]
        g[0] += 1
        g[1] += bl["valu"]
        g[2] += bl["salu"]
        g[3] += bl["mem"]
        if a.blocks:
            top = ", ".join(f"{f}:{ln}" for (f, ln), _ in bl["lines"].most_common(4))
            print(f"{bl['label']:>14} {reg:>12} V{bl['valu']:4d} S{bl['salu']:4d} M{bl['mem']:3d}  {top}")
    if a.json:
        import json

        json.dump({k: {"blocks": v[0], "valu": v[1], "salu": v[2], "mem": v[3]} for k, v in agg.items()},
                  open(a.json, "w"), indent=1)
    print(f"{'region':>14} {'blocks':>6} {'VALU':>6} {'SALU':>6} {'mem':>5}")
    for name in [r[0] for r in rules] + ["other"]:
        if name in agg:
            g = agg[name]
            print(f"{name:>14} {g[0]:6d} {g[1]:6d} {g[2]:6d} {g[3]:5d}")


if __name__ == "__main__":
    main()
