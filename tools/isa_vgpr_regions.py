#!/usr/bin/env python3
"""Where a kernel's VGPR peak comes from: prints the ISA lines of one kernel (from a
`hipcc -S --cuda-device-only` dump) that touch VGPRs at or above a threshold, with the nearest
preceding source-location comment, so a register-pressure regression can be traced to its code.
Usage: isa_vgpr_regions.py dump.s KERNEL_SYMBOL [threshold]"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    thr = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    lines = open(path).read().split("\n")
    try:
        a = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    except StopIteration:
        raise SystemExit(f"{sym} not found")
    b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[a:b]
    hits, loc = [], ""
    for i, l in enumerate(body):
        s = l.strip()
        if s.startswith(";") and ".hip:" in s or ".h:" in s:
            loc = s
        if not s or s.startswith(";"):
            continue
        regs = [int(x) for x in re.findall(r"\bv(\d+)\b", s)]
        regs += [int(y) for _, y in re.findall(r"v\[(\d+):(\d+)\]", s)]
        if regs and max(regs) >= thr:
            hits.append((i, max(regs), s, loc))
    print(f"{len(hits)} of {len(body)} lines use v>={thr}")
    seen = set()
    for i, m, s, l in hits:
        if l not in seen:
            seen.add(l)
            print(f"{i:6d} v{m:<4d} {s[:70]:70s} {l[:90]}")


if __name__ == "__main__":
    main()
