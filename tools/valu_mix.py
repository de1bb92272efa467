#!/usr/bin/env python3
"""The instruction-mix VALU model beside bench.py's hard issue bound (roofline.models.mix): each wave64 VALU
instruction of the closest-hit kernels priced at the measured issue cost of its class, weighted by how often
the kernel executes it.

Inputs (no GPU needed):
  * the ISA of csrc/tt_trace.hip for gfx950 (hipcc -S with line tables, compiled here with the product flags);
  * per-ray wave executions of the node step and the triangle pass (profiles/r05/diag/diag_blocks_c2.json,
    tools/diag_blocks.py on the bench's C2 launches);
  * VALU instructions per ray and the busy fractions of the same kernels (profiles/units_latest.json, PMC);
  * per-instruction issue costs measured on gfx950 (profiles/r01_micro_valu_ops.txt, tools/micro/valu_ops.hip:
    many independent waves), used relative to v_fma_f32 and anchored at the 2-cycle wave64 fast-op issue.

Dynamic mix per ray = node steps/ray x the node-step blocks' instruction histogram + triangle passes/ray x the
triangle blocks' + the rest of the PMC's VALU/ray spread over the remaining blocks' static histogram (refill,
ray setup, records, loop control: executed far less often, so a static mix is used for them). The model's
cycles per instruction = sum(count x cost) / sum(count). It is a model, not a bound (bench.py's roofline.frac
is against the hard 2-cycle bound); it explains why the step runs at ~3.7 cycles per VALU instruction.

Writes mix_cycles_per_instr and the class breakdown into profiles/units_latest.json (per kernel) and prints
the summary. Usage: tools/valu_mix.py [--isa /tmp/tt_trace.s] [--diag ...] [--units ...] [--no-write]"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from isa_blocks import parse  # noqa: E402

CSRC = os.path.join(REPO, "truetrace-unity-pathtracer_amd", "csrc")
KERNELS = {"1": "_Z15tt_trace_kernelILb0ELb0ELi1EEv9TraceArgs", "2": "_Z15tt_trace_kernelILb0ELb0ELi2EEv9TraceArgs"}
# source regions (file: line ranges) of the node step and the triangle pass (node_intersect / intersect_triangle
# are inlined: their instructions carry tt_traverse.h lines)
NODE = [("tt_traverse.h", 139, 208), ("tt_trace.hip", 423, 459)]
TRI = [("tt_traverse.h", 292, 390), ("tt_trace.hip", 475, 486)]
WIDE = [("tt_wide.h", 1, 10000)]
FAST = ("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_and_b32", "v_or_b32",
        "v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32", "v_cndmask_b32", "v_not_b32",
        "v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_mul_lo_u32", "v_readfirstlane_b32", "v_nop")
TRANS = ("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")


def costs():
    """Issue cycles per wave64 instruction per SIMD by mnemonic: the micro's measured costs RELATIVE to v_fma_f32,
    anchored at the wave64 fast-op issue of 2 cycles (MI355X_MICROARCH.md, per-instruction constants). The micro
    states absolute cycles at an assumed 2.1 GHz (2.71 for v_fma_f32); only the ratios are used, since the
    kernel's own instruction stream issues faster than the micro's absolute figures imply."""
    raw = raw_costs()
    ref = raw.get("v_fma_f32", 2.71)
    return {k: 2.0 * v / ref for k, v in raw.items()}


def raw_costs():
    c = {}
    for ln in open(os.path.join(REPO, "profiles", "r01_micro_valu_ops.txt")):
        m = re.match(r"\s*(v_\w+)\s+\S+ ms\s+\S+ ns/wave-instr/SIMD\s+\((\S+) cycles", ln)
        if m:
            c[m.group(1)] = float(m.group(2))
    m = re.search(r"v_cmp\+v_cndmask\s+\S+ ms\s+\S+ ns/wave-instr/SIMD\s+\((\S+) cycles",
                  open(os.path.join(REPO, "profiles", "r01_micro_valu_ops.txt")).read())
    if m and "v_cmp_lt_f32" in c:  # the pair's cost minus the compare's: the select alone (its own row is a
        c["v_cndmask_b32"] = max(1.0, 2 * float(m.group(1)) - c["v_cmp_lt_f32"])  # dependent-VCC artefact)
    return c


def cost_of(op, table):
    base = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0].split("_dpp")[0]
    if base in table:
        return table[base], "measured"
    fast = table.get("v_fma_f32", 2.0)
    slow = table.get("v_max_f32", 3.1)
    if base.startswith(TRANS):
        return table.get("v_rcp_f32", 5.5), "trans"
    if base.startswith(FAST):
        return fast, "fast"
    return slow, "slow"


def region_of(block):
    lines = block["lines"]
    for name, rules in (("wide", WIDE), ("node", NODE), ("tri", TRI)):
        if any(f == fl and lo <= ln <= hi for (fl, ln) in lines for f, lo, hi in rules):
            return name
    return "rest"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--isa", default="/tmp/tt_trace_mix.s")
    ap.add_argument("--diag", default=os.path.join(REPO, "profiles", "r05", "diag", "diag_blocks_c2.json"))
    ap.add_argument("--units", default=os.path.join(REPO, "profiles", "units_latest.json"))
    ap.add_argument("--no-write", action="store_true")
    a = ap.parse_args()
    if not os.path.exists(a.isa):
        subprocess.run(["/opt/rocm/bin/hipcc", "-S", "--cuda-device-only", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-ffp-contract=off", "-fno-slp-vectorize", "-gline-tables-only",
                        os.path.join(CSRC, "tt_trace.hip"), "-o", a.isa], check=True)
    table = costs()
    diag = json.load(open(a.diag))["launches"]
    units = json.load(open(a.units))
    out = {}
    for info, sym in KERNELS.items():
        blocks = parse(a.isa, sym)
        ops = collections.defaultdict(collections.Counter)
        for b in blocks:
            ops[region_of(b)].update(b["ops"])
        d = diag[f"bounce{int(info) - 1}"]["per_ray"]
        per_ray = {"node": d["node_steps"], "tri": d["tri_passes"]}
        kname = next(k for k in units["per_kernel"] if k.endswith(f"false, false, {info}>"))
        pmc_vpr = units["per_kernel"][kname]["valu_instr_per_ray"]
        dyn = collections.Counter()
        for r in ("node", "tri"):
            for op, n in ops[r].items():
                dyn[op] += n * per_ray[r]
        rest = pmc_vpr - sum(dyn.values())
        n_rest = sum(ops["rest"].values())
        for op, n in ops["rest"].items():
            dyn[op] += max(rest, 0.0) * n / n_rest
        total = sum(dyn.values())
        cyc = 0.0
        classes = collections.Counter()
        for op, n in dyn.items():
            c, kind = cost_of(op, table)
            cyc += n * c
            classes[kind if kind != "measured" else ("fast" if c < 2.4 else "trans" if c > 4.5 else "slow")] += n
        cpi = cyc / total
        out[kname] = {"mix_cycles_per_instr": round(cpi, 3),
                      "mix_classes_per_ray": {k: round(v, 2) for k, v in sorted(classes.items())},
                      "mix_valu_per_ray_model": round(total, 2), "pmc_valu_per_ray": pmc_vpr,
                      "node_step_valu": sum(ops["node"].values()), "tri_pass_valu": sum(ops["tri"].values()),
                      "node_steps_per_ray": per_ray["node"], "tri_passes_per_ray": per_ray["tri"]}
        print(f"{kname}: {total:.1f} VALU/ray (PMC {pmc_vpr}), mix {cpi:.3f} cycles/instr, classes "
              f"{dict((k, round(v, 1)) for k, v in classes.items())}; node step {sum(ops['node'].values())} VALU x "
              f"{per_ray['node']}/ray, tri pass {sum(ops['tri'].values())} x {per_ray['tri']}/ray")
    if not a.no_write:
        for k, v in out.items():
            units["per_kernel"][k].update(v)
        units["mix_source"] = ("tools/valu_mix.py: the kernels' ISA (csrc/tt_trace.hip, product flags) x per-ray block "
                               f"executions ({os.path.relpath(a.diag, REPO)}) x issue costs "
                               "(profiles/r01_micro_valu_ops.txt)")
        json.dump(units, open(a.units, "w"), indent=1)
    return out


if __name__ == "__main__":
    main()
