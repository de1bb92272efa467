#!/usr/bin/env python3
"""Randomized sweep of the GPU BLAS builder (tt_blas_build_device) against the host build: seeded
meshes of 1 - 200k triangles from several generators -- soups, props, snapped-to-grid and duplicated
triangles (exact SAH ties), signed zeros, thin slivers, degenerate (zero-area) triangles -- each
built both ways and compared byte for byte (nodes, leaf-ordered triangles, leaf order, BVH2 depth).
Usage: builder_sweep.py [--cases 120] [--seed 1]. Prints one JSON document (commit under profiles/)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def mesh_for(tthip, rng, kind, n):
    if kind == "soup":
        return tthip.Mesh.soup(int(rng.integers(1 << 30)), n, float(rng.uniform(0.5, 20)), float(rng.uniform(0.01, 0.5)))
    if kind == "prop":
        return tthip.Mesh.prop(int(rng.integers(1 << 30)), max(n, 200))
    pos = rng.uniform(-4, 4, (3 * n, 3)).astype(np.float32)
    if kind == "snapped":  # coordinates on a coarse grid: many equal centroids and box faces
        pos = np.round(pos * 2) / 2
    elif kind == "duplicated":  # every triangle present twice or three times
        k = max(1, n // 3)
        base = pos[: 3 * k]
        pos = np.concatenate([base] * 4)[: 3 * n]
    elif kind == "signed_zero":
        pos = np.round(pos).astype(np.float32)
        pos[rng.random(pos.shape) < 0.4] = -0.0
    elif kind == "slivers":  # long thin triangles along one axis
        pos[1::3] = pos[0::3] + np.array([rng.uniform(2, 8), 1e-4, 0], np.float32)
        pos[2::3] = pos[0::3] + np.array([0, 0, 1e-4], np.float32)
    elif kind == "degenerate":  # a third of the triangles have zero area
        m = rng.random(n) < 0.33
        pos[1::3][m] = pos[0::3][m]
        pos[2::3][m] = pos[0::3][m]
    return tthip.Mesh.from_arrays(pos.astype(np.float32), np.arange(3 * n, dtype=np.int32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=120)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import torch  # noqa: F401
    import tthip

    eng = tthip.Engine(0)
    rng = np.random.default_rng(a.seed)
    kinds = ["soup", "prop", "snapped", "duplicated", "signed_zero", "slivers", "degenerate"]
    rows, bad = [], 0
    t0 = time.time()
    for c in range(a.cases):
        kind = kinds[c % len(kinds)]
        n = int(np.exp(rng.uniform(0, np.log(200_000))))
        mesh = mesh_for(tthip, rng, kind, n)
        host = tthip.Blas(mesh)
        v = mesh.view()
        aabbs = np.zeros((host.n_tris, 6), np.float32)
        tthip.scene_lib().tt_blas_prepare_aabbs(v, aabbs.ctypes.data)
        ph = np.zeros((3, host.n_tris), np.int32)
        pd = np.zeros((3, host.n_tris), np.int32)
        tthip.scene_lib().tt_bvh2_presort(aabbs.ctypes.data, host.n_tris, ph.ctypes.data)
        st = eng.L.tt_bvh2_presort_device(eng.h, aabbs.ctypes.data, host.n_tris, pd.ctypes.data)
        presort_same = bool(np.array_equal(ph, pd)) if st == 0 else None  # None: declined (host sorts)
        try:
            dev = tthip.Blas(mesh, engine=eng)
            nh, th = host.arrays()
            nd, td = dev.arrays()
            same = (nh.tobytes() == nd.tobytes() and th.tobytes() == td.tobytes()
                    and bool(np.array_equal(host.leaf_order(), dev.leaf_order()))
                    and host.info.bvh2_depth == dev.info.bvh2_depth)
        except tthip.TTError as e:
            same = False
            print(f"[sweep] case {c} {kind} n={n}: {e}", file=sys.stderr)
        same = same and presort_same is not False
        bad += 0 if same else 1
        rows.append({"case": c, "kind": kind, "tris": host.n_tris, "nodes": host.n_nodes, "identical": same,
                     "device_presort": presort_same})
        if not same:
            print(f"[sweep] MISMATCH case {c} {kind} n={n}", file=sys.stderr, flush=True)
    eng.close()
    out = {"tool": "tools/builder_sweep.py", "seed": a.seed, "cases": a.cases, "mismatches": bad,
           "triangles_total": int(sum(r["tris"] for r in rows)), "seconds": round(time.time() - t0, 1), "rows": rows}
    print(json.dumps(out))
    print(f"[sweep] {a.cases} cases, {bad} mismatches, {out['triangles_total']} triangles", file=sys.stderr)


if __name__ == "__main__":
    main()
