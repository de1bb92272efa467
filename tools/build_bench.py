#!/usr/bin/env python3
"""BLAS build times, host vs the GPU stages (row f4's builder half: BVH2 only, BVH2 + BVH8), on the BASELINE meshes:
C2 Sponza-shaped (262k tris) and C5 San-Miguel-shaped (10M tris). Both builds must be byte-identical
(nodes, leaf-ordered triangles, leaf order). Usage: build_bench.py [--meshes c2,c5]
Prints one JSON document (commit under profiles/)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--meshes", default="c2,c5")
    a = ap.parse_args()
    import torch  # noqa: F401  (binds the HIP runtime first)
    import tthip

    eng = tthip.Engine(0)
    out = {"tool": "tools/build_bench.py", "host_threads": os.cpu_count(), "rows": []}
    for name in a.meshes.split(","):
        mesh = {"c2": tthip.Mesh.sponza, "c5": tthip.Mesh.san_miguel}[name]()
        t0 = time.perf_counter()
        host = tthip.Blas(mesh)
        t_host = time.perf_counter() - t0
        tim2 = {}
        t0 = time.perf_counter()
        dev2 = tthip.Blas(mesh, engine=eng, timings=tim2, device_stages="bvh2")
        t_dev2 = time.perf_counter() - t0
        same2 = dev2.arrays()[0].tobytes() == host.arrays()[0].tobytes()
        del dev2
        tim = {}
        t0 = time.perf_counter()
        dev = tthip.Blas(mesh, engine=eng, timings=tim)
        t_dev = time.perf_counter() - t0
        nh, th = host.arrays()
        nd, td = dev.arrays()
        same = (nh.tobytes() == nd.tobytes() and th.tobytes() == td.tobytes()
                and bool(np.array_equal(host.leaf_order(), dev.leaf_order())))
        row = {"mesh": name, "tris": host.n_tris, "cwbvh_nodes": host.n_nodes, "bvh2_depth": host.info.bvh2_depth,
               "host_build_s": round(t_host, 3),
               "device_bvh2_host_bvh8_s": round(t_dev2, 3), "device_bvh2_host_bvh8_stages_s": {k: round(v, 3) for k, v in tim2.items()},
               "device_bvh2_bvh8_s": round(t_dev, 3), "device_bvh2_bvh8_stages_s": {k: round(v, 3) for k, v in tim.items()},
               "identical": same and same2}
        out["rows"].append(row)
        print(f"[build] {row}", file=sys.stderr, flush=True)
        del host, dev
    eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
