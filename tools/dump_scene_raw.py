#!/usr/bin/env python3
"""Writes a BASELINE config's trace inputs as raw little-endian buffers for
bindings/csharp/ScalarTraversal.cs (the north star's scalar C# baseline):

  nodes.bin meshdata.bin tris.bin tlas.bin materials.bin   AssetManager buffers, byte-exact
  rays.bin            2*W*H RayData (48 B), primary rays of the config's view
  expected_hits.bin   n x 16 B hit records from the oracle (the C# program checks itself)
  params.txt          "n_rays bounce far_plane width height"

usage: python tools/dump_scene_raw.py OUT_DIR [--config c1|c2] [--width W --height H]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def dump(out_dir, config="c2", width=0, height=0, threads=8):
    import oracle_ctypes as O  # the oracle produces the expected records (test infrastructure)
    import ttconfigs as T

    sc, view = {"c1": (T.c1_cornell, T.C1_VIEW), "c2": (T.c2_sponza, T.C2_VIEW)}[config]
    sc = sc()
    W, H = width or view.width, height or view.height
    c2w, ip = view.camera(W, H)
    rays = O.generate(c2w, ip, W, H, T.NEAR, T.FAR)
    os.makedirs(out_dir, exist_ok=True)
    for name, arr in (("nodes", sc.nodes), ("tris", sc.tris), ("tlas", sc.tlas), ("meshdata", sc.meshdata),
                      ("materials", sc.materials), ("rays", rays)):
        np.ascontiguousarray(arr).view(np.uint8).tofile(os.path.join(out_dir, f"{name}.bin"))
    ref = rays.copy()
    st, _ = O.trace(sc, ref, W * H, 0, T.FAR, W, H, nthreads=threads)
    assert st == 0
    np.ascontiguousarray(ref["hits"][: W * H]).astype(np.uint32).tofile(os.path.join(out_dir, "expected_hits.bin"))
    with open(os.path.join(out_dir, "params.txt"), "w") as f:
        f.write(f"{W * H} 0 {T.FAR!r} {W} {H}\n")
    return sc, rays, ref


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("out_dir")
    ap.add_argument("--config", default="c2", choices=["c1", "c2"])
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    a = ap.parse_args()
    dump(a.out_dir, a.config, a.width, a.height)
