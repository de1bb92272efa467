"""Loader for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import os

import numpy as np

import tthip

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["cornell", "pedestal", "soup", "instanced", "invisible"]


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    sc = tthip.Scene(z["nodes"].view(tthip.NODE_DTYPE).copy(), z["tris"].view(tthip.TRI_DTYPE).copy(),
                     z["tlas"].astype(np.int32), z["meshdata"].view(tthip.MESH_DTYPE).copy(),
                     z["materials"].view(tthip.MAT_DTYPE).copy(), tlas_nodes=int(z["tlas_nodes"]))
    W, H = int(z["width"]), int(z["height"])
    g = {k: z[k] for k in z.files}
    rays0 = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    rays0[: W * H] = z["rays0"].view(tthip.RAY_DTYPE)
    n1 = int(z["n1"])
    rays1 = np.zeros(2 * W * H, tthip.RAY_DTYPE)
    rays1[W * H:W * H + n1] = z["rays1"].view(tthip.RAY_DTYPE)
    g.update(scene=sc, W=W, H=H, far=float(z["far"]), rays0=rays0, rays1=rays1, n1=n1,
             colors=z["colors"].view(tthip.COL_DTYPE).copy())
    return g
