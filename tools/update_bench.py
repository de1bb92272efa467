"""Host-side cost of the per-frame scene updates on C4 (2,401 _MeshData records, 393 TLAS nodes):
tt_scene_update_meshdata of all records and tt_scene_update_nodes of the TLAS region, each timed
on the host (median of 20 calls; the lib under TT_HIP_LIB), and whether the call returned before
the GPU finished (no stream sync). Usage: python tools/update_bench.py  -> one JSON line."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import torch  # noqa: E402,F401
import tthip  # noqa: E402
import ttconfigs as T  # noqa: E402

sc = T.c4_bistro()
eng = tthip.Engine(0)
eng.upload(sc)
md = sc.meshdata.copy()
nodes = sc.nodes[: sc.tlas_nodes].copy()
t_md, t_nd = [], []
for k in range(25):
    md["W2L"][1:, 12] += np.float32(1e-3)  # a small shift of every instance
    t0 = time.perf_counter()
    eng.update_meshdata(0, md)
    t1 = time.perf_counter()
    eng.update_nodes(0, nodes)
    t2 = time.perf_counter()
    if k >= 5:
        t_md.append(t1 - t0)
        t_nd.append(t2 - t1)
    eng.sync()
print(json.dumps({"lib": os.path.basename(os.environ.get("TT_HIP_LIB", "libtruetrace_hip.so")), "records": int(len(md)),
                  "tlas_nodes": int(sc.tlas_nodes), "scene_nodes": int(len(sc.nodes)),
                  "update_meshdata_host_ms": round(float(np.median(t_md)) * 1e3, 4),
                  "update_nodes_host_ms": round(float(np.median(t_nd)) * 1e3, 4)}))
