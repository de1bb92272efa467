"""Runs inside a subprocess with the oracle built under AddressSanitizer/UBSan (tests/test_native.py):
traces the committed golden scenes (closest hit, any-hit with the f1 accumulations, refit) through
the ASan build, so out-of-bounds reads or writes in the restatement abort the process."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "truetrace-unity-pathtracer_amd", "python"))
import golden_io  # noqa: E402
import oracle_ctypes as O  # noqa: E402
import tthip  # noqa: E402

assert O.lib()._name == os.environ["TT_ORACLE_LIB"]
for name in golden_io.NAMES:
    g = golden_io.load(name)
    sc, W, H = g["scene"], g["W"], g["H"]
    buf = g["rays0"].copy()
    info = np.zeros((W * H, 4), np.uint32)
    st, _ = O.trace(sc, buf, W * H, 0, 1000.0, W, H, info=info, counts=True, nthreads=4)
    assert st == 0, (name, st)
    r1 = g["rays1"].copy()
    st, _ = O.trace(sc, r1, g["n1"], 1, 1000.0, W, H, info=info, colors=g["colors"], counts=True, nthreads=4)
    assert st == 0, (name, st)
    sr = np.zeros(W * H // 2, tthip.SHADOW_DTYPE)
    sr["origin"] = buf["origin"][: len(sr)]
    sr["direction"] = -buf["direction"][: len(sr)]
    sr["t"] = np.where(np.arange(len(sr)) % 3 == 0, -5.0, 5.0)
    sr["illumination"] = 1.5
    sr["PixelIndex"] = np.arange(len(sr))
    col = np.zeros(W * H, tthip.COL_DTYPE)
    cache = np.zeros(W * H, tthip.CACHE_DTYPE)
    vis = np.zeros((len(sr), 4), np.float32)
    for flags in (0, tthip.TT_SHADOW_RADIANCE_CACHE, tthip.TT_SHADOW_VISIBILITY_CHECK):
        st, _ = O.shadow(sc, sr.copy(), len(sr), 1, W, H, visibility=vis, colors=col, cache=cache, flags=flags,
                         nthreads=4)
        assert st == 0, (name, flags, st)
print("asan oracle ok")
