"""Child process of tests/test_gpu_lifecycle.py::test_exit_with_live_dedicated_streams: a host that makes
dedicated streams (tt_stream_create), traces on them, and exits WITHOUT tt_stream_destroy -- what a Unity
domain reload or a crashed host script does. The library's own exit handler must destroy them before the
HIP runtime tears down (a CU-mask queue alive at that point crashed the exit in __cxa_finalize,
gpurun_out/qmap.out). Deliberately not tthip.dedicated_stream(): that path has a Python atexit hook of
its own, which would hide a missing library-side fix. Prints "live N" then "ok"; exit status 0.

Modes (argv[1]): keep-contexts (the contexts are never destroyed either); worker-thread (streams made and
traced on only from a worker thread, as a Unity render thread does -- the exit teardown then runs from the
library's atexit handler); worker-shutdown (the same, then tt_shutdown from the main thread: the contexts on
the destroyed streams refuse launches, and their destruction after it is clean)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (tthip binds to torch's HIP runtime)

import tthip  # noqa: E402


def work(mode, out):
    L = tthip.hip_lib()
    handles = []
    for _ in range(3):
        h = C.c_void_p()
        assert L.tt_stream_create(0, C.byref(h)) == tthip.TT_OK
        handles.append(h.value)
    sc = tthip.single_object_scene(tthip.Mesh.soup(5, 2000, 1.0, 0.1))
    W, H = 64, 48
    c2w, ip = tthip.unity_camera((0.3, 0.2, 2.4), (-0.1, -0.05, -1.0), (0, 1, 0), 60.0, W, H, 0.05, 1000.0)
    engines = []
    for h in handles:
        e = tthip.Engine(0, stream=h)
        e.upload(sc)
        rays = np.zeros(2 * W * H, tthip.RAY_DTYPE)
        e.generate(rays, c2w, ip, W, H, 0.05, 1000.0, jitter=1)
        e.trace(rays, W * H, 0, 1000.0, W, H)
        engines.append(e)
    print("live", L.tt_stream_live_count(), flush=True)
    out.extend(engines)
    if mode == "keep-contexts":
        # the contexts stay alive too (they are never destroyed: os-level exit right after)
        tthip._ENGINES.clear()
        for e in engines:
            e.h = None  # Engine.__del__ must not destroy them either


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    engines = []
    if mode.startswith("worker"):
        import threading

        t = threading.Thread(target=work, args=(mode, engines))
        t.start()
        t.join()
        assert len(engines) == 3, "the worker failed"
    else:
        work(mode, engines)
    if mode == "worker-shutdown":
        L = tthip.hip_lib()
        assert L.tt_shutdown() == tthip.TT_OK
        assert L.tt_stream_live_count() == 0
        rays = np.zeros(2 * 64 * 48, tthip.RAY_DTYPE)
        s, st = engines[0].trace(rays, 64 * 48, 0, 1000.0, 64, 48, check=False)
        assert st == tthip.TT_ERR_INVALID_ARG, st  # its stream is gone: refused, not a launch on a dead queue
        assert L.tt_shutdown() == tthip.TT_OK  # idempotent
        for e in engines:
            e.close()
    print("ok", flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
