"""Context / stream lifecycle on the GPU: the library's own teardown of dedicated streams a host never
destroyed, and the TT_ROOT_LEAF fast path's bookkeeping across scene updates (tt_api.hip: the host's copy
of node 0 is trusted after an upload or an update of node 0, and not after a device-side TLAS refit)."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import tthip
from parity_util import FAR

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(REPO, "tests", "native", "stream_exit_child.py")


def _run(cmd, tmp):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    if env.get("TT_HIP_LIB"):  # (the child runs in tmp: a variant library named relative to the repo)
        env["TT_HIP_LIB"] = os.path.abspath(env["TT_HIP_LIB"])
    return subprocess.run(cmd, capture_output=True, text=True, timeout=90, cwd=tmp, env=env)


@pytest.mark.parametrize("mode", ["contexts-destroyed", "keep-contexts", "worker-thread", "worker-shutdown"])
def test_exit_with_live_dedicated_streams(tmp_path, mode):
    """A process that made 3 dedicated streams, traced on them, and exits without tt_stream_destroy ends
    with status 0 -- plainly and under rocprofv3 --kernel-trace, where the CU-mask queues alive at HIP
    teardown used to crash the exit (SIGSEGV in __cxa_finalize), and where a teardown from an atexit handler
    alone aborts in the tool's per-thread stream table (destroyed with the thread's thread_locals, before any
    atexit handler runs; tt_api.hip arms the teardown from a main-thread thread_local for that reason, and the
    atexit form runs it on a fresh thread). The worker modes trace only from a worker thread (Unity's render
    thread shape): without tt_shutdown (the atexit path) and with it."""
    args = [sys.executable, CHILD] + ([mode] if mode != "contexts-destroyed" else [])
    r = _run(args, str(tmp_path))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "live 3" in r.stdout and "ok" in r.stdout
    prof = shutil.which("rocprofv3")
    if prof is None or os.environ.get("TT_TEST_ROCPROF") == "0":
        pytest.skip("no rocprofv3 (or TT_TEST_ROCPROF=0)")
    r = _run([prof, "--kernel-trace", "-d", str(tmp_path / "prof"), "-o", "run", "--"] + args, str(tmp_path))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "ok" in r.stdout


def test_stream_destroy_refuses_foreign_and_double():
    import ctypes as C

    import torch

    L = tthip.hip_lib()
    n0 = L.tt_stream_live_count()
    h = C.c_void_p()
    assert L.tt_stream_create(0, C.byref(h)) == tthip.TT_OK
    assert L.tt_stream_live_count() == n0 + 1
    foreign = torch.cuda.Stream(torch.device("cuda:0"))
    assert L.tt_stream_destroy(C.c_void_p(foreign.cuda_stream)) == tthip.TT_ERR_INVALID_ARG
    assert L.tt_stream_destroy(h) == tthip.TT_OK
    assert L.tt_stream_destroy(h) == tthip.TT_ERR_INVALID_ARG  # destroyed already
    assert L.tt_stream_live_count() == n0


def _one_instance(mesh, pos):
    return tthip.single_object_scene(mesh, tthip.trs_matrix(pos, 20.0, 1.0))


def test_root_leaf_bookkeeping_across_updates():
    """One-instance scenes take the root-leaf fast path (the root's one child stepped at ray start from the
    host's copy of node 0). Moving the instance with update_meshdata + a device tlas_refit must turn the fast
    path off (node 0 changed on the device only), and an update_nodes of node 0 must turn it back on with the
    new bytes -- each trace equal to a fresh context uploaded with the same state (on which the fast path is
    on), on the updated context and on a borrower of it."""
    import torch

    dev = torch.device("cuda:0")
    W, H = 256, 160
    WH = W * H
    mesh = tthip.Mesh.soup(77, 6000, 1.0, 0.08)
    a = _one_instance(mesh, (0.0, 0.0, 0.0))
    b = _one_instance(mesh, (0.35, -0.1, 0.2))  # moved: a different root box and W2L
    assert a.tlas_nodes == b.tlas_nodes and len(a.nodes) == len(b.nodes)
    T = a.tlas_nodes
    c2w, ip = tthip.unity_camera((0.2, 0.3, 3.0), (-0.05, -0.1, -1.0), (0, 1, 0), 50.0, W, H, 0.05, FAR)
    rays0 = torch.zeros(2 * WH * 48, dtype=torch.uint8, device=dev)

    def trace(e):
        r = rays0.clone()
        torch.cuda.synchronize(dev)
        e.trace(r, WH, 0, FAR, W, H, device=True)
        return r.view(-1, 48)[:WH, 32:48].cpu().numpy()

    def fresh(scene, nodes=None):
        e = tthip.Engine(0)
        try:
            s = scene if nodes is None else tthip.Scene(nodes, scene.tris, scene.tlas, scene.meshdata,
                                                         scene.materials, tlas_nodes=scene.tlas_nodes, meta=scene.meta)
            e.upload(s)
            return trace(e)
        finally:
            e.close()

    eng = tthip.Engine(0)
    bor = tthip.Engine(0, stream=torch.cuda.Stream(dev).cuda_stream)
    try:
        eng.upload(a)
        eng.generate(rays0, c2w, ip, W, H, 0.05, FAR, jitter=1, frames=0, max_bounce=1, device=True)
        torch.cuda.synchronize(dev)
        bor.share_scene(eng)
        exp_a = fresh(a)
        assert np.array_equal(trace(eng), exp_a) and np.array_equal(trace(bor), exp_a)
        # move the instance: the records and a device refit of the TLAS (node 0 rewritten on the device)
        eng.update_meshdata(0, b.meshdata)
        eng.tlas_refit(T, np.ascontiguousarray(b.meta["mesh_aabbs"], np.float32))
        refit_nodes = eng.scene_nodes(0, len(a.nodes))
        assert not np.array_equal(refit_nodes[:T], a.nodes[:T])  # the root box moved
        exp_refit = fresh(b, refit_nodes)
        assert not np.array_equal(exp_refit, exp_a)
        assert np.array_equal(trace(eng), exp_refit), "after tlas_refit (fast path must be off)"
        assert np.array_equal(trace(bor), exp_refit), "borrower after the lender's tlas_refit"
        # the host writes the TLAS nodes back (node 0 included): the fast path is on again, with b's bytes
        eng.update_nodes(0, b.nodes[:T])
        exp_b = fresh(b)
        assert np.array_equal(trace(eng), exp_b), "after update_nodes(0)"
        assert np.array_equal(trace(bor), exp_b), "borrower after the lender's update_nodes(0)"
        # and back to a by the same two routes
        eng.update_meshdata(0, a.meshdata)
        eng.update_nodes(0, a.nodes[:T])
        assert np.array_equal(trace(eng), exp_a) and np.array_equal(trace(bor), exp_a)
    finally:
        eng.close()
