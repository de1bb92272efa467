"""The C ABI from a plain C host (examples/tt_frame.c): the binary builds with -std=c99 -Wpedantic
-Werror against include/*.h, links both shared libraries, and (GPU) drives one frame — primary
rays, bounce 0 with _PrimaryTriangleInfo, diffuse enqueue, bounce 1 — whose dumped buffers the CPU
oracle re-traces bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import oracle_ctypes as O
import tthip
from parity_util import CPU_THREADS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "examples", "bin", "tt_frame")


def _need_bin():
    if not os.path.exists(BIN):
        pytest.skip("examples/bin/tt_frame not built (run __graft_entry__.build())")


def test_c_host_links_and_reports_no_device():
    _need_bin()
    if tthip.device_count() > 0:
        pytest.skip("a GPU is visible (covered by the gpu test)")
    r = subprocess.run([BIN, "16", "16"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "no HIP device" in r.stderr, (r.returncode, r.stderr)


def load_dump(path):
    raw = open(path, "rb").read()
    hdr = np.frombuffer(raw, np.uint32, 10)
    assert hdr[0] == 0x54544652
    W, H, nn, nt, ntl, nm, nmat, tlas_nodes, n1 = (int(x) for x in hdr[1:])
    off = 40

    def take(dtype, n):
        nonlocal off
        a = np.frombuffer(raw, dtype, n, off).copy()
        off += a.nbytes
        return a

    sc = tthip.Scene(take(tthip.NODE_DTYPE, nn), take(tthip.TRI_DTYPE, nt), take(np.int32, ntl),
                     take(tthip.MESH_DTYPE, nm), take(tthip.MAT_DTYPE, nmat), tlas_nodes=tlas_nodes)
    rays = take(tthip.RAY_DTYPE, 2 * W * H)
    info = take(np.uint32, 4 * W * H).reshape(-1, 4)
    assert off == len(raw)
    return sc, W, H, n1, rays, info


@pytest.mark.gpu
def test_c_host_frame_matches_oracle(tmp_path):
    _need_bin()
    if tthip.device_count() == 0:
        pytest.skip("no GPU visible")
    W, H = 200, 136
    dump = str(tmp_path / "frame.bin")
    r = subprocess.run([BIN, str(W), str(H), dump], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "tt_frame" in r.stdout
    assert "tt_frame group: 2 members, 0 of" in r.stdout  # the tt_group_* frame of the same camera
    sc, W2, H2, n1, rays, info = load_dump(dump)
    assert (W2, H2) == (W, H)
    assert int((rays["hits"][: W * H, 1] != 0xFFFFFFFF).sum()) > W * H // 2  # the room surrounds the view
    assert 0 < n1 <= W * H
    ref = rays.copy()
    ref_info = np.zeros_like(info)
    st, _ = O.trace(sc, ref, W * H, 0, 1000.0, W, H, info=ref_info, nthreads=CPU_THREADS)
    assert st == 0
    st, _ = O.trace(sc, ref, n1, 1, 1000.0, W, H, nthreads=CPU_THREADS)
    assert st == 0
    assert np.array_equal(rays["hits"][: W * H], ref["hits"][: W * H])
    assert np.array_equal(rays["hits"][W * H:W * H + n1], ref["hits"][W * H:W * H + n1])
    assert np.array_equal(info, ref_info)
