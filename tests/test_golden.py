"""Committed golden vectors: the oracle and the builder restatement reproduce them bit-exactly
(pins both over time; the GPU side of the same fixtures is in test_gpu_parity.py)."""
import numpy as np
import pytest

import golden_io
import oracle_ctypes as O
import tthip

sys_path_ok = True


@pytest.mark.parametrize("name", golden_io.NAMES)
def test_oracle_reproduces_golden(name):
    g = golden_io.load(name)
    sc, W, H, far = g["scene"], g["W"], g["H"], g["far"]
    r0 = g["rays0"].copy()
    info0 = np.zeros((W * H, 4), np.uint32)
    st, c0 = O.trace(sc, r0, W * H, 0, far, W, H, info=info0, counts=True)
    assert st == 0
    assert np.array_equal(r0["hits"][: W * H], g["hits0"])
    assert np.array_equal(info0, g["info0"])
    assert c0.tobytes() == g["counts0"].tobytes()
    r1 = g["rays1"].copy()
    info1 = np.zeros((W * H, 4), np.uint32)
    st, c1 = O.trace(sc, r1, g["n1"], 1, far, W, H, info=info1, colors=g["colors"], counts=True)
    assert st == 0
    assert np.array_equal(r1["hits"][W * H:W * H + g["n1"]], g["hits1"])
    assert np.array_equal(info1, g["info1"])
    assert c1.tobytes() == g["counts1"].tobytes()


@pytest.mark.parametrize("name", golden_io.NAMES)
def test_builder_reproduces_golden_scene(name):
    import sys
    import os

    sys.path.insert(0, golden_io.GOLDEN)
    import make_golden

    sc, _ = make_golden.scenes()[name]
    g = golden_io.load(name)["scene"]
    assert sc.nodes.tobytes() == g.nodes.tobytes()
    assert sc.tris.tobytes() == g.tris.tobytes()
    assert sc.tlas.tolist() == g.tlas.tolist()
    assert sc.meshdata.tobytes() == g.meshdata.tobytes()


def test_golden_multithreaded_oracle_agrees():
    g = golden_io.load("soup")
    r = g["rays0"].copy()
    st, _ = O.trace(g["scene"], r, g["W"] * g["H"], 0, g["far"], g["W"], g["H"], nthreads=4)
    assert st == 0 and np.array_equal(r["hits"][: g["W"] * g["H"]], g["hits0"])
