"""C-ABI surface: every function the public headers declare is exported by the built libraries,
struct layouts agree between C and Python, and the engine refuses to run without a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import tthip

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(tt_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def test_hip_library_exports_every_declared_symbol():
    names = declared("truetrace_hip.h")
    assert "tt_trace_closest" in names and "tt_scene_upload" in names
    lib = C.CDLL(os.path.join(tthip.LIB_DIR, "libtruetrace_hip.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(tthip.HIP_SYMBOLS) <= set(names)


def test_scene_library_exports_every_declared_symbol():
    names = declared("truetrace_scene.h")
    lib = C.CDLL(os.path.join(tthip.LIB_DIR, "libtruetrace_scene.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_layouts():
    L = tthip.hip_lib()
    assert L.tt_abi_version() == 1
    assert C.sizeof(tthip.TraceParams) == 24
    assert C.sizeof(tthip.Stats) == 8 * 8 + 8
    assert tthip.RAY_DTYPE.fields["hits"][1] == 32  # RayData.hits at byte 32 (CommonData.cginc:106)
    assert tthip.MESH_DTYPE.fields["TriOffset"][1] == 64
    assert tthip.MESH_DTYPE.fields["mesh_data_bvh_offsets"][1] == 76
    assert tthip.COL_DTYPE.fields["Data"][1] == 48


@pytest.mark.skipif(tthip.device_count() > 0, reason="checks the no-GPU behaviour")
def test_no_device_is_loud():
    L = tthip.hip_lib()
    assert L.tt_device_count() == 0
    with pytest.raises(tthip.TTError) as e:
        tthip.Engine(0)
    assert e.value.status == tthip.TT_ERR_NO_DEVICE


@pytest.mark.skipif(tthip.device_count() > 0, reason="checks the no-GPU behaviour")
def test_stream_create_without_device_is_loud():
    L = tthip.hip_lib()
    h = C.c_void_p()
    assert L.tt_stream_create(0, C.byref(h)) == tthip.TT_ERR_NO_DEVICE
    assert h.value is None
    assert L.tt_stream_create(0, None) == tthip.TT_ERR_INVALID_ARG
    assert L.tt_stream_destroy(None) == tthip.TT_ERR_INVALID_ARG
    assert L.tt_stream_destroy(C.c_void_p(0x1000)) == tthip.TT_ERR_INVALID_ARG  # not made by tt_stream_create
    assert L.tt_stream_live_count() == 0


def test_null_context_is_rejected():
    L = tthip.hip_lib()
    p = tthip.TraceParams(n_rays=1, bounce=0, far_plane=1.0, screen_width=1, screen_height=1, flags=0)
    assert L.tt_trace_closest(None, C.byref(p), None, None, None, None) == tthip.TT_ERR_INVALID_ARG
    assert L.tt_scene_upload(None, None, 0, None, 0, None, 0, None, 0, None, 0) == tthip.TT_ERR_INVALID_ARG
    assert L.tt_last_error(None) == b"null context"


def test_every_bound_hip_function_has_a_prototype():
    """ctypes defaults to int arguments: a bound function without argtypes would truncate the
    64-bit context pointer. Every declared function that takes arguments must carry argtypes."""
    L = tthip.hip_lib()
    src = open(os.path.join(REPO, "include", "truetrace_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    no_args = set(re.findall(r"\b(tt_[a-z0-9_]+)\s*\(\s*(?:void)?\s*\)", src))
    missing = [n for n in declared("truetrace_hip.h") if n not in no_args and getattr(L, n).argtypes is None]
    assert not missing, missing


def test_null_context_selftest_is_rejected():
    L = tthip.hip_lib()
    n = C.c_uint64()
    assert L.tt_selftest_rcp(None, C.addressof(n)) == tthip.TT_ERR_INVALID_ARG


def test_flag_constants_match_the_header():
    """Every TT_TRACE_* / TT_SHADOW_* / TT_ERR_* constant tthip binds equals the header's enum value."""
    src = open(os.path.join(REPO, "include", "truetrace_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    hdr = {}
    for name, expr in re.findall(r"\b(TT_(?:TRACE|SHADOW|ERR)_[A-Z0-9_]+)\s*=\s*([^,\n}]+)", src):
        hdr[name] = int(eval(expr.replace("u", ""), {}))  # "1u << 7" -> 1 << 7
    bound = {k: getattr(tthip, k) for k in dir(tthip) if re.fullmatch(r"TT_(TRACE|SHADOW|ERR)_[A-Z0-9_]+", k)}
    assert "TT_TRACE_ADAPTIVE_ORDER" in bound and "TT_TRACE_DEVICE_PTRS" in bound
    for k, v in bound.items():
        assert k in hdr, f"{k} is bound in tthip but not declared in truetrace_hip.h"
        assert hdr[k] == v, (k, hdr[k], v)
