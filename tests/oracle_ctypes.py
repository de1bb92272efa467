"""ctypes loader for the CPU oracle (oracle/libtt_oracle*.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / CPU baseline; the product path never touches the oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
import tthip  # noqa: E402

COUNTS_DTYPE = np.dtype([("node_visits", "<u4"), ("tri_tests", "<u4"), ("blas_entries", "<u4"),
                         ("accepts", "<u4"), ("max_stack", "<u4"), ("status", "<u4")])

_LIB = None


def _cpu_has_v3() -> bool:
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return all(f" {f} " in flags or f" {f}\n" in flags for f in ("fma", "avx2", "bmi2", "movbe"))


def lib(prefer_v3: bool = True):
    global _LIB
    if _LIB is None:
        d = os.path.join(REPO, "oracle")
        path = os.path.join(d, "libtt_oracle_v3.so") if prefer_v3 and _cpu_has_v3() else os.path.join(d, "libtt_oracle.so")
        if os.environ.get("TT_ORACLE_LIB"):  # e.g. the AddressSanitizer build (tests/test_native.py)
            path = os.environ["TT_ORACLE_LIB"]
        if not os.path.exists(path):
            path = os.path.join(d, "libtt_oracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError("oracle not built: run `make -C oracle`")
        L = C.CDLL(path)
        vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
        L.tt_oracle_trace.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, vp, u32, C.POINTER(tthip.TraceParams), vp,
                                      vp, vp, vp, i32]
        L.tt_oracle_trace.restype = i32
        L.tt_oracle_resolve_normals.argtypes = [vp, u32, vp, u32, C.POINTER(tthip.TraceParams), vp, vp]
        L.tt_oracle_resolve_normals.restype = i32
        L.tt_oracle_generate.argtypes = [vp, vp, u32, u32, C.c_float, C.c_float, i32, i32, i32, vp]
        L.tt_oracle_generate.restype = i32
        L.tt_oracle_hardware_threads.restype = i32
        L.tt_oracle_enqueue_diffuse_bounce.argtypes = [vp, u32, vp, u32, C.POINTER(tthip.TraceParams), vp, i32, i32,
                                                       C.POINTER(u32)]
        L.tt_oracle_enqueue_diffuse_bounce.restype = i32
        L.tt_oracle_sincos_pinned.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.tt_oracle_sincos_pinned.restype = None
        L.tt_oracle_shadow.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, vp, u32, C.POINTER(tthip.ShadowParams), vp,
                                       vp, vp, vp, vp, vp, i32]
        for name in ("tt_oracle_pack_rgbe", "tt_oracle_encode_rgb"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = u32
        for name in ("tt_oracle_unpack_rgbe", "tt_oracle_decode_rgb"):
            getattr(L, name).argtypes = [u32, vp]
            getattr(L, name).restype = None
        L.tt_oracle_pow.argtypes = [C.c_float, C.c_float]
        L.tt_oracle_pow.restype = C.c_float
        L.tt_oracle_shadow.restype = i32
        L.tt_oracle_set_alpha_atlas.argtypes = [vp, u32, u32]
        L.tt_oracle_set_alpha_atlas.restype = None
        L.tt_oracle_set_texture_atlas.argtypes = [vp, u32, u32]
        L.tt_oracle_set_texture_atlas.restype = None
        L.tt_oracle_tlas_refit.argtypes = [vp, u32, vp, u32, vp, u32]
        L.tt_oracle_tlas_refit.restype = i32
        L.tt_oracle_blas_refit.argtypes = [vp, u32, vp, u32, vp, u32, u32, vp, u32, u32, vp, u32, vp, vp]
        L.tt_oracle_blas_refit.restype = i32
        L._path = path
        _LIB = L
    return _LIB


_ATLAS_KEEP = None
_TEX_KEEP = None


def _set_atlas(scene):
    """The oracle's alpha and texture atlases are process-global: point them at the scene's (or
    clear them)."""
    global _ATLAS_KEEP, _TEX_KEEP
    a = getattr(scene, "alpha_atlas", None)
    if a is None:
        _ATLAS_KEEP = None
        lib().tt_oracle_set_alpha_atlas(None, 0, 0)
    else:
        _ATLAS_KEEP = np.ascontiguousarray(a, np.uint8)
        lib().tt_oracle_set_alpha_atlas(_ATLAS_KEEP.ctypes.data, _ATLAS_KEEP.shape[1], _ATLAS_KEEP.shape[0])
    t = getattr(scene, "texture_atlas", None)
    if t is None:
        _TEX_KEEP = None
        lib().tt_oracle_set_texture_atlas(None, 0, 0)
    else:
        _TEX_KEEP = np.ascontiguousarray(t, np.float16)
        lib().tt_oracle_set_texture_atlas(_TEX_KEEP.ctypes.data, _TEX_KEEP.shape[1], _TEX_KEEP.shape[0])


def trace(scene: "tthip.Scene", rays: np.ndarray, n_rays: int, bounce: int, far_plane: float, width: int,
          height: int, info=None, colors=None, flags: int = 0, counts: bool = False, nthreads: int = 1,
          materials: bool = True):
    """Runs the oracle in place on ``rays`` (and ``info``). Returns (status, counts or None)."""
    L = lib()
    p = tthip.TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width,
                          screen_height=height, flags=flags)
    cnt = np.zeros(n_rays, COUNTS_DTYPE) if counts else None
    mats = scene.materials if materials else None
    _set_atlas(scene)
    st = L.tt_oracle_trace(scene.nodes.ctypes.data, len(scene.nodes), scene.tris.ctypes.data, len(scene.tris),
                           scene.tlas.ctypes.data, len(scene.tlas), scene.meshdata.ctypes.data, len(scene.meshdata),
                           None if mats is None else mats.ctypes.data, 0 if mats is None else len(mats), C.byref(p),
                           rays.ctypes.data, None if info is None else info.ctypes.data,
                           None if colors is None else colors.ctypes.data,
                           None if cnt is None else cnt.ctypes.data, nthreads)
    return st, cnt


def shadow(scene: "tthip.Scene", srays: np.ndarray, n_rays: int, bounce: int, width: int, height: int,
           visibility=None, colors=None, nee_pos=None, counts: bool = False, nthreads: int = 1, flags: int = 0,
           cache=None):
    """Any-hit oracle in place on ``srays`` (SHADOW_DTYPE) and the optional outputs (``cache``: CACHE_DTYPE
    per pixel, the RadianceCache CacheBuffer). Returns (status, counts or None); counts.status 0 reached
    |t| (visible in TT_SHADOW_VISIBILITY_CHECK mode), 4 occluded, 1 Reps exhausted."""
    L = lib()
    p = tthip.ShadowParams(n_rays=n_rays, bounce=bounce, screen_width=width, screen_height=height, flags=flags)
    cnt = np.zeros(n_rays, COUNTS_DTYPE) if counts else None
    mats = scene.materials
    _set_atlas(scene)
    st = L.tt_oracle_shadow(scene.nodes.ctypes.data, len(scene.nodes), scene.tris.ctypes.data, len(scene.tris),
                            scene.tlas.ctypes.data, len(scene.tlas), scene.meshdata.ctypes.data, len(scene.meshdata),
                            None if mats is None or len(mats) == 0 else mats.ctypes.data,
                            0 if mats is None else len(mats), C.byref(p), srays.ctypes.data,
                            None if visibility is None else visibility.ctypes.data,
                            None if colors is None else colors.ctypes.data,
                            None if nee_pos is None else nee_pos.ctypes.data,
                            None if cache is None else cache.ctypes.data,
                            None if cnt is None else cnt.ctypes.data, nthreads)
    return st, cnt


def pack_rgbe(v):
    a = np.ascontiguousarray(v, np.float32)
    return int(lib().tt_oracle_pack_rgbe(a.ctypes.data))


def unpack_rgbe(x):
    o = np.zeros(3, np.float32)
    lib().tt_oracle_unpack_rgbe(int(x), o.ctypes.data)
    return o


def encode_rgb(c):
    a = np.ascontiguousarray(c, np.float32)
    return int(lib().tt_oracle_encode_rgb(a.ctypes.data))


def decode_rgb(x):
    o = np.zeros(3, np.float32)
    lib().tt_oracle_decode_rgb(int(x), o.ctypes.data)
    return o


def hlsl_pow(x, y):
    return float(lib().tt_oracle_pow(float(x), float(y)))


def resolve_normals(scene, rays, n_rays, bounce, far_plane, width, height):
    L = lib()
    p = tthip.TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width,
                          screen_height=height, flags=0)
    out = np.zeros((n_rays, 6), np.float32)
    st = L.tt_oracle_resolve_normals(scene.tris.ctypes.data, len(scene.tris), scene.meshdata.ctypes.data,
                                     len(scene.meshdata), C.byref(p), rays.ctypes.data, out.ctypes.data)
    assert st == 0
    return out


def generate(cam_to_world, cam_inv_proj, width, height, near, far, jitter=0, frames=0, max_bounce=3):
    L = lib()
    rays = np.zeros(2 * width * height, tthip.RAY_DTYPE)
    c2w = tthip.unity_colmajor(cam_to_world)
    ip = tthip.unity_colmajor(cam_inv_proj)
    st = L.tt_oracle_generate(c2w.ctypes.data, ip.ctypes.data, width, height, near, far, jitter, frames,
                              max_bounce, rays.ctypes.data)
    assert st == 0
    return rays


def enqueue_bounce(scene, rays, n_rays, bounce, far_plane, width, height, frames=0, max_bounce=3):
    """Oracle diffuse-bounce enqueue in place on `rays` (2*W*H RayData); returns the survivor count."""
    L = lib()
    p = tthip.TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width,
                          screen_height=height, flags=0)
    n = C.c_uint32()
    st = L.tt_oracle_enqueue_diffuse_bounce(scene.tris.ctypes.data, len(scene.tris), scene.meshdata.ctypes.data,
                                            len(scene.meshdata), C.byref(p), rays.ctypes.data, frames, max_bounce,
                                            C.byref(n))
    assert st == 0, st
    return n.value


def sincos_pinned(phi):
    L = lib()
    s, c = C.c_float(), C.c_float()
    L.tt_oracle_sincos_pinned(float(phi), C.byref(s), C.byref(c))
    return s.value, c.value


def tlas_refit(scene: "tthip.Scene", mesh_aabbs: np.ndarray, n_tlas_nodes=None):
    """Oracle TLAS refit: returns (status, nodes) with nodes[0, n_tlas) rewritten."""
    nodes = scene.nodes.copy()
    n = scene.tlas_nodes if n_tlas_nodes is None else n_tlas_nodes
    boxes = np.ascontiguousarray(mesh_aabbs, np.float32)
    st = lib().tt_oracle_tlas_refit(nodes.ctypes.data, n, scene.tlas.ctypes.data, len(scene.tlas), boxes.ctypes.data,
                                    boxes.shape[0])
    return st, nodes


def blas_refit(scene: "tthip.Scene", mesh_index: int, vertices: np.ndarray, indices: np.ndarray,
               leaf_of_triangle: np.ndarray, transform=None):
    """Oracle BLAS refit (ParentObject.RefitMesh): returns (status, nodes, tris) with the mesh's
    triangles and BLAS nodes rewritten."""
    nodes, tris = scene.nodes.copy(), scene.tris.copy()
    v = np.ascontiguousarray(vertices, np.float32)
    idx = np.ascontiguousarray(indices, np.int32).reshape(-1)
    leaf = np.ascontiguousarray(leaf_of_triangle, np.int32)
    m = tthip.unity_colmajor(np.eye(4) if transform is None else np.asarray(transform))
    st = lib().tt_oracle_blas_refit(nodes.ctypes.data, len(nodes), tris.ctypes.data, len(tris),
                                    scene.meshdata.ctypes.data, len(scene.meshdata), mesh_index, v.ctypes.data,
                                    v.shape[0], v.shape[1], idx.ctypes.data, len(idx) // 3, leaf.ctypes.data,
                                    m.ctypes.data)
    return st, nodes, tris
