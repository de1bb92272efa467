"""tthip — Python (ctypes) view of the C ABI in include/truetrace_hip.h and
include/truetrace_scene.h.

The product is the C-ABI library ``lib/libtruetrace_hip.so`` (gfx950 kernels); this module is
thin plumbing so tests and bench.py can drive it. It never falls back to a CPU path: if the
HIP library is missing or no GPU is visible, the trace entry points raise.

Names mirror the reference dispatch surface:
  * ``AssetManager`` — owns the aggregated buffers (AssetManager.cs:75-88 SetMeshTraceBuffers,
    :986-1227 AccumulateData, :1610-1766 UpdateTLAS) and uploads them (tt_scene_upload);
  * ``Engine.trace`` — one ``kernel_trace`` dispatch (RayTracingMaster.cs:964-970).
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_DIR, "lib")

# ---------------------------------------------------------------- status codes
TT_OK = 0
TT_ERR_INVALID_ARG = 1
TT_ERR_OOM = 2
TT_ERR_HIP = 3
TT_ERR_UNSUPPORTED = 4
TT_ERR_STACK_OVERFLOW = 5
TT_ERR_NO_DEVICE = 6
TT_ERR_NO_SCENE = 7
STATUS_NAMES = {0: "TT_OK", 1: "TT_ERR_INVALID_ARG", 2: "TT_ERR_OOM", 3: "TT_ERR_HIP", 4: "TT_ERR_UNSUPPORTED",
                5: "TT_ERR_STACK_OVERFLOW", 6: "TT_ERR_NO_DEVICE", 7: "TT_ERR_NO_SCENE"}

TT_TRACE_DEVICE_PTRS = 1 << 0
TT_TRACE_USE_RESTIRGI = 1 << 1
TT_TRACE_USE_ASVGF = 1 << 2
TT_TRACE_STATS = 1 << 3
TT_TRACE_ASYNC = 1 << 4
TT_TRACE_IGNORE_GLASS = 1 << 5       # IgnoreGlassMain (IntersectionKernels.compute:42-44)
TT_TRACE_IGNORE_BACKFACING = 1 << 6  # IgnoreBackfacing (IntersectionKernels.compute:45-47)
TT_TRACE_ADAPTIVE_ORDER = 1 << 7  # dequeue the previous launch's costliest tiles first (tt_order.hip)
TT_SHADOW_RADIANCE_CACHE = 1 << 7    # RadianceCache define (GlobalDefines.cginc:15) for tt_trace_shadow_ex
TT_SHADOW_VISIBILITY_CHECK = 1 << 8  # VisabilityCheckCompute semantics (CommonData.cginc:710-819)
TT_STACK_SIZE = 16
TT_MAX_REPS = 1000

# ---------------------------------------------------------------- numpy layouts
NODE_DTYPE = np.dtype([("p", "<f4", 3), ("e_imask", "<u4"), ("base_child", "<u4"), ("base_tri", "<u4"),
                       ("meta", "<u4", 2), ("qlo_x", "<u4", 2), ("qhi_x", "<u4", 2), ("qlo_y", "<u4", 2),
                       ("qhi_y", "<u4", 2), ("qlo_z", "<u4", 2), ("qhi_z", "<u4", 2)])
TRI_DTYPE = np.dtype([("pos0", "<f4", 3), ("posedge1", "<f4", 3), ("posedge2", "<f4", 3), ("norms", "<u4", 3),
                      ("tans", "<u4", 3), ("tex0", "<f4", 2), ("texedge1", "<f4", 2), ("texedge2", "<f4", 2),
                      ("MatDat", "<u4")])
MESH_DTYPE = np.dtype([("W2L", "<f4", 16), ("TriOffset", "<i4"), ("NodeOffset", "<i4"), ("MaterialOffset", "<i4"),
                       ("mesh_data_bvh_offsets", "<i4"), ("LightTriCount", "<i4"), ("LightNodeOffset", "<i4")])
MAT_DTYPE = np.dtype([("AlbedoTex", "<i4", 2), ("NormalTex", "<i4", 2), ("EmissiveTex", "<i4", 2),
                      ("MetallicTex", "<i4", 2), ("RoughnessTex", "<i4", 2), ("AlphaTex", "<i4", 2),
                      ("MatCapMask", "<i4", 2), ("MatCapTex", "<i4", 2), ("surfaceColor", "<f4", 3),
                      ("emmissive", "<f4"), ("EmissionColor", "<f4", 3), ("Tag", "<u4"), ("roughness", "<f4"),
                      ("MatType", "<i4"), ("transmittanceColor", "<f4", 3), ("ior", "<f4"), ("metallic", "<f4"),
                      ("sheen", "<f4"), ("sheenTint", "<f4"), ("specularTint", "<f4"), ("clearcoat", "<f4"),
                      ("clearcoatGloss", "<f4"), ("anisotropic", "<f4"), ("flatness", "<f4"), ("diffTrans", "<f4"),
                      ("specTrans", "<f4"), ("Specular", "<f4"), ("scatterDistance", "<f4"),
                      ("AlbedoTexScale", "<f4", 4), ("MetallicRemap", "<f4", 2), ("RoughnessRemap", "<f4", 2),
                      ("AlphaCutoff", "<f4"), ("NormalStrength", "<f4"), ("Hue", "<f4"), ("Saturation", "<f4"),
                      ("Contrast", "<f4"), ("Brightness", "<f4"), ("BlendColor", "<f4", 3), ("BlendFactor", "<f4"),
                      ("SecondaryTexScale", "<f4", 2), ("Rotation", "<f4")])
RAY_DTYPE = np.dtype([("origin", "<f4", 3), ("PixelIndex", "<u4"), ("direction", "<f4", 3), ("last_pdf", "<f4"),
                      ("hits", "<u4", 4)])
COL_DTYPE = np.dtype([("throughput", "<f4", 3), ("Direct", "<f4", 3), ("Indirect", "<f4", 3),
                      ("PrimaryNEERay", "<u4"), ("Flags", "<u4"), ("MetRoughIsSpec", "<u4"), ("Data", "<f4", 4)])
for _dt, _sz in ((NODE_DTYPE, 80), (TRI_DTYPE, 88), (MESH_DTYPE, 88), (MAT_DTYPE, 252), (RAY_DTYPE, 48),
                 (COL_DTYPE, 64)):
    assert _dt.itemsize == _sz, (_dt, _sz)
assert MAT_DTYPE.fields["Tag"][1] == 92 and MAT_DTYPE.fields["MatType"][1] == 100
assert MAT_DTYPE.fields["AlbedoTexScale"][1] == 168 and MAT_DTYPE.fields["AlphaCutoff"][1] == 200

MAT_CUTOUT_INDEX = 2
FLAG_INVISIBLE = 7


# ---------------------------------------------------------------- ctypes structs
# ShadowRayData (CommonData.cginc:116-123)
SHADOW_DTYPE = np.dtype([("origin", "<f4", 3), ("LuminanceIncomming", "<f4"), ("direction", "<f4", 3), ("t", "<f4"),
                         ("illumination", "<f4", 3), ("PixelIndex", "<u4")])
assert SHADOW_DTYPE.itemsize == 48
# PropogatedCacheData (CommonData.cginc:1621-1627, PropDepth 4): the RadianceCache record per pixel
CACHE_DTYPE = np.dtype([("samples", "<u4", (4, 2)), ("throughput", "<u4"), ("pathLength", "<u4"),
                        ("CurrentIlluminance", "<u4"), ("Norm", "<u4")])
assert CACHE_DTYPE.itemsize == 48 and CACHE_DTYPE.fields["CurrentIlluminance"][1] == 40
TT_FLAG_IS_BACKGROUND, TT_FLAG_SHADOW_CASTER = 5, 6


class ShadowParams(C.Structure):
    _fields_ = [("n_rays", C.c_uint32), ("bounce", C.c_int32), ("screen_width", C.c_uint32),
                ("screen_height", C.c_uint32), ("flags", C.c_uint32)]


class BlasRefitParams(C.Structure):
    _fields_ = [("mesh_index", C.c_uint32), ("n_tris", C.c_uint32), ("n_vertices", C.c_uint32),
                ("vertex_stride", C.c_uint32), ("transform", C.c_float * 16), ("flags", C.c_uint32)]


class TraceParams(C.Structure):
    _fields_ = [("n_rays", C.c_uint32), ("bounce", C.c_int32), ("far_plane", C.c_float),
                ("screen_width", C.c_uint32), ("screen_height", C.c_uint32), ("flags", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("blas_entries", C.c_uint64), ("hits", C.c_uint64), ("reps_exhausted", C.c_uint64),
                ("stack_overflows", C.c_uint64), ("accepts", C.c_uint64), ("kernel_ms", C.c_float),
                ("pad", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32), ("max_rays", C.c_uint64), ("stream", C.c_void_p)]


class Camera(C.Structure):
    _fields_ = [("cam_to_world", C.c_float * 16), ("cam_inv_proj", C.c_float * 16), ("near_plane", C.c_float),
                ("far_plane", C.c_float), ("width", C.c_uint32), ("height", C.c_uint32), ("jitter", C.c_int32),
                ("frames_accumulated", C.c_int32), ("max_bounce", C.c_int32), ("flags", C.c_uint32)]


class MeshInput(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("n_vertices", C.c_uint32), ("normals", C.c_void_p),
                ("tangents", C.c_void_p), ("uvs", C.c_void_p), ("indices", C.c_void_p), ("n_indices", C.c_uint32),
                ("matdat", C.c_void_p), ("lossy_scale", C.c_float * 3)]


class BlasInfo(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_tris", C.c_uint32), ("bvh2_depth", C.c_uint32),
                ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("build_seconds", C.c_double)]


class ParentDesc(C.Structure):
    _fields_ = [("blas", C.c_void_p), ("local_to_world", C.c_float * 16), ("world_to_local", C.c_float * 16),
                ("material_count", C.c_uint32)]


class InstanceDesc(C.Structure):
    _fields_ = [("instance_parent", C.c_uint32), ("local_to_world", C.c_float * 16),
                ("world_to_local", C.c_float * 16)]


class SceneBuildInfo(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_tris", C.c_uint32), ("n_tlas_indices", C.c_uint32),
                ("n_mesh", C.c_uint32), ("tlas_nodes", C.c_uint32), ("pad", C.c_uint32)]


class TTError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def _check(st: int, what: str):
    if st != TT_OK:
        raise TTError(st, what)


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"], "arrays passed to the C ABI must be contiguous"
        return a.ctypes.data
    if hasattr(a, "data_ptr"):  # torch tensor
        return a.data_ptr()
    return int(a)


# ---------------------------------------------------------------- library loading
_SCENE = None
_HIP = None

HIP_SYMBOLS = ["tt_abi_version", "tt_device_count", "tt_ctx_create", "tt_ctx_destroy", "tt_last_error",
               "tt_scene_upload", "tt_scene_update_nodes", "tt_scene_update_meshdata", "tt_scene_bytes",
               "tt_trace_closest", "tt_sync", "tt_ctx_stream", "tt_resolve_normals", "tt_generate_primary",
               "tt_enqueue_diffuse_bounce", "tt_trace_closest_indirect", "tt_enqueue_diffuse_bounce_indirect",
               "tt_trace_shadow_ex_indirect", "tt_timing_reset", "tt_timing_read", "tt_scene_validate", "tt_trace_diagnostics",
               "tt_selftest_rcp", "tt_trace_closest_hits", "tt_ctx_share_scene"]
SCENE_SYMBOLS = ["tt_blas_build", "tt_blas_get_info", "tt_blas_copy", "tt_blas_free", "tt_scene_assemble",
                 "tt_scene_build_get_info", "tt_scene_build_copy", "tt_scene_build_free", "tt_pack_octahedral",
                 "tt_bvh2_build", "tt_dotnet_sort_by_key", "tt_synth_cornell", "tt_synth_soup", "tt_synth_sponza",
                 "tt_synth_prop", "tt_synth_ground", "tt_synth_san_miguel", "tt_synth_mesh_view", "tt_synth_mesh_free",
                 "tt_synth_mesh_from_arrays", "tt_blas_copy_leaf_order", "tt_blas_prepare_aabbs", "tt_bvh2_presort",
                 "tt_blas_build_from_bvh2", "tt_blas_build_from_cwbvh", "tt_blas_prepare",
                 "tt_blas_build_from_cwbvh_prepared", "tt_blas_prep_free"]


def scene_lib():
    global _SCENE
    if _SCENE is None:
        path = os.path.join(LIB_DIR, "libtruetrace_scene.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C truetrace-unity-pathtracer_amd` or __graft_entry__.build()")
        L = C.CDLL(path)
        vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
        L.tt_blas_build.argtypes = [C.POINTER(MeshInput), C.POINTER(vp)]
        L.tt_blas_get_info.argtypes = [vp, C.POINTER(BlasInfo)]
        L.tt_blas_copy.argtypes = [vp, vp, vp]
        L.tt_blas_free.argtypes = [vp]
        L.tt_blas_free.restype = None
        L.tt_blas_copy_leaf_order.argtypes = [vp, vp]
        L.tt_blas_copy_leaf_order.restype = i32
        L.tt_scene_assemble.argtypes = [vp, u32, vp, u32, vp, u32, C.POINTER(vp)]
        L.tt_scene_build_get_info.argtypes = [vp, C.POINTER(SceneBuildInfo)]
        L.tt_scene_build_copy.argtypes = [vp, vp, vp, vp, vp]
        L.tt_scene_build_free.argtypes = [vp]
        L.tt_scene_build_copy_mesh_aabbs.argtypes = [vp, vp]
        L.tt_scene_build_free.restype = None
        L.tt_pack_octahedral.argtypes = [C.c_float, C.c_float, C.c_float]
        L.tt_pack_octahedral.restype = u32
        L.tt_bvh2_build.argtypes = [vp, u32, vp, vp, vp, vp]
        L.tt_blas_prepare_aabbs.argtypes = [C.POINTER(MeshInput), vp]
        L.tt_bvh2_presort.argtypes = [vp, u32, vp]
        L.tt_blas_build_from_bvh2.argtypes = [C.POINTER(MeshInput), vp, vp, vp, vp, u32, C.POINTER(vp)]
        L.tt_blas_build_from_cwbvh.argtypes = [C.POINTER(MeshInput), vp, u32, vp, u32, C.POINTER(vp)]
        L.tt_blas_prepare.argtypes = [C.POINTER(MeshInput), vp, C.POINTER(vp)]
        L.tt_blas_build_from_cwbvh_prepared.argtypes = [vp, vp, u32, vp, u32, C.POINTER(vp)]
        L.tt_blas_prep_free.argtypes = [vp]
        L.tt_blas_prep_free.restype = None
        L.tt_dotnet_sort_by_key.argtypes = [vp, u32, vp]
        L.tt_dotnet_sort_by_key.restype = None
        L.tt_synth_cornell.argtypes = [C.POINTER(vp)]
        L.tt_synth_soup.argtypes = [C.c_uint64, u32, C.c_float, C.c_float, C.POINTER(vp)]
        L.tt_synth_sponza.argtypes = [C.c_uint64, u32, C.POINTER(vp)]
        L.tt_synth_prop.argtypes = [C.c_uint64, u32, C.POINTER(vp)]
        L.tt_synth_ground.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, u32, u32, C.POINTER(vp)]
        L.tt_synth_san_miguel.argtypes = [C.c_uint64, u32, C.POINTER(vp)]
        L.tt_synth_mesh_view.argtypes = [vp, C.POINTER(MeshInput)]
        L.tt_synth_mesh_free.argtypes = [vp]
        L.tt_synth_mesh_free.restype = None
        L.tt_synth_mesh_from_arrays.argtypes = [vp, u32, vp, u32, vp]
        L.tt_synth_mesh_from_arrays.restype = vp
        for s in ["tt_blas_build", "tt_blas_get_info", "tt_blas_copy", "tt_scene_assemble", "tt_scene_build_get_info",
                  "tt_scene_build_copy", "tt_bvh2_build", "tt_synth_cornell", "tt_synth_soup", "tt_synth_sponza",
                  "tt_synth_prop", "tt_synth_ground", "tt_synth_san_miguel", "tt_synth_mesh_view"]:
            getattr(L, s).restype = i32
        _SCENE = L
    return _SCENE


def hip_lib():
    """The gfx950 engine. Raises if the library was not built — there is no CPU fallback."""
    global _HIP
    if _HIP is None:
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME libamdhip64.so.7). Load it
        # first so our NEEDED libamdhip64.so.7 binds to that same runtime: two HIP/HSA runtimes in one
        # process break torch.cuda / RCCL. Without torch the system ROCm runtime is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get("TT_HIP_LIB") or os.path.join(LIB_DIR, "libtruetrace_hip.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: the HIP engine was not built (no fallback exists)")
        L = C.CDLL(path)
        vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
        L.tt_abi_version.restype = i32
        L.tt_device_count.restype = i32
        L.tt_ctx_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
        L.tt_ctx_destroy.argtypes = [vp]
        L.tt_last_error.argtypes = [vp]
        L.tt_last_error.restype = C.c_char_p
        L.tt_scene_upload.argtypes = [vp, vp, u32, vp, u32, vp, u32, vp, u32, vp, u32]
        L.tt_scene_update_nodes.argtypes = [vp, u32, u32, vp]
        L.tt_scene_update_meshdata.argtypes = [vp, u32, u32, vp]
        L.tt_scene_bytes.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.tt_trace_closest.argtypes = [vp, C.POINTER(TraceParams), vp, vp, vp, C.POINTER(Stats)]
        L.tt_trace_shadow.argtypes = [vp, C.POINTER(ShadowParams), vp, vp, vp, vp, C.POINTER(Stats)]
        L.tt_trace_shadow_ex.argtypes = [vp, C.POINTER(ShadowParams), vp, vp, vp, vp, vp, C.POINTER(Stats)]
        if hasattr(L, "tt_trace_closest_indirect"):  # (absent from round-2 variant libraries, tools/run_variants.py)
            L.tt_trace_closest_indirect.argtypes = [vp, C.POINTER(TraceParams), vp, vp, vp, vp]
            L.tt_trace_shadow_ex_indirect.argtypes = [vp, C.POINTER(ShadowParams), vp, vp, vp, vp, vp, vp]
            L.tt_enqueue_diffuse_bounce_indirect.argtypes = [vp, C.POINTER(TraceParams), vp, vp, i32, i32, vp]
        if hasattr(L, "tt_ctx_share_scene"):
            L.tt_ctx_share_scene.argtypes = [vp, vp]
        if hasattr(L, "tt_ctx_share_blas"):
            L.tt_ctx_share_blas.argtypes = [vp, vp, u32]
        if hasattr(L, "tt_trace_chunk_costs"):
            L.tt_trace_chunk_costs.argtypes = [vp, i32, vp, u32, C.POINTER(u32)]
            L.tt_trace_chunk_costs.restype = i32
        if hasattr(L, "tt_trace_closest_hits"):
            L.tt_trace_closest_hits.argtypes = [vp, C.POINTER(TraceParams), vp, vp, vp, vp]
        L.tt_scene_upload_alpha_atlas.argtypes = [vp, vp, u32, u32]
        L.tt_scene_upload_texture_atlas.argtypes = [vp, vp, u32, u32]
        L.tt_tlas_refit.argtypes = [vp, u32, vp, u32, u32]
        L.tt_scene_read_nodes.argtypes = [vp, u32, u32, vp]
        L.tt_scene_read_tris.argtypes = [vp, u32, u32, vp]
        L.tt_blas_refit.argtypes = [vp, C.POINTER(BlasRefitParams), vp, vp, vp]
        L.tt_bvh2_build_device.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp, C.POINTER(u32)]
        L.tt_blas_build_device.argtypes = [vp, vp, u32, vp, vp, u32, C.POINTER(u32), vp, C.POINTER(u32)]
        L.tt_bvh2_presort_device.argtypes = [vp, vp, u32, vp]
        L.tt_sync.argtypes = [vp]
        if hasattr(L, "tt_stream_create"):
            L.tt_stream_create.argtypes = [i32, C.POINTER(vp)]
            L.tt_stream_create.restype = i32
            L.tt_stream_destroy.argtypes = [vp]
            L.tt_stream_destroy.restype = i32
        if hasattr(L, "tt_stream_live_count"):
            L.tt_stream_live_count.restype = u32
        L.tt_async_overflows.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.tt_ctx_stream.argtypes = [vp]
        L.tt_ctx_stream.restype = vp
        L.tt_resolve_normals.argtypes = [vp, C.POINTER(TraceParams), vp, vp]
        L.tt_generate_primary.argtypes = [vp, C.POINTER(Camera), vp]
        L.tt_enqueue_diffuse_bounce.argtypes = [vp, C.POINTER(TraceParams), vp, i32, i32, C.POINTER(u32)]
        L.tt_scene_validate.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, vp, u32, C.c_char_p, u32]
        L.tt_scene_validate.restype = i32
        L.tt_trace_diagnostics.argtypes = [vp, vp]
        L.tt_trace_diagnostics.restype = i32
        L.tt_selftest_rcp.argtypes = [vp, vp]
        L.tt_selftest_rcp.restype = i32
        L.tt_timing_reset.argtypes = [vp]
        L.tt_timing_read.argtypes = [vp, vp, u32, C.POINTER(u32)]
        L.tt_ctx_set_timing.argtypes = [vp, i32]
        L.tt_ctx_set_timing.restype = i32
        L.tt_ctx_set_frame_pixels.argtypes = [vp, C.c_uint32]
        L.tt_ctx_set_frame_pixels.restype = i32
        for s in ["tt_ctx_create", "tt_ctx_destroy", "tt_scene_upload", "tt_scene_update_nodes",
                  "tt_scene_update_meshdata", "tt_scene_bytes", "tt_trace_closest", "tt_sync", "tt_resolve_normals",
                  "tt_generate_primary", "tt_enqueue_diffuse_bounce", "tt_timing_reset", "tt_timing_read"]:
            getattr(L, s).restype = i32
        if hasattr(L, "tt_group_create"):  # (absent from older variant libraries)
            _bind_group(L)
        _HIP = L
    return _HIP


# ---------------------------------------------------------------- matrices
def trs_matrix(translation=(0, 0, 0), rotation_y_deg=0.0, scale=1.0) -> np.ndarray:
    """4x4 localToWorld (row-major numpy, math convention) of a rigid + uniform scale transform."""
    a = np.deg2rad(rotation_y_deg)
    c, s = np.cos(a), np.sin(a)
    m = np.eye(4)
    m[:3, :3] = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]]) * scale
    m[:3, 3] = translation
    return m


def unity_colmajor(m: np.ndarray) -> np.ndarray:
    """Unity stores Matrix4x4 column-major: element (r, c) at [c*4 + r]."""
    return np.asarray(m, dtype=np.float64).T.reshape(16).astype(np.float32)


def unity_camera(position, forward, up, vfov_deg, width, height, near=0.3, far=1000.0):
    """(cameraToWorldMatrix, projectionMatrix.inverse) as Unity computes them (OpenGL conventions:
    camera looks down -z in camera space)."""
    f = np.asarray(forward, np.float64)
    f = f / np.linalg.norm(f)
    r = np.cross(np.asarray(up, np.float64), f)  # Unity is left-handed: right = up x forward
    r = r / np.linalg.norm(r)
    u = np.cross(f, r)
    l2w = np.eye(4)
    l2w[:3, 0], l2w[:3, 1], l2w[:3, 2], l2w[:3, 3] = r, u, f, position
    c2w = l2w @ np.diag([1.0, 1.0, -1.0, 1.0])
    aspect = width / height
    ft = 1.0 / np.tan(np.deg2rad(vfov_deg) / 2.0)
    P = np.zeros((4, 4))
    P[0, 0], P[1, 1] = ft / aspect, ft
    P[2, 2], P[2, 3] = (far + near) / (near - far), 2 * far * near / (near - far)
    P[3, 2] = -1.0
    return c2w, np.linalg.inv(P)


# ---------------------------------------------------------------- scene building
class Mesh:
    """A ParentObject's merged object-space mesh (owned by the scene library)."""

    def __init__(self, handle: int):
        self.h = handle

    @staticmethod
    def _check(st, what):
        if st != TT_OK:
            raise TTError(st, what)

    @classmethod
    def cornell(cls) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_cornell(C.byref(h)), "tt_synth_cornell")
        return cls(h.value)

    @classmethod
    def soup(cls, seed: int, n_tris: int, extent: float = 1.0, tri_size: float = 0.1) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_soup(seed, n_tris, extent, tri_size, C.byref(h)), "tt_synth_soup")
        return cls(h.value)

    @classmethod
    def sponza(cls, seed: int = 0x53504F4E, n_tris: int = 262267) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_sponza(seed, n_tris, C.byref(h)), "tt_synth_sponza")
        return cls(h.value)

    @classmethod
    def prop(cls, seed: int, n_tris: int) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_prop(seed, n_tris, C.byref(h)), "tt_synth_prop")
        return cls(h.value)

    @classmethod
    def ground(cls, x0: float, x1: float, z0: float, z1: float, nu: int, nv: int) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_ground(x0, x1, z0, z1, nu, nv, C.byref(h)), "tt_synth_ground")
        return cls(h.value)

    @classmethod
    def san_miguel(cls, seed: int = 0x5A4E4D, n_tris: int = 10_000_000) -> "Mesh":
        h = C.c_void_p()
        cls._check(scene_lib().tt_synth_san_miguel(seed, n_tris, C.byref(h)), "tt_synth_san_miguel")
        return cls(h.value)

    @classmethod
    def from_arrays(cls, positions: np.ndarray, indices: np.ndarray, matdat: Optional[np.ndarray] = None) -> "Mesh":
        pos = np.ascontiguousarray(positions, np.float32).reshape(-1)
        idx = np.ascontiguousarray(indices, np.int32).reshape(-1)
        md = None if matdat is None else np.ascontiguousarray(matdat, np.int32)
        h = scene_lib().tt_synth_mesh_from_arrays(pos.ctypes.data, pos.size // 3, idx.ctypes.data, idx.size,
                                                  None if md is None else md.ctypes.data)
        if not h:
            raise TTError(TT_ERR_OOM, "tt_synth_mesh_from_arrays")
        return cls(h)

    def arrays(self):
        """(positions (n,3), normals (n,3), indices (3*tris,)) copies of the mesh."""
        v = self.view()
        n, k = v.n_vertices, v.n_indices
        fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int32)
        pos = np.ctypeslib.as_array(C.cast(v.positions, fp), (3 * n,)).reshape(n, 3).copy()
        nrm = (np.ctypeslib.as_array(C.cast(v.normals, fp), (3 * n,)).reshape(n, 3).copy() if v.normals
               else np.tile(np.float32([0, 1, 0]), (n, 1)))
        idx = np.ctypeslib.as_array(C.cast(v.indices, ip), (k,)).copy()
        return pos, nrm, idx

    def view(self) -> MeshInput:
        v = MeshInput()
        self._check(scene_lib().tt_synth_mesh_view(self.h, C.byref(v)), "tt_synth_mesh_view")
        v._owner = self  # the view points into this mesh's native arrays: it keeps the mesh alive
        return v

    def __del__(self):
        if getattr(self, "h", None) and _SCENE is not None:
            _SCENE.tt_synth_mesh_free(self.h)
            self.h = None


_BUILD_ENGINE = None
_BUILD_MIN_TRIS = 0


def set_build_engine(engine: "Engine" = None, min_tris: int = 100_000):
    """Route every later Blas(mesh) of at least ``min_tris`` triangles through ``engine``'s GPU
    (tt_blas_build_device; byte-identical to the host build). None: host builds again."""
    global _BUILD_ENGINE, _BUILD_MIN_TRIS
    _BUILD_ENGINE, _BUILD_MIN_TRIS = engine, int(min_tris)


class Blas:
    """A built ParentObject: CWBVH8 nodes + leaf-ordered CudaTriangles (ParentObject.BuildTotal)."""

    def __init__(self, mesh: Mesh, lossy_scale=(1.0, 1.0, 1.0), engine: "Engine" = None, timings: dict = None,
                 device_stages: str = "bvh2+bvh8"):
        """engine: build on that engine's GPU after the host's presort -- device_stages "bvh2+bvh8"
        (tt_blas_build_device) or "bvh2" (tt_bvh2_build_device, BVH8 on the host); either way the
        result is byte-identical to the host build. timings (dict): the stage times in seconds."""
        v = mesh.view()
        v.lossy_scale[:] = lossy_scale
        h = C.c_void_p()
        L = scene_lib()
        if engine is None and _BUILD_ENGINE is not None and v.n_indices // 3 >= _BUILD_MIN_TRIS:
            engine = _BUILD_ENGINE
        if engine is None:
            st = L.tt_blas_build(C.byref(v), C.byref(h))
            if st != TT_OK:
                raise TTError(st, "tt_blas_build")
        else:
            import time
            t0 = time.perf_counter()
            n = v.n_indices // 3
            aabbs = np.zeros((n, 6), np.float32)
            prep = C.c_void_p()  # the prepared triangles, kept for the final assembly (bvh2+bvh8)
            if device_stages == "bvh2+bvh8":
                _check(L.tt_blas_prepare(C.byref(v), aabbs.ctypes.data, C.byref(prep)), "tt_blas_prepare")
            else:
                _check(L.tt_blas_prepare_aabbs(C.byref(v), aabbs.ctypes.data), "tt_blas_prepare_aabbs")
            t1 = time.perf_counter()
            pre = np.zeros((3, n), np.int32)
            if engine.L.tt_bvh2_presort_device(engine.h, aabbs.ctypes.data, n, pre.ctypes.data) != TT_OK:
                st = L.tt_bvh2_presort(aabbs.ctypes.data, n, pre.ctypes.data)
                if st != TT_OK:
                    if prep:
                        L.tt_blas_prep_free(prep)
                    raise TTError(st, "tt_bvh2_presort")
            t2 = time.perf_counter()
            if device_stages == "bvh2+bvh8":
                cap = max(1, n - 1)
                nodes = np.zeros(cap, NODE_DTYPE)
                cw = np.zeros(n, np.int32)
                nn, depth = C.c_uint32(0), C.c_uint32(0)
                st = engine.L.tt_blas_build_device(engine.h, aabbs.ctypes.data, n, pre.ctypes.data, nodes.ctypes.data,
                                                   cap, C.byref(nn), cw.ctypes.data, C.byref(depth))
                if st != TT_OK:
                    L.tt_blas_prep_free(prep)
                    raise TTError(st, "tt_blas_build_device")
                t3 = time.perf_counter()
                _check(L.tt_blas_build_from_cwbvh_prepared(prep, nodes.ctypes.data, nn.value, cw.ctypes.data,
                                                           depth.value, C.byref(h)),
                       "tt_blas_build_from_cwbvh_prepared")  # consumes prep
                if timings is not None:
                    timings.update(prepare_s=t1 - t0, presort_s=t2 - t1, device_s=t3 - t2,
                                   assemble_s=time.perf_counter() - t3)
                self.h = h.value
                info = BlasInfo()
                L.tt_blas_get_info(self.h, C.byref(info))
                self.info = info
                return
            fi = np.zeros(n, np.int32)
            boxes = np.zeros((2 * n, 6), np.float32)
            left = np.zeros(2 * n, np.int32)
            count = np.zeros(2 * n, np.uint32)
            depth = C.c_uint32(0)
            st = engine.L.tt_bvh2_build_device(engine.h, aabbs.ctypes.data, n, pre.ctypes.data, fi.ctypes.data,
                                               boxes.ctypes.data, left.ctypes.data, count.ctypes.data, C.byref(depth))
            if st != TT_OK:
                raise TTError(st, "tt_bvh2_build_device")
            t3 = time.perf_counter()
            _check(L.tt_blas_build_from_bvh2(C.byref(v), fi.ctypes.data, boxes.ctypes.data, left.ctypes.data,
                                             count.ctypes.data, depth.value, C.byref(h)), "tt_blas_build_from_bvh2")
            if timings is not None:
                timings.update(prepare_s=t1 - t0, presort_s=t2 - t1, bvh2_device_s=t3 - t2,
                               bvh8_s=time.perf_counter() - t3)
        self.h = h.value
        info = BlasInfo()
        L.tt_blas_get_info(self.h, C.byref(info))
        self.info = info

    @property
    def n_nodes(self):
        return self.info.n_nodes

    @property
    def n_tris(self):
        return self.info.n_tris

    def leaf_order(self) -> np.ndarray:
        """CWBVHIndicesBufferInverted: source triangle -> position in the leaf-ordered triangles."""
        out = np.zeros(self.info.n_tris, np.int32)
        scene_lib().tt_blas_copy_leaf_order(self.h, out.ctypes.data)
        return out

    def arrays(self):
        nodes = np.zeros(self.info.n_nodes, NODE_DTYPE)
        tris = np.zeros(self.info.n_tris, TRI_DTYPE)
        scene_lib().tt_blas_copy(self.h, nodes.ctypes.data, tris.ctypes.data)
        return nodes, tris

    def __del__(self):
        if getattr(self, "h", None) and _SCENE is not None:
            _SCENE.tt_blas_free(self.h)
            self.h = None


@dataclass
class Scene:
    """Aggregated trace buffers exactly as AssetManager.SetMeshTraceBuffers binds them."""
    nodes: np.ndarray
    tris: np.ndarray
    tlas: np.ndarray
    meshdata: np.ndarray
    materials: np.ndarray
    tlas_nodes: int = 0
    meta: dict = field(default_factory=dict)
    alpha_atlas: Optional[np.ndarray] = None  # _AlphaAtlas, uint8 [height, width] (Cutout materials)
    texture_atlas: Optional[np.ndarray] = None  # _TextureAtlas decoded, float16 [height, width, 4] (glass)

    def save(self, path: str):
        np.savez_compressed(path, nodes=self.nodes.view(np.uint8), tris=self.tris.view(np.uint8),
                            tlas=self.tlas, meshdata=self.meshdata.view(np.uint8),
                            materials=self.materials.view(np.uint8), tlas_nodes=np.int64(self.tlas_nodes))

    @classmethod
    def load(cls, path: str) -> "Scene":
        z = np.load(path, allow_pickle=False)
        return cls(nodes=z["nodes"].view(NODE_DTYPE).copy(), tris=z["tris"].view(TRI_DTYPE).copy(),
                   tlas=z["tlas"].astype(np.int32), meshdata=z["meshdata"].view(MESH_DTYPE).copy(),
                   materials=z["materials"].view(MAT_DTYPE).copy(), tlas_nodes=int(z["tlas_nodes"]))


class AssetManager:
    """Host mirror of the reference AssetManager's aggregation (AccumulateData + UpdateTLAS +
    ConstructNewTLAS): RenderQue parents, InstanceData parents and InstancedObjects."""

    def __init__(self):
        self.parents: List = []          # (Blas, l2w 4x4, material_count)
        self.instance_parents: List = []  # (Blas, material_count)
        self.instances: List = []        # (instance_parent index, l2w 4x4)
        self.materials: List[np.ndarray] = []

    def add_parent(self, blas: Blas, local_to_world=None, materials: Optional[np.ndarray] = None):
        mats = materials if materials is not None else np.zeros(1, MAT_DTYPE)
        self.parents.append((blas, np.eye(4) if local_to_world is None else np.asarray(local_to_world), len(mats)))
        self.materials.append(mats)

    def add_instance_parent(self, blas: Blas, materials: Optional[np.ndarray] = None) -> int:
        mats = materials if materials is not None else np.zeros(1, MAT_DTYPE)
        self.instance_parents.append((blas, len(mats)))
        self._ip_mats = getattr(self, "_ip_mats", [])
        self._ip_mats.append(mats)
        return len(self.instance_parents) - 1

    def add_instance(self, parent_index: int, local_to_world):
        self.instances.append((parent_index, np.asarray(local_to_world)))

    def build(self) -> Scene:
        P = (ParentDesc * max(1, len(self.parents)))()
        for i, (b, l2w, nm) in enumerate(self.parents):
            P[i].blas = b.h
            P[i].local_to_world[:] = unity_colmajor(l2w)
            P[i].world_to_local[:] = unity_colmajor(np.linalg.inv(l2w))
            P[i].material_count = nm
        IP = (ParentDesc * max(1, len(self.instance_parents)))()
        for i, (b, nm) in enumerate(self.instance_parents):
            IP[i].blas = b.h
            IP[i].local_to_world[:] = unity_colmajor(np.eye(4))
            IP[i].world_to_local[:] = unity_colmajor(np.eye(4))
            IP[i].material_count = nm
        I = (InstanceDesc * max(1, len(self.instances)))()
        for i, (pi, l2w) in enumerate(self.instances):
            I[i].instance_parent = pi
            I[i].local_to_world[:] = unity_colmajor(l2w)
            I[i].world_to_local[:] = unity_colmajor(np.linalg.inv(l2w))
        h = C.c_void_p()
        L = scene_lib()
        st = L.tt_scene_assemble(C.addressof(P), len(self.parents), C.addressof(IP), len(self.instance_parents),
                                 C.addressof(I), len(self.instances), C.byref(h))
        if st != TT_OK:
            raise TTError(st, "tt_scene_assemble")
        try:
            info = SceneBuildInfo()
            L.tt_scene_build_get_info(h, C.byref(info))
            nodes = np.zeros(info.n_nodes, NODE_DTYPE)
            tris = np.zeros(info.n_tris, TRI_DTYPE)
            tlas = np.zeros(info.n_tlas_indices, np.int32)
            md = np.zeros(info.n_mesh, MESH_DTYPE)
            L.tt_scene_build_copy(h, nodes.ctypes.data, tris.ctypes.data, tlas.ctypes.data, md.ctypes.data)
            aabbs = np.zeros((info.n_mesh, 6), np.float32)
            L.tt_scene_build_copy_mesh_aabbs(h, aabbs.ctypes.data)
        finally:
            L.tt_scene_build_free(h)
        mats = self.materials + getattr(self, "_ip_mats", [])
        materials = np.concatenate(mats) if mats else np.zeros(1, MAT_DTYPE)
        return Scene(nodes, tris, tlas, md, materials, tlas_nodes=info.tlas_nodes, meta={"mesh_aabbs": aabbs})


def single_object_scene(mesh: Mesh, local_to_world=None, n_materials: int = 8) -> Scene:
    am = AssetManager()
    am.add_parent(Blas(mesh), local_to_world, np.zeros(n_materials, MAT_DTYPE))
    return am.build()


# ---------------------------------------------------------------- ray buffers
def camera_rays_host(cam_to_world: np.ndarray, cam_inv_proj: np.ndarray, width: int, height: int,
                     near: float, far: float) -> np.ndarray:
    """Vectorised float32 restatement of Generate for tests without a GPU (pinned like the
    kernel up to normalize's rounding; parity tests use rays from one source on both sides)."""
    c2w = unity_colmajor(cam_to_world).reshape(4, 4).T.astype(np.float32)
    ip = unity_colmajor(cam_inv_proj).reshape(4, 4).T.astype(np.float32)
    ys, xs = np.meshgrid(np.arange(height, dtype=np.float32), np.arange(width, dtype=np.float32), indexing="ij")
    uvx = xs / np.float32(width) * np.float32(2) - np.float32(1)
    uvy = ys / np.float32(height) * np.float32(2) - np.float32(1)
    d = np.stack([ip[r, 0] * uvx + ip[r, 1] * uvy + ip[r, 3] for r in range(3)], -1).astype(np.float32)
    d = np.stack([c2w[r, 0] * d[..., 0] + c2w[r, 1] * d[..., 1] + c2w[r, 2] * d[..., 2] for r in range(3)], -1)
    d = (d / np.sqrt((d * d).sum(-1, keepdims=True))).astype(np.float32)
    o = c2w[:3, 3].astype(np.float32)
    rays = np.zeros(2 * width * height, RAY_DTYPE)
    prim = rays[: width * height]
    prim["origin"] = (o + np.float32(near) * d).reshape(-1, 3)
    prim["direction"] = d.reshape(-1, 3)
    prim["PixelIndex"] = np.arange(width * height, dtype=np.uint32)
    prim["hits"][:, 2] = np.array([far], np.float32).view(np.uint32)[0]
    return rays


# ---------------------------------------------------------------- engine
class Engine:
    """One context per GPU (tt_ctx_create). ``trace`` is the kernel_trace dispatch."""

    def __init__(self, device: int = 0, max_rays: int = 0, stream: Optional[int] = None):
        L = hip_lib()
        cfg = Config(device=device, flags=0, max_rays=max_rays, stream=stream)
        h = C.c_void_p()
        st = L.tt_ctx_create(C.byref(cfg), C.byref(h))
        if st != TT_OK:
            raise TTError(st, "tt_ctx_create (no GPU visible?)")
        self.L, self.h = L, h.value
        _ENGINES.add(self)

    def _check(self, st, what):
        if st != TT_OK:
            raise TTError(st, f"{what}: {self.L.tt_last_error(self.h).decode()}")

    def _unlink_lender(self):
        """Drops this engine from its lender's borrower list (re-share or close)."""
        lender = getattr(self, "_lender", None)
        if lender is not None:
            lender._borrowers = [r for r in getattr(lender, "_borrowers", []) if r() is not None and r() is not self]
        self._lender = None

    def close(self):
        if getattr(self, "h", None):
            for b in list(getattr(self, "_borrowers", [])):  # contexts tracing this one's scene go first
                e = b()
                if e is not None:
                    e.close()
            self._borrowers = []
            self._unlink_lender()
            self.L.tt_ctx_destroy(self.h)
            self.h = None

    def share_scene(self, src: "Engine"):
        """tt_ctx_share_scene: trace `src`'s scene (its device buffers, no copy) on this context's stream."""
        import weakref

        self._check(self.L.tt_ctx_share_scene(self.h, src.h), "tt_ctx_share_scene")
        self._unlink_lender()  # a re-share leaves the previous lender's list
        self._lender = src  # keeps the lender alive while this context reads its buffers
        if not hasattr(src, "_borrowers"):
            src._borrowers = []
        src._borrowers.append(weakref.ref(self))

    def chunk_costs(self, bounce: int = 0, max_chunks: int = 1 << 22) -> np.ndarray:
        """tt_trace_chunk_costs: the last TT_TRACE_ADAPTIVE_ORDER launch's per-64-ray-chunk costs (max Reps;
        full-frame launches: one per 8x8 pixel tile, row-major over the (W/8) x (H/8) tile grid)."""
        out = np.zeros(max_chunks, np.uint32)
        n = C.c_uint32()
        self._check(self.L.tt_trace_chunk_costs(self.h, int(bounce), out.ctypes.data, max_chunks, C.byref(n)),
                    "tt_trace_chunk_costs")
        return out[: n.value].copy()

    def share_blas(self, src: "Engine", n_tlas_nodes: int):
        """tt_ctx_share_blas: a frame slot over `src`'s scene -- src's BLASes and triangles (no copy) under a TLAS,
        TLASBVH8Indices and _MeshData of this context's own (copied from src now), which tlas_refit /
        update_meshdata / update_nodes on this context change without waiting for src or other slots."""
        import weakref

        self._check(self.L.tt_ctx_share_blas(self.h, src.h, int(n_tlas_nodes)), "tt_ctx_share_blas")
        self._unlink_lender()
        self._lender = src
        if not hasattr(src, "_borrowers"):
            src._borrowers = []
        src._borrowers.append(weakref.ref(self))

    __del__ = close

    @property
    def stream(self) -> int:
        return self.L.tt_ctx_stream(self.h)

    def upload(self, s: Scene):
        """AssetManager.SetMeshTraceBuffers — copies the aggregated buffers into HBM."""
        st = self.L.tt_scene_upload(self.h, _ptr(s.nodes), len(s.nodes), _ptr(s.tris), len(s.tris), _ptr(s.tlas),
                                    len(s.tlas), _ptr(s.meshdata), len(s.meshdata), _ptr(s.materials),
                                    len(s.materials))
        self._check(st, "tt_scene_upload")
        if s.alpha_atlas is not None:
            self.upload_alpha_atlas(s.alpha_atlas)
        if s.texture_atlas is not None:
            self.upload_texture_atlas(s.texture_atlas)

    def upload_alpha_atlas(self, atlas: np.ndarray):
        """_AlphaAtlas (AssetManager.cs:260-262): R8 texels, row 0 = v in [0, 1/height)."""
        a = np.ascontiguousarray(atlas, np.uint8)
        self._check(self.L.tt_scene_upload_alpha_atlas(self.h, _ptr(a), a.shape[1], a.shape[0]),
                    "tt_scene_upload_alpha_atlas")

    def upload_texture_atlas(self, atlas: np.ndarray):
        """_TextureAtlas (AssetManager.cs:275) decoded to RGBA half: float16 [height, width, 4]."""
        a = np.ascontiguousarray(atlas, np.float16)
        assert a.ndim == 3 and a.shape[2] == 4
        self._check(self.L.tt_scene_upload_texture_atlas(self.h, _ptr(a), a.shape[1], a.shape[0]),
                    "tt_scene_upload_texture_atlas")

    def update_nodes(self, first: int, nodes: np.ndarray):
        self._check(self.L.tt_scene_update_nodes(self.h, first, len(nodes), _ptr(nodes)), "tt_scene_update_nodes")

    def update_meshdata(self, first: int, md: np.ndarray):
        self._check(self.L.tt_scene_update_meshdata(self.h, first, len(md), _ptr(md)), "tt_scene_update_meshdata")

    def sync(self):
        self._check(self.L.tt_sync(self.h), "tt_sync")

    def async_overflows(self) -> int:
        """tt_async_overflows: stack overflows of all launches since the last call (then reset)."""
        n = C.c_uint64()
        st = self.L.tt_async_overflows(self.h, C.byref(n))
        if st not in (TT_OK, TT_ERR_STACK_OVERFLOW):
            self._check(st, "tt_async_overflows")
        return int(n.value)

    def timing_reset(self):
        self._check(self.L.tt_timing_reset(self.h), "tt_timing_reset")

    def set_timing(self, enabled: bool):
        """tt_ctx_set_timing: off, asynchronous calls record no HIP events (and add no timing entry)."""
        self._check(self.L.tt_ctx_set_timing(self.h, 1 if enabled else 0), "tt_ctx_set_timing")

    def set_frame_pixels(self, frame_pixels: int):
        """tt_ctx_set_frame_pixels: batched frames (PixelIndex + j W H) draw frame j's bounce random numbers
        at frames + j from their frame-local pixel; 0 restores the reference's form."""
        self._check(self.L.tt_ctx_set_frame_pixels(self.h, int(frame_pixels)), "tt_ctx_set_frame_pixels")

    def timing_read(self) -> np.ndarray:
        ms = np.zeros(256, np.float32)
        n = C.c_uint32()
        self._check(self.L.tt_timing_read(self.h, ms.ctypes.data, 256, C.byref(n)), "tt_timing_read")
        return ms[: n.value].copy()

    def diagnostics(self) -> dict:
        d = np.zeros(8, np.uint64)
        self._check(self.L.tt_trace_diagnostics(self.h, d.ctypes.data), "tt_trace_diagnostics")
        keys = ["iterations", "node_iters", "node_lanes", "tri_iters", "tri_lanes", "active_lanes", "lead_same_lanes",
                "uniform_node_iters"]
        return {k: int(v) for k, v in zip(keys, d)}

    def selftest_rcp(self) -> int:
        """Inputs (of all 2^32 fp32 bit patterns) where the kernels' fast reciprocal differs from the
        correctly rounded 1.0f/x on this device (tt_selftest_rcp); must be 0."""
        n = C.c_uint64()
        self._check(self.L.tt_selftest_rcp(self.h, C.addressof(n)), "tt_selftest_rcp")
        return n.value

    def scene_bytes(self) -> int:
        b = C.c_uint64()
        self._check(self.L.tt_scene_bytes(self.h, C.byref(b)), "tt_scene_bytes")
        return b.value

    def trace(self, rays, n_rays: int, bounce: int, far_plane: float, width: int, height: int, info=None,
              colors=None, flags: int = 0, device: bool = False, stats: bool = False, check: bool = True,
              asynchronous: bool = False, hits_out=None):
        p = TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width, screen_height=height,
                        flags=flags | (TT_TRACE_DEVICE_PTRS if device else 0) | (TT_TRACE_STATS if stats else 0)
                        | (TT_TRACE_ASYNC if asynchronous else 0))
        s = Stats()
        if hits_out is not None:  # tt_trace_closest_hits: also the compact hit-record stream (no stats)
            st = self.L.tt_trace_closest_hits(self.h, C.byref(p), _ptr(rays), _ptr(info), _ptr(colors), _ptr(hits_out))
        else:
            st = self.L.tt_trace_closest(self.h, C.byref(p), _ptr(rays), _ptr(info), _ptr(colors), C.byref(s))
        if check:
            self._check(st, "tt_trace_closest")
        return (s, st) if not check else s

    def trace_indirect(self, rays, n_rays_dev, capacity: int, bounce: int, far_plane: float, width: int, height: int,
                       info=None, colors=None, flags: int = 0, check: bool = True):
        """tt_trace_closest_indirect: traces min(*n_rays_dev, capacity) rays, the count read on the device
        (a uint32 device tensor, e.g. the n_next_dev of enqueue_bounce_indirect); device pointers, async."""
        p = TraceParams(n_rays=capacity, bounce=bounce, far_plane=far_plane, screen_width=width, screen_height=height,
                        flags=flags | TT_TRACE_DEVICE_PTRS)
        st = self.L.tt_trace_closest_indirect(self.h, C.byref(p), _ptr(n_rays_dev), _ptr(rays), _ptr(info),
                                              _ptr(colors))
        if check:
            self._check(st, "tt_trace_closest_indirect")
        return st

    def tlas_refit(self, n_tlas_nodes: int, mesh_aabbs, device: bool = False, asynchronous: bool = False):
        """tt_tlas_refit (AssetManager.RefitTLAS): re-quantize TLAS nodes [0, n_tlas_nodes) in HBM from
        per-mesh world AABBs (n_mesh x {BBMax, BBMin})."""
        n = int(mesh_aabbs.shape[0]) if hasattr(mesh_aabbs, "shape") else len(mesh_aabbs) // 6
        flags = (TT_TRACE_DEVICE_PTRS if device else 0) | (TT_TRACE_ASYNC if asynchronous else 0)
        self._check(self.L.tt_tlas_refit(self.h, n_tlas_nodes, _ptr(mesh_aabbs), n, flags), "tt_tlas_refit")

    def blas_refit(self, mesh_index: int, vertices, indices, leaf_of_triangle, transform=None,
                   device: bool = False, asynchronous: bool = False):
        """tt_blas_refit (ParentObject.RefitMesh): re-derive the mesh's triangles from `vertices`
        (n x stride floats: position at +0, normal at +3) and refit its BLAS nodes in HBM.
        `transform` is a row-major 4x4 (identity by default)."""
        stride = int(vertices.shape[1]) if hasattr(vertices, "shape") and len(vertices.shape) == 2 else 6
        nv = int(vertices.shape[0]) if hasattr(vertices, "shape") and len(vertices.shape) == 2 else len(vertices) // 6
        n_tris = int(indices.shape[0]) // 3 if len(indices.shape) == 1 else int(indices.shape[0])
        p = BlasRefitParams(mesh_index=mesh_index, n_tris=n_tris, n_vertices=nv, vertex_stride=stride,
                            flags=(TT_TRACE_DEVICE_PTRS if device else 0) | (TT_TRACE_ASYNC if asynchronous else 0))
        p.transform[:] = unity_colmajor(np.eye(4) if transform is None else np.asarray(transform))
        self._check(self.L.tt_blas_refit(self.h, C.byref(p), _ptr(vertices), _ptr(indices), _ptr(leaf_of_triangle)),
                    "tt_blas_refit")

    def scene_tris(self, first: int, count: int) -> np.ndarray:
        """Reads AggTris [first, first+count) back from HBM (parity checks of the BLAS refit)."""
        out = np.zeros(count, TRI_DTYPE)
        self._check(self.L.tt_scene_read_tris(self.h, first, count, _ptr(out)), "tt_scene_read_tris")
        return out

    def scene_nodes(self, first: int, count: int) -> np.ndarray:
        """Reads nodes [first, first+count) back from HBM (parity checks of the refit)."""
        out = np.zeros(count, NODE_DTYPE)
        self._check(self.L.tt_scene_read_nodes(self.h, first, count, _ptr(out)), "tt_scene_read_nodes")
        return out

    def trace_shadow(self, shadow_rays, n_rays: int, bounce: int, width: int, height: int, visibility=None,
                     colors=None, nee_pos=None, device: bool = False, stats: bool = False, check: bool = True,
                     asynchronous: bool = False, flags: int = 0, cache=None, legacy: bool = False):
        """tt_trace_shadow_ex (kernel_shadow replacement): any-hit visibility of ShadowRayData rays and
        the GlobalColors / CacheBuffer accumulations (flags: TT_SHADOW_*, TT_TRACE_USE_RESTIRGI).
        legacy=True calls tt_trace_shadow instead (Direct at bounce 0 + NEEPosA only, no cache)."""
        p = ShadowParams(n_rays=n_rays, bounce=bounce, screen_width=width, screen_height=height,
                         flags=flags | (TT_TRACE_DEVICE_PTRS if device else 0) | (TT_TRACE_STATS if stats else 0)
                         | (TT_TRACE_ASYNC if asynchronous else 0))
        s = Stats()
        if legacy:
            assert cache is None, "tt_trace_shadow takes no CacheBuffer"
            st = self.L.tt_trace_shadow(self.h, C.byref(p), _ptr(shadow_rays), _ptr(visibility), _ptr(colors),
                                        _ptr(nee_pos), C.byref(s))
        else:
            st = self.L.tt_trace_shadow_ex(self.h, C.byref(p), _ptr(shadow_rays), _ptr(visibility), _ptr(colors),
                                           _ptr(nee_pos), _ptr(cache), C.byref(s))
        if check:
            self._check(st, "tt_trace_shadow" if legacy else "tt_trace_shadow_ex")
        return (s, st) if not check else s

    def trace_shadow_indirect(self, shadow_rays, n_rays_dev, capacity: int, bounce: int, width: int, height: int,
                              visibility=None, colors=None, nee_pos=None, flags: int = 0, cache=None, check: bool = True):
        """tt_trace_shadow_ex_indirect: min(*n_rays_dev, capacity) shadow rays; device pointers, async."""
        p = ShadowParams(n_rays=capacity, bounce=bounce, screen_width=width, screen_height=height,
                         flags=flags | TT_TRACE_DEVICE_PTRS)
        st = self.L.tt_trace_shadow_ex_indirect(self.h, C.byref(p), _ptr(n_rays_dev), _ptr(shadow_rays),
                                                _ptr(visibility), _ptr(colors), _ptr(nee_pos), _ptr(cache))
        if check:
            self._check(st, "tt_trace_shadow_ex_indirect")
        return st

    def resolve_normals(self, rays, n_rays: int, bounce: int, far_plane: float, width: int, height: int,
                        out=None, device: bool = False):
        p = TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width, screen_height=height,
                        flags=TT_TRACE_DEVICE_PTRS if device else 0)
        if out is None:
            out = np.zeros((n_rays, 6), np.float32)
        self._check(self.L.tt_resolve_normals(self.h, C.byref(p), _ptr(rays), _ptr(out)), "tt_resolve_normals")
        return out

    def generate(self, rays, cam_to_world, cam_inv_proj, width, height, near, far, jitter=0, frames=0,
                 max_bounce=3, device=False, asynchronous=False):
        cam = Camera()
        cam.cam_to_world[:] = unity_colmajor(cam_to_world)
        cam.cam_inv_proj[:] = unity_colmajor(cam_inv_proj)
        cam.near_plane, cam.far_plane, cam.width, cam.height = near, far, width, height
        cam.jitter, cam.frames_accumulated, cam.max_bounce = jitter, frames, max_bounce
        cam.flags = (TT_TRACE_DEVICE_PTRS if device else 0) | (TT_TRACE_ASYNC if (device and asynchronous) else 0)
        self._check(self.L.tt_generate_primary(self.h, C.byref(cam), _ptr(rays)), "tt_generate_primary")

    def enqueue_bounce(self, rays, n_rays, bounce, far_plane, width, height, frames=0, max_bounce=3,
                       device=False) -> int:
        p = TraceParams(n_rays=n_rays, bounce=bounce, far_plane=far_plane, screen_width=width, screen_height=height,
                        flags=TT_TRACE_DEVICE_PTRS if device else 0)
        n = C.c_uint32()
        self._check(self.L.tt_enqueue_diffuse_bounce(self.h, C.byref(p), _ptr(rays), frames, max_bounce,
                                                     C.byref(n)), "tt_enqueue_diffuse_bounce")
        return n.value

    def enqueue_bounce_indirect(self, rays, n_rays_dev, capacity, n_next_dev, bounce, far_plane, width, height,
                                frames=0, max_bounce=3, check: bool = True):
        """tt_enqueue_diffuse_bounce_indirect: the traced count from n_rays_dev (None: capacity), the survivor
        count written to the device uint32 n_next_dev; no synchronization."""
        p = TraceParams(n_rays=capacity, bounce=bounce, far_plane=far_plane, screen_width=width, screen_height=height,
                        flags=TT_TRACE_DEVICE_PTRS)
        st = self.L.tt_enqueue_diffuse_bounce_indirect(self.h, C.byref(p), _ptr(n_rays_dev), _ptr(rays), frames,
                                                       max_bounce, _ptr(n_next_dev))
        if check:
            self._check(st, "tt_enqueue_diffuse_bounce_indirect")
        return st


class DedicatedStream:
    """A HIP stream on a hardware queue of its own (tt_stream_create) wrapped as a torch ExternalStream.

    Concurrent trace launches (the parts / frame slots of ttlayout.FrameLayout, the gather stream) need
    streams that do not share a HW queue: a process's plain streams are dealt round-robin over a few
    queues, and two persistent grids on one queue run back to back instead of overlapping each other's
    drain (profiles/r04/streams/). ``close()`` synchronises and destroys it."""

    def __init__(self, torch, dev):
        L = hip_lib()
        h = C.c_void_p()
        _check(L.tt_stream_create(int(dev.index or 0), C.byref(h)), "tt_stream_create")
        self.handle = h.value
        self.stream = torch.cuda.ExternalStream(self.handle, device=dev)

    def close(self):
        if self.handle:
            _check(hip_lib().tt_stream_destroy(C.c_void_p(self.handle)), "tt_stream_destroy")
            self.handle = None
            self.stream = None


_DEDICATED = {}
_ENGINES = weakref.WeakSet()  # live contexts: closed before the dedicated streams they may issue on


def release_dedicated_streams():
    """Synchronises and destroys every process-wide dedicated stream (registered with atexit on the first
    one): a queue made with a CU mask that is still alive when the HIP runtime tears down takes the process
    down with it under rocprofv3 (exit status 139 in __cxa_finalize, gpurun_out/r04o). Torch's current
    stream is reset to the default stream first, so nothing issues on a destroyed handle."""
    if not _DEDICATED:
        return
    try:
        import torch

        for dev_i in {k[0] for k in _DEDICATED}:
            torch.cuda.synchronize(dev_i)
            torch.cuda.set_stream(torch.cuda.default_stream(dev_i))
    except Exception:  # noqa: BLE001 -- teardown: the streams go regardless
        pass
    for e in list(_ENGINES):  # a context synchronises its stream when destroyed: destroy it first
        try:
            e.close()
        except Exception:  # noqa: BLE001
            pass
    for d in list(_DEDICATED.values()):
        try:
            d.close()
        except Exception:  # noqa: BLE001
            pass
    _DEDICATED.clear()


def dedicated_stream(torch, dev, i: int):
    """The i-th process-wide stream with a HW queue of its own (a DedicatedStream made on first use and
    kept for the process's lifetime), as a torch ExternalStream. Layouts take streams 0, 1, ... in turn,
    so a process holds as many dedicated queues as its widest layout needs however many layouts it
    builds (tools/strong_replay.py builds one per rank), and a stream outlives every tensor, event and
    collective that was ever ordered on it."""
    key = (int(dev.index or 0), int(i))
    d = _DEDICATED.get(key)
    if d is None:
        if not _DEDICATED:
            import atexit

            atexit.register(release_dedicated_streams)
        d = DedicatedStream(torch, dev)
        _DEDICATED[key] = d
    return d.stream


def validate(s: Scene):
    """tt_scene_validate: (status, message) of the structural check tt_scene_upload runs."""
    buf = C.create_string_buffer(512)
    st = hip_lib().tt_scene_validate(_ptr(s.nodes), len(s.nodes), _ptr(s.tris), len(s.tris), _ptr(s.tlas),
                                     len(s.tlas), _ptr(s.meshdata), len(s.meshdata), _ptr(s.materials),
                                     len(s.materials), buf, 512)
    return st, buf.value.decode()


def device_count() -> int:
    try:
        return hip_lib().tt_device_count()
    except (FileNotFoundError, OSError):
        return 0


# ---------------------------------------------------------------- multi-GPU group (tt_group_*)
TT_GROUP_COPY_GATHER = 1 << 0
TT_GROUP_BOUNCE = 1 << 1
TT_GROUP_INFO = 1 << 2
GROUP_SYMBOLS = ["tt_group_create", "tt_group_unique_id", "tt_group_create_rank", "tt_group_destroy",
                 "tt_group_last_error", "tt_group_local_members", "tt_group_member_ctx", "tt_group_scene_upload",
                 "tt_group_trace_frame", "tt_group_sync", "tt_group_frame_rays", "tt_group_tile_pixels", "tt_shutdown"]


class GroupConfig(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("tile", C.c_uint32), ("slots", C.c_uint32),
                ("flags", C.c_uint32), ("batch", C.c_uint32)]


def _group_lib():
    L = hip_lib()
    if not getattr(L, "_group_bound", False):
        _bind_group(L)
    return L


def _bind_group(L):
    if True:
        vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
        L.tt_group_create.argtypes = [vp, u32, C.POINTER(GroupConfig), C.POINTER(vp)]
        L.tt_group_unique_id.argtypes = [vp]
        L.tt_group_create_rank.argtypes = [vp, u32, u32, i32, C.POINTER(GroupConfig), C.POINTER(vp)]
        L.tt_group_destroy.argtypes = [vp]
        L.tt_group_last_error.argtypes = [vp]
        L.tt_group_last_error.restype = C.c_char_p
        L.tt_group_local_members.argtypes = [vp]
        L.tt_group_local_members.restype = u32
        L.tt_group_member_ctx.argtypes = [vp, u32]
        L.tt_group_member_ctx.restype = vp
        L.tt_group_scene_upload.argtypes = [vp, vp, u32, vp, u32, vp, u32, vp, u32, vp, u32]
        L.tt_group_trace_frame.argtypes = [vp, C.POINTER(Camera), vp, vp, u32]
        L.tt_group_scene_upload_alpha_atlas.argtypes = [vp, vp, u32, u32]
        L.tt_group_scene_update_meshdata.argtypes = [vp, u32, u32, vp]
        L.tt_group_scene_update_nodes.argtypes = [vp, u32, u32, vp]
        L.tt_group_tlas_refit.argtypes = [vp, u32, vp, u32, u32]
        L.tt_group_scene_upload_texture_atlas.argtypes = [vp, vp, u32, u32]
        L.tt_group_sync.argtypes = [vp]
        L.tt_group_frame_rays.argtypes = [vp, u32, C.POINTER(u32), C.POINTER(u32), C.POINTER(vp)]
        L.tt_group_tile_pixels.argtypes = [u32, u32, u32, u32, u32, vp, u32, C.POINTER(u32)]
        for s in ["tt_group_create", "tt_group_unique_id", "tt_group_create_rank", "tt_group_destroy",
                  "tt_group_scene_upload", "tt_group_trace_frame", "tt_group_sync", "tt_group_frame_rays",
                  "tt_group_tile_pixels", "tt_shutdown", "tt_group_scene_upload_alpha_atlas",
                  "tt_group_scene_upload_texture_atlas", "tt_group_scene_update_meshdata",
                  "tt_group_scene_update_nodes", "tt_group_tlas_refit"]:
            getattr(L, s).restype = i32
        L._group_bound = True


def group_tile_pixels(width: int, height: int, world: int, rank: int, tile: int = 64) -> np.ndarray:
    """tt_group_tile_pixels: the library's own shard of `rank` (host arithmetic, no GPU)."""
    L = _group_lib()
    n = C.c_uint32()
    _check(L.tt_group_tile_pixels(width, height, tile, world, rank, None, 0, C.byref(n)), "tt_group_tile_pixels")
    out = np.zeros(max(1, n.value), np.uint32)
    _check(L.tt_group_tile_pixels(width, height, tile, world, rank, out.ctypes.data, n.value, C.byref(n)),
           "tt_group_tile_pixels")
    return out[: n.value]


def group_unique_id() -> bytes:
    """tt_group_unique_id: the 128-byte RCCL id rank 0 makes for tt_group_create_rank."""
    buf = (C.c_uint8 * 128)()
    _check(_group_lib().tt_group_unique_id(C.addressof(buf)), "tt_group_unique_id")
    return bytes(buf)


def shutdown():
    """tt_shutdown: destroys every library stream still alive (hosts tracing from a non-main thread)."""
    _check(hip_lib().tt_shutdown(), "tt_shutdown")


class Group:
    """A multi-GPU tile-sharded frame (tt_group_*): ``devices`` in one process (tt_group_create), or this
    process as ``rank`` of ``world`` on ``device`` with the RCCL id ``uid`` (tt_group_create_rank)."""

    def __init__(self, width: int, height: int, devices=None, tile: int = 64, slots: int = 2, bounce: bool = False,
                 copy: bool = False, rank: int = None, world: int = None, uid: bytes = None, device: int = None,
                 info: bool = False, batch: int = 1):
        L = _group_lib()
        cfg = GroupConfig(width=width, height=height, tile=tile, slots=slots, batch=batch,
                          flags=(TT_GROUP_BOUNCE if bounce else 0) | (TT_GROUP_COPY_GATHER if copy else 0)
                          | (TT_GROUP_INFO if info else 0))
        h = C.c_void_p()
        if devices is not None:
            devs = np.ascontiguousarray(devices, np.int32)
            st = L.tt_group_create(devs.ctypes.data, len(devs), C.byref(cfg), C.byref(h))
            self.world = len(devs)
        else:
            idb = (C.c_uint8 * 128).from_buffer_copy(uid)
            st = L.tt_group_create_rank(C.addressof(idb), world, rank, device, C.byref(cfg), C.byref(h))
            self.world = world
        if st != TT_OK:
            raise TTError(st, "tt_group_create")
        self.L, self.h = L, h.value
        self.width, self.height, self.bounce, self.batch = width, height, bounce, max(1, batch)

    def _check(self, st, what):
        if st != TT_OK:
            raise TTError(st, f"{what}: {self.L.tt_group_last_error(self.h).decode()}")

    def local_members(self) -> int:
        return int(self.L.tt_group_local_members(self.h))

    def member_ctx(self, m: int) -> int:
        return self.L.tt_group_member_ctx(self.h, m)

    def upload(self, s: Scene):
        st = self.L.tt_group_scene_upload(self.h, _ptr(s.nodes), len(s.nodes), _ptr(s.tris), len(s.tris),
                                          _ptr(s.tlas), len(s.tlas), _ptr(s.meshdata), len(s.meshdata),
                                          _ptr(s.materials), len(s.materials))
        self._check(st, "tt_group_scene_upload")
        if s.alpha_atlas is not None:
            a = np.ascontiguousarray(s.alpha_atlas, np.uint8)
            self._check(self.L.tt_group_scene_upload_alpha_atlas(self.h, a.ctypes.data, a.shape[1], a.shape[0]),
                        "tt_group_scene_upload_alpha_atlas")
        if s.texture_atlas is not None:
            t = np.ascontiguousarray(s.texture_atlas, np.float16)
            self._check(self.L.tt_group_scene_upload_texture_atlas(self.h, t.ctypes.data, t.shape[1], t.shape[0]),
                        "tt_group_scene_upload_texture_atlas")

    def trace_frame(self, hits_out, cam_to_world, cam_inv_proj, near, far, jitter=1, frames=0, max_bounce=1,
                    asynchronous=False, info_out=None):
        cam = Camera()
        cam.cam_to_world[:] = unity_colmajor(cam_to_world)
        cam.cam_inv_proj[:] = unity_colmajor(cam_inv_proj)
        cam.near_plane, cam.far_plane, cam.width, cam.height = near, far, self.width, self.height
        cam.jitter, cam.frames_accumulated, cam.max_bounce = jitter, frames, max_bounce
        cam.flags = TT_TRACE_DEVICE_PTRS
        self._check(self.L.tt_group_trace_frame(self.h, C.byref(cam), _ptr(hits_out), _ptr(info_out),
                                                TT_TRACE_ASYNC if asynchronous else 0), "tt_group_trace_frame")

    def sync(self):
        self._check(self.L.tt_group_sync(self.h), "tt_group_sync")

    def update_meshdata(self, first: int, md: np.ndarray):
        self._check(self.L.tt_group_scene_update_meshdata(self.h, first, len(md), _ptr(md)),
                    "tt_group_scene_update_meshdata")

    def update_nodes(self, first: int, nodes: np.ndarray):
        self._check(self.L.tt_group_scene_update_nodes(self.h, first, len(nodes), _ptr(nodes)),
                    "tt_group_scene_update_nodes")

    def tlas_refit(self, n_tlas_nodes: int, mesh_aabbs: np.ndarray, asynchronous: bool = False):
        a = np.ascontiguousarray(mesh_aabbs, np.float32)
        self._check(self.L.tt_group_tlas_refit(self.h, n_tlas_nodes, a.ctypes.data, a.shape[0],
                                               TT_TRACE_ASYNC if asynchronous else 0), "tt_group_tlas_refit")

    def frame_rays(self, m: int = 0):
        """(n_primary, n_bounce, device pointer of the ray buffer) of member m's latest frame."""
        a, b, p = C.c_uint32(), C.c_uint32(), C.c_void_p()
        self._check(self.L.tt_group_frame_rays(self.h, m, C.byref(a), C.byref(b), C.byref(p)), "tt_group_frame_rays")
        return a.value, b.value, p.value

    def close(self):
        if getattr(self, "h", None):
            self.L.tt_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
