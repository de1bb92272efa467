"""ttconfigs — the BASELINE.json configurations as scene + camera builders (SURVEY.md §8(d),
"Synthetic inputs"), shared by bench.py and the tests.

The reference's Sponza / Bistro / San Miguel assets are not in its tree
(``.MISSING_LARGE_BLOBS:14-15``), so each config is a seeded synthetic scene of the stated shape,
built through the host AssetManager restatement (``tthip.AssetManager``) into the exact buffers
``AssetManager.SetMeshTraceBuffers`` binds (``AssetManager.cs:75-88``):

  C1  Cornell, 12 tris, 256x256 primary (CPU-runnable case)
  C2  Sponza-shaped hall, 262,267 tris in one BLAS under a 1-node TLAS, 1920x1080
  C3  C2 geometry, primary + 3 diffuse bounces (compacted survivors per bounce)
  C4  Bistro-shaped street grid: 600 unique BLAS (200-40k tris, log-uniform) referenced by 2,400
      rigid + uniform-scale instances over 200x200 m, plus the street plane, 1920x1080
  C5  San-Miguel-shaped courtyard, 10M tris (~60% foliage-like small tris), 3840x2160,
      64x64 tiles round-robin over 8 GPUs (``ttdist.tile_pixels``)

Generators are deterministic: C++ ``std::mt19937_64`` inside the scene library, and numpy's PCG64
(``default_rng``) for the C4 instance layout.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

import tthip

FAR = 1000.0
NEAR = 0.3


@dataclass(frozen=True)
class View:
    position: Tuple[float, float, float]
    forward: Tuple[float, float, float]
    vfov: float
    width: int
    height: int
    up: Tuple[float, float, float] = (0.0, 1.0, 0.0)

    def camera(self, width: int = 0, height: int = 0):
        """(cam_to_world, cam_inverse_projection) as Unity builds them (``unity_camera``)."""
        return tthip.unity_camera(self.position, self.forward, self.up, self.vfov, width or self.width,
                                  height or self.height, NEAR, FAR)


C1_VIEW = View((0.0, 0.0, 3.4), (0.0, 0.0, -1.0), 40.0, 256, 256)
C2_VIEW = View((-10.0, 2.0, 0.0), (1.0, 0.0, 0.0), 60.0, 1920, 1080)
C4_VIEW = View((-20.0, 1.8, -95.0), (0.0, -0.03, 1.0), 60.0, 1920, 1080)
C5_VIEW = View((-12.0, 1.7, -13.0), (1.0, 0.06, 1.3), 60.0, 3840, 2160)

C2_SEED, C4_SEED, C5_SEED = 0x53504F4E, 0xB1575A0, 0x5A4E4D
C2_TRIS, C5_TRIS = 262267, 10_000_000


def c1_cornell() -> tthip.Scene:
    return tthip.single_object_scene(tthip.Mesh.cornell(), n_materials=4)


def c2_sponza(seed: int = C2_SEED, n_tris: int = C2_TRIS) -> tthip.Scene:
    """One ParentObject (an imported OBJ) -> one BLAS under a 1-node TLAS. Materials 0..6."""
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.sponza(seed, n_tris)), None, np.zeros(7, tthip.MAT_DTYPE))
    return am.build()


def _mix_seed(seed: int, k: int) -> int:
    return (seed * 0x9E3779B97F4A7C15 + (k + 1) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF


def c4_bistro(seed: int = C4_SEED, n_unique: int = 600, n_instances: int = 2400, min_tris: int = 200,
              max_tris: int = 40000) -> tthip.Scene:
    """Two-level scene (AssetManager.cs:1714-1750): the street plane as a RenderQue parent, then
    ``n_unique`` InstanceData parents (facades/props from ``tt_synth_prop``, tri counts
    log-uniform in [min_tris, max_tris]) and ``n_instances`` InstancedObjects dealt round-robin
    over them, placed 12-20 m off the centre lines of a 40 m street grid over [-100, 100]^2
    (keeping 14 m clear of the crossings), facing the street, with a random yaw jitter and
    uniform scale 0.6-1.6 (rigid + uniform scale W2L)."""
    rng = np.random.default_rng(seed)
    sizes = np.exp(rng.uniform(np.log(min_tris), np.log(max_tris), n_unique)).astype(np.int64)
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.ground(-110.0, 110.0, -110.0, 110.0, 128, 128)), None,
                  np.zeros(1, tthip.MAT_DTYPE))
    mats = np.zeros(3, tthip.MAT_DTYPE)
    parents = [am.add_instance_parent(tthip.Blas(tthip.Mesh.prop(_mix_seed(seed, k), int(sizes[k]))), mats)
               for k in range(n_unique)]
    lines = np.arange(-100.0, 100.0 + 1e-3, 40.0)
    for i in range(n_instances):
        along_x = bool(rng.integers(0, 2))
        line = float(lines[rng.integers(0, len(lines))])
        while True:
            t = float(rng.uniform(-100.0, 100.0))
            if np.abs(lines - t).min() >= 14.0:
                break
        side = 1.0 if rng.integers(0, 2) else -1.0
        off = float(rng.uniform(12.0, 20.0))
        scale = float(rng.uniform(0.6, 1.6))
        yaw = float((0.0 if along_x else 90.0) + (0.0 if side > 0 else 180.0) + rng.uniform(-6.0, 6.0))
        pos = (t, 0.0, line + side * off) if along_x else (line + side * off, 0.0, t)
        am.add_instance(parents[i % n_unique], tthip.trs_matrix(pos, yaw, scale))
    sc = am.build()
    sc.meta.update({"unique_blas": n_unique, "instances": n_instances,
                    "unique_tris": int(len(sc.tris)), "instanced_tris": int(sizes[np.arange(n_instances) % n_unique].sum())})
    return sc


def c5_san_miguel(seed: int = C5_SEED, n_tris: int = C5_TRIS) -> tthip.Scene:
    """One ParentObject with ``n_tris`` triangles (the San Miguel OBJ imports as one mesh)."""
    am = tthip.AssetManager()
    am.add_parent(tthip.Blas(tthip.Mesh.san_miguel(seed, n_tris)), None, np.zeros(8, tthip.MAT_DTYPE))
    return am.build()
