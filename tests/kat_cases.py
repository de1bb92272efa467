"""Known-answer cases for the closest-hit traversal (test infrastructure).

Every case is a hand-built scene (tests/handbuilt.py) whose expected hit record follows from
the reference's semantics with exact dyadic arithmetic, so it holds under any legal rounding of
the reference HLSL (IntersectionKernels.compute:14-260, CommonData.cginc:635-707). The same
cases run against the oracle (tests/test_oracle_kat.py) and the GPU (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import numpy as np

import handbuilt as hb
import tthip

E6 = 121  # scale 2^-6


def _leaf_root(tris_count=1, z_lo=63, z_hi=65):
    # BLAS root: p = (-1,-1,-1), scale 1/64: box x,y in [0, 1], z in [-1/64, 1/64]
    return hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                        [(0, "leaf", (64, 64, z_lo), (128, 128, z_hi), (0, tris_count))])


UNIT_TRI = hb.tri((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0))


def case_single_triangle():
    sc = hb.scene([_leaf_root()], [UNIT_TRI])
    rays = hb.rays_buffer([(0.25, 0.25, 1.0), (0.0, 0.0, 1.0), (2.0, 2.0, 1.0), (0.25, 0.25, -1.0)],
                          [(0.0, 0.0, -1.0), (0.5, 0.25, -1.0), (0.0, 0.0, -1.0), (0.0, 0.0, -1.0)])
    far = np.uint32(np.float32(1000.0).view(np.uint32))
    expected = [hb.expected_hit(0, 0, 1.0, 0.25, 0.25),   # axis-parallel: NaN slabs ignored (maxNum)
                hb.expected_hit(0, 0, 1.0, 0.5, 0.25),    # oblique, exact
                [0, 0xFFFFFFFF, int(far), 0],             # outside the node box: miss
                [0, 0xFFFFFFFF, int(far), 0]]             # behind the origin: t < 0 rejected
    return "single_triangle", sc, rays, 4, expected


def case_tie_first_found_wins():
    # two coincident triangles in one leaf: bit 1 is visited first (IntersectionKernels.compute:222)
    # and the strict t < best.t (:33) keeps it.
    sc = hb.scene([_leaf_root(2)], [UNIT_TRI, UNIT_TRI])
    rays = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    return "tie_first_found_wins", sc, rays, 1, [hb.expected_hit(0, 1, 1.0, 0.25, 0.25)]


def _two_child_scene():
    # root with two internal children: k=0 far (z = -0.5), k=1 near (z = 0)
    root = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 1, 0,
                        [(0, "inner", (64, 64, 31), (128, 128, 33), 0),
                         (1, "inner", (64, 64, 63), (128, 128, 65), 1)])
    far_child = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                             [(0, "leaf", (64, 64, 31), (128, 128, 33), (0, 1))])
    near_child = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 1,
                              [(0, "leaf", (64, 64, 63), (128, 128, 65), (0, 1))])
    tris = [hb.tri((0.0, 0.0, -0.5), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0)), UNIT_TRI]
    return hb.scene([root, far_child, near_child], tris)


def case_octant_order_and_culling():
    # dir.z < 0, x,y >= 0: oct byte 6, child k=1 sits at bit 24 + (1^6) = 31 and is visited first;
    # the near hit (t = 1) then culls the far child's leaf (tri tests = 1).
    sc = _two_child_scene()
    rays = hb.rays_buffer([(0.25, 0.25, 1.0), (0.25, 0.25, -2.0)], [(0.0, 0.0, -1.0), (0.0, 0.0, 1.0)])
    # second ray travels +z from below: hits far tri (z=-0.5) at t=1.5 first in distance
    expected = [hb.expected_hit(0, 1, 1.0, 0.25, 0.25), hb.expected_hit(0, 0, 1.5, 0.25, 0.25)]
    return "octant_order_and_culling", sc, rays, 2, expected


def case_reps_exhausted():
    # a chain of 1001 internal nodes: the ray reaches Reps == 1000 and writes nothing (:155)
    n = 1001
    nodes = []
    for i in range(n):
        if i < n - 1:
            nodes.append(hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), i + 1, 0,
                                      [(0, "inner", (0, 0, 0), (255, 255, 255), 0)]))
        else:
            nodes.append(_leaf_root())
    sc = hb.scene(nodes, [UNIT_TRI])
    rays = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    rays["hits"][0] = [7, 8, 9, 10]  # sentinel: must survive
    return "reps_exhausted", sc, rays, 1, [[7, 8, 9, 10]]


def case_chain_within_bound():
    # 998 internal nodes + the leaf node: 999 node visits below the TLAS node => 1000 total, the
    # ray finishes in the same iteration it reaches Reps == 1000 and writes its hit.
    n = 999
    nodes = []
    for i in range(n):
        if i < n - 1:
            nodes.append(hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), i + 1, 0,
                                      [(0, "inner", (0, 0, 0), (255, 255, 255), 0)]))
        else:
            nodes.append(_leaf_root())
    sc = hb.scene(nodes, [UNIT_TRI])
    rays = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    return "chain_within_bound", sc, rays, 1, [hb.expected_hit(0, 0, 1.0, 0.25, 0.25)]


def stack_overflow_scene(depth=18):
    """Every level has two internal children that the ray hits; descending one pushes the
    other, so the stack grows by one per level and overflows past 16 (:65, :166-168)."""
    nodes = []
    for i in range(depth):
        # children: k=0 -> next level (index 2*i+1), k=1 -> an empty dead-end node (2*i+2)
        nodes.append(hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 2 * i + 1, 0,
                                  [(0, "inner", (0, 0, 0), (255, 255, 255), 0),
                                   (1, "inner", (0, 0, 0), (255, 255, 255), 1)]))
        nodes.append(hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0, []))
    nodes.append(_leaf_root())
    sc = hb.scene(nodes, [UNIT_TRI])
    rays = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    return sc, rays


def case_two_instances():
    """Two instances of one BLAS (AssetManager.cs:1714-1750): translations (+4,0,0) and (0,0,0).
    TLAS node 0 holds both in one leaf; slot bit 1 (tlas[1]) is entered first."""
    blas = [_leaf_root()]
    nodes = np.zeros(4 + 1, tthip.NODE_DTYPE)  # TLAS region 2*2 = 4 slots, BLAS at 4
    nodes[0] = hb.make_node((-8.0, -8.0, -8.0), (E6 + 3, E6 + 3, E6 + 3), 0, 0,
                            [(0, "leaf", (64, 64, 56), (128, 128, 72), (0, 2))])
    nodes[4] = blas[0]
    t_a = np.eye(4)
    t_a[0, 3] = 4.0
    md = np.zeros(2, tthip.MESH_DTYPE)
    md[0] = hb.mesh_record(4, 0, 4, tthip.unity_colmajor(np.linalg.inv(t_a)))
    md[1] = hb.mesh_record(4, 0, 4, tthip.unity_colmajor(np.eye(4)))
    sc = tthip.Scene(nodes, np.array([UNIT_TRI], tthip.TRI_DTYPE), np.array([0, 1], np.int32), md,
                     np.zeros(1, tthip.MAT_DTYPE), tlas_nodes=1)
    rays = hb.rays_buffer([(4.25, 0.25, 1.0), (0.25, 0.25, 1.0), (2.25, 0.25, 1.0)],
                          [(0.0, 0.0, -1.0), (0.0, 0.0, -1.0), (0.0, 0.0, -1.0)])
    far = int(np.float32(1000.0).view(np.uint32))
    expected = [hb.expected_hit(0, 0, 1.0, 0.25, 0.25), hb.expected_hit(1, 0, 1.0, 0.25, 0.25), [0, 0xFFFFFFFF, far, 0]]
    return "two_instances", sc, rays, 3, expected


def case_invisible_bounce0():
    """Material Invisible flag (bit 7 of Tag) hides a triangle at CurBounce == 0 only (:48)."""
    tris = [hb.tri((0.0, 0.0, -0.5), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=0),
            hb.tri((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=1)]
    root = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                        [(0, "leaf", (64, 64, 31), (128, 128, 65), (0, 2))])
    mats = np.zeros(2, tthip.MAT_DTYPE)
    mats[1]["Tag"] = 1 << tthip.FLAG_INVISIBLE
    sc = hb.scene([root], tris, materials=mats)
    rays = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    return sc, rays, hb.expected_hit(0, 0, 1.5, 0.25, 0.25), hb.expected_hit(0, 1, 1.0, 0.25, 0.25)


ALL_CASES = [case_single_triangle, case_tie_first_found_wins, case_octant_order_and_culling, case_reps_exhausted,
             case_chain_within_bound, case_two_instances]


# ------------------------------------------------------------------- any-hit (kernel_shadow)
def shadow_case_single_triangle():
    """Unit triangle at z = 0, rays straight down from z = 1 (the hit is at t = 1 exactly).
    Returns (scene, shadow rays, expected status per ray: 0 reached |t|, 4 occluded)."""
    sc = hb.scene([_leaf_root()], [UNIT_TRI])
    o, d = (0.25, 0.25, 1.0), (0.0, 0.0, -1.0)
    rays = hb.shadow_rays([o, o, o, o, (2.0, 2.0, 1.0), o, (0.25, 0.25, -1.0)],
                          [d, d, d, d, d, d, d],
                          [2.0, 0.5, -2.0, -0.5, 2.0, 1.0, 2.0])
    # t = 2 occluded; 0.5 short of the surface; -2 occluded (|t|); -0.5 short; miss in x,y;
    # |t| = 1 exactly: strict t < max_distance keeps it visible; origin below, t = -1 behind
    return "shadow_single_triangle", sc, rays, [4, 0, 4, 0, 0, 0, 0]


def shadow_case_flags():
    """A ShadowCaster and an IsBackground surface never occlude (CommonData.cginc:612); a plain
    one behind them does."""
    tris = [hb.tri((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=1),
            hb.tri((0.0, 0.0, -0.25), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=2),
            hb.tri((0.0, 0.0, -0.5), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=0)]
    root = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                        [(0, "leaf", (64, 64, 31), (128, 128, 65), (0, 3))])
    mats = np.zeros(3, tthip.MAT_DTYPE)
    mats[1]["Tag"] = 1 << tthip.TT_FLAG_SHADOW_CASTER
    mats[2]["Tag"] = 1 << tthip.TT_FLAG_IS_BACKGROUND
    sc = hb.scene([root], tris, materials=mats)
    o, d = (0.25, 0.25, 1.0), (0.0, 0.0, -1.0)
    rays = hb.shadow_rays([o, o, o], [d, d, d], [1.4, 1.6, 1.2])
    # 1.4: only the flagged surfaces lie within |t| -> reaches the light; 1.6: the plain one at
    # t = 1.5 occludes; 1.2: flagged surfaces only
    return "shadow_flags", sc, rays, [0, 4, 0]


def shadow_case_two_instances():
    name, sc, _, _, _ = case_two_instances()
    d = (0.0, 0.0, -1.0)
    rays = hb.shadow_rays([(4.25, 0.25, 1.0), (0.25, 0.25, 1.0), (2.25, 0.25, 1.0), (0.25, 0.25, 1.0)],
                          [d, d, d, d], [3.0, 3.0, 3.0, 0.75])
    return "shadow_two_instances", sc, rays, [4, 4, 0, 0]


SHADOW_CASES = [shadow_case_single_triangle, shadow_case_flags, shadow_case_two_instances]


# ------------------------------------------------------------------ Cutout alpha test (§8 f3)
def _cutout_scene(scale=(1.0, 1.0, 0.0, 0.0), alpha_tex=(16384 | (16384 << 15), 0)):
    """Cutout unit triangle at z = 0 (material 1, UVs = barycentrics) over an opaque one at
    z = -0.5. Alpha atlas 4x4: columns 0-1 transparent (0), columns 2-3 opaque (255)."""
    tris = [hb.tri((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=1),
            hb.tri((0.0, 0.0, -0.5), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=0)]
    tris[0]["tex0"], tris[0]["texedge1"], tris[0]["texedge2"] = (0.0, 0.0), (1.0, 0.0), (0.0, 1.0)
    root = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                        [(0, "leaf", (64, 64, 31), (128, 128, 65), (0, 2))])
    mats = np.zeros(2, tthip.MAT_DTYPE)
    mats[1]["MatType"] = tthip.MAT_CUTOUT_INDEX
    mats[1]["AlphaCutoff"] = 0.5
    mats[1]["AlbedoTexScale"] = scale
    mats[1]["AlphaTex"] = alpha_tex
    sc = hb.scene([root], tris, materials=mats)
    atlas = np.zeros((4, 4), np.uint8)
    atlas[:, 2:] = 255
    sc.alpha_atlas = atlas
    return sc


def case_cutout():
    """IntersectionKernels.compute:35-40 with the pinned bilinear filter: at uv (0.25, 0.25) all four
    taps are transparent (alpha 0 < 0.5: the cutout triangle is skipped and the opaque one behind is
    hit); at uv (0.6, 0.2) the taps are columns 1 and 2 with weight 0.9 on the opaque one."""
    sc = _cutout_scene()
    rays = hb.rays_buffer([(0.25, 0.25, 1.0), (0.6, 0.2, 1.0)], [(0.0, 0.0, -1.0), (0.0, 0.0, -1.0)])
    return "cutout", sc, rays, 2, [hb.expected_hit(0, 1, 1.5, 0.25, 0.25), hb.expected_hit(0, 0, 1.0, 0.6, 0.2)]


def case_cutout_wrap_and_no_texture():
    """AlignUV (CommonData.cginc:569-591): TexScale offset -0.5 wraps u = 0.25 to 0.75 (opaque);
    AlphaTex.x <= 0 samples uv (-1, -1), i.e. the clamped corner texel (transparent)."""
    wrap = _cutout_scene(scale=(1.0, 1.0, -0.5, 0.0))
    none = _cutout_scene(alpha_tex=(0, 0))
    r = hb.rays_buffer([(0.25, 0.25, 1.0)], [(0.0, 0.0, -1.0)])
    return wrap, none, r, hb.expected_hit(0, 0, 1.0, 0.25, 0.25), hb.expected_hit(0, 1, 1.5, 0.25, 0.25)


def shadow_case_cutout():
    """Point-sampled cutout in the shadow test (CommonData.cginc:613-616): uv (0.25, 0.25) -> texel
    (1, 1) transparent, the opaque triangle at t = 1.5 decides; uv (0.6, 0.2) -> texel (2, 0) opaque."""
    sc = _cutout_scene()
    d = (0.0, 0.0, -1.0)
    rays = hb.shadow_rays([(0.25, 0.25, 1.0), (0.25, 0.25, 1.0), (0.6, 0.2, 1.0)], [d, d, d], [1.25, 2.0, 1.25])
    return "shadow_cutout", sc, rays, [0, 4, 4]


ALL_CASES.append(case_cutout)
SHADOW_CASES.append(shadow_case_cutout)


# ------------------------------------------ stained-glass shadow tint (§8 f1, CommonData.cginc:613-625)
GLASS_COLORS = {1: (0.5, 1.0, 0.25), 2: (1.0, 0.75, 1.0), 3: (0.8, 0.6, 0.4)}


def glass_texture_atlas():
    """4x4 RGBA half atlas with a distinct value per texel and channel."""
    y, x = np.mgrid[0:4, 0:4]
    a = np.zeros((4, 4, 4), np.float16)
    a[..., 0] = 0.1 * x + 0.01 * y
    a[..., 1] = 0.5 + 0.125 * x - 0.03 * y
    a[..., 2] = 1.7 - 0.2 * x + 0.07 * y
    a[..., 3] = 1.0
    return a


def glass_factor(mat, texel_xy, atlas):
    """surfaceColor * (texel.xyz + 2) / 3 in float32, per component."""
    c = np.asarray(GLASS_COLORS[mat], np.float32)
    t = atlas[texel_xy[1], texel_xy[0], :3].astype(np.float32)
    return (c * (t + np.float32(2.0))) / np.float32(3.0)


def shadow_case_glass():
    """Four unit triangles in two leaves of one node, visited z = -1, -0.5, -0.25, 0 (highest
    triangle bit first): an
    opaque one at z = -1 (t = 2), glass + Cutout at z = -0.5 (alpha atlas: columns 0-1
    transparent), plain glass without an albedo texture at z = -0.25 (AlignUV -> (-1, -1) -> texel
    (0, 0)), glass at z = 0 with the atlas rectangle = the whole atlas (uv = barycentrics).
    Glass never occludes and tints even beyond |t| (the material checks precede the t test);
    a Cutout-rejected glass surface does not tint. Returns (name, scene, rays, status, throughput)."""
    tris = [hb.tri((0.0, 0.0, z), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), matdat=m)
            for z, m in ((0.0, 1), (-0.25, 2), (-0.5, 3), (-1.0, 0))]
    for t in tris:
        t["tex0"], t["texedge1"], t["texedge2"] = (0.0, 0.0), (1.0, 0.0), (0.0, 1.0)
    root = hb.make_node((-1.0, -1.0, -1.0), (E6, E6, E6), 0, 0,
                        [(0, "leaf", (64, 64, 0), (128, 128, 65), (0, 3)),
                         (1, "leaf", (64, 64, 0), (128, 128, 65), (3, 1))])
    mats = np.zeros(4, tthip.MAT_DTYPE)
    whole = (16384 | (16384 << 15), 0)
    for m, col in GLASS_COLORS.items():
        mats[m]["specTrans"] = 1.0
        mats[m]["surfaceColor"] = col
        mats[m]["AlbedoTexScale"] = (1.0, 1.0, 0.0, 0.0)
        mats[m]["AlbedoTex"] = whole if m != 2 else (0, 0)
    mats[3]["MatType"] = tthip.MAT_CUTOUT_INDEX
    mats[3]["AlphaCutoff"] = 0.5
    mats[3]["AlphaTex"] = whole
    sc = hb.scene([root], tris, materials=mats)
    alpha = np.zeros((4, 4), np.uint8)
    alpha[:, 2:] = 255
    sc.alpha_atlas = alpha
    sc.texture_atlas = glass_texture_atlas()
    d = (0.0, 0.0, -1.0)
    a, c = (0.25, 0.25, 1.0), (0.6, 0.2, 1.0)
    rays = hb.shadow_rays([a, a, c, a, a], [d] * 5, [1.75, 2.5, 1.75, 0.5, 1.1])
    at = sc.texture_atlas
    f0a = glass_factor(1, (1, 1), at)   # z = 0 at uv (0.25, 0.25)
    f1 = glass_factor(2, (0, 0), at)    # no albedo texture: texel (0, 0)
    f0c = glass_factor(1, (2, 0), at)   # z = 0 at uv (0.6, 0.2)
    f2c = glass_factor(3, (2, 0), at)   # glass + cutout passes the alpha test at uv (0.6, 0.2)
    one = np.ones(3, np.float32)
    thr = [(one * f1) * f0a, None, ((one * f2c) * f1) * f0c, one, (one * f1) * f0a]
    # 1.75: reaches, tinted by z = -0.25 and z = 0 (z = -0.5 rejected by the alpha test);
    # 2.5: the opaque triangle at t = 2 occludes; uv (0.6, 0.2): all three glass surfaces tint;
    # 0.5: the leaf box starts beyond |t| (culled, no tint); 1.1: the glass at t = 1.25 lies beyond
    # |t| and still tints
    return "shadow_glass", sc, rays, [0, 4, 0, 0, 0], thr
