/*
 * tt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of TrueTrace's closest-hit CWBVH8 traversal
 * (kernel_trace / IntersectBVH, TrueTrace/Resources/MainCompute/IntersectionKernels.compute:14-260)
 * and of the few producers/consumers either side of it that the parity tests need
 * (camera ray generation, diffuse bounce enqueue, normal resolve).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline. The product path (libtruetrace_hip.so)
 * never links or calls it.
 *
 * Parity status: the reference (HLSL compiled by Unity's DXC for D3D12) cannot be compiled
 * or run in this environment and ships no golden vectors, so parity against reference
 * OUTPUTS is UNPINNED. The oracle is pinned by (1) analytic known-answer vectors whose
 * results are exact under any legal rounding of the reference HLSL (tests/test_oracle_kat.py)
 * and (2) the numerics contract in include/truetrace_hip.h, which the GPU kernel also follows.
 */
#ifndef TT_ORACLE_H
#define TT_ORACLE_H
#include "../include/truetrace_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tt_oracle_ray_counts {
    uint32_t node_visits;  /* Reps: internal node tests            */
    uint32_t tri_tests;    /* IntersectTriangle calls              */
    uint32_t blas_entries; /* TLAS -> BLAS switches                */
    uint32_t accepts;      /* candidate t passed (0 < t < best.t)  */
    uint32_t max_stack;    /* deepest stack_size reached            */
    uint32_t status;       /* 0 = wrote, 1 = Reps exhausted, 2 = stack overflow, 3 = unsupported */
} tt_oracle_ray_counts;

/* Trace rays [0, p->n_rays) (ray i lives at GlobalRays[i + (bounce odd ? W*H : 0)]).
 * Writes hits in place, and primary_info if non-NULL. counts (nullable) is indexed by i.
 * nthreads <= 1: single-threaded. Returns TT_OK or the first error (TT_ERR_STACK_OVERFLOW
 * when any ray overflowed, TT_ERR_UNSUPPORTED for cutout materials). */
tt_status tt_oracle_trace(const tt_cwbvh_node* nodes, uint32_t n_nodes,
                          const tt_cuda_triangle* tris, uint32_t n_tris,
                          const int32_t* tlas_indices, uint32_t n_tlas,
                          const tt_mesh_data* meshdata, uint32_t n_mesh,
                          const tt_material* materials, uint32_t n_mat,
                          const tt_trace_params* p, tt_ray_data* global_rays,
                          uint32_t* primary_info, const tt_col_data* global_colors,
                          tt_oracle_ray_counts* counts, int32_t nthreads);

/* Any-hit visibility (kernel_shadow / IntersectBVHShadow, IntersectionKernels.compute:264-505);
 * outputs as tt_trace_shadow. counts[i].status: 0 reached |t|, 4 occluded, 1 Reps exhausted,
 * 2 stack overflow, 3 unsupported material. */
tt_status tt_oracle_shadow(const tt_cwbvh_node* nodes, uint32_t n_nodes,
                           const tt_cuda_triangle* tris, uint32_t n_tris,
                           const int32_t* tlas_indices, uint32_t n_tlas,
                           const tt_mesh_data* meshdata, uint32_t n_mesh,
                           const tt_material* materials, uint32_t n_mat,
                           const tt_shadow_params* p, tt_shadow_ray* shadow_rays, float* visibility,
                           tt_col_data* global_colors, float* nee_pos, tt_cache_data* cache,
                           tt_oracle_ray_counts* counts, int32_t nthreads);

/* Shading / geometric normal for the hit stored in GlobalRays (see tt_resolve_normals). */
tt_status tt_oracle_resolve_normals(const tt_cuda_triangle* tris, uint32_t n_tris,
                                    const tt_mesh_data* meshdata, uint32_t n_mesh,
                                    const tt_trace_params* p, const tt_ray_data* global_rays,
                                    float* normals6);

/* Generate (RayGenKernels.compute:40-57) + CreateCameraRay (CommonData.cginc:511-567),
 * UseDoF off. cam_to_world / cam_inv_proj are Unity matrices, column-major (m[c*4+r]).
 * jitter != 0 applies random(0, pixel) - 0.5 (the !UseReCur branch) with
 * frames_accumulated/MaxBounce/CurBounce=0 as the non-ASVGF random() path. */
tt_status tt_oracle_generate(const float* cam_to_world, const float* cam_inv_proj,
                             uint32_t width, uint32_t height, float near_plane,
                             float far_plane, int32_t jitter, int32_t frames_accumulated,
                             int32_t max_bounce, tt_ray_data* global_rays);

/* Diffuse-bounce enqueue (RayTracingShader.compute:52-84, 99-124, 284, 293, 498-506): the survivors
 * of rays [0, n_rays) of the bounce's half, appended in source order to the other half. */
tt_status tt_oracle_enqueue_diffuse_bounce(const tt_cuda_triangle* tris, uint32_t n_tris, const tt_mesh_data* meshdata,
                                           uint32_t n_mesh, const tt_trace_params* p, tt_ray_data* global_rays,
                                           int32_t frames, int32_t max_bounce, uint32_t* n_next);
/* The pinned sincos of the cosine-lobe sample (both sides evaluate exactly this). */
void tt_oracle_sincos_pinned(float phi, float* s, float* c);
int32_t tt_oracle_hardware_threads(void);
/* The pinned row-f1 encoders (CommonData.cginc:479-509, :1576-1619) and HLSL pow, for tests. */
uint32_t tt_oracle_pack_rgbe(const float v[3]);
void tt_oracle_unpack_rgbe(uint32_t x, float v[3]);
uint32_t tt_oracle_encode_rgb(const float c[3]);
void tt_oracle_decode_rgb(uint32_t x, float v[3]);
float tt_oracle_pow(float x, float y);

/* TLAS refit (AssetManager.RefitTLAS, AssetManager.cs:1473-1548, with the NodePair / layer
 * structures of ConstructNewTLAS :1256-1390 and BVHRefitter.compute RefitBVHLayer / NodeUpdate /
 * NodeCompress): rewrites p, e and the quantized boxes of nodes[0, n_tlas_nodes) in place from
 * per-mesh world AABBs (mesh_aabbs: n_mesh x {BBMax[3], BBMin[3]}). Topology (meta, imask, base
 * indices) is read from the nodes and left unchanged. */
tt_status tt_oracle_tlas_refit(tt_cwbvh_node* nodes, uint32_t n_tlas_nodes, const int32_t* tlas_indices,
                               uint32_t n_tlas_indices, const float* mesh_aabbs, uint32_t n_mesh);
/* BLAS refit of a deforming / skinned mesh (ParentObject.RefitMesh, ParentObject.cs:750-917):
 * Construct (BVHRefitter.compute:72-120) into tris[TriOffset + leaf], then the refit of the mesh's
 * BLAS nodes [NodeOffset, ...). Same contract as tt_blas_refit (include/truetrace_hip.h). */
tt_status tt_oracle_blas_refit(tt_cwbvh_node* nodes, uint32_t n_nodes, tt_cuda_triangle* tris, uint32_t n_tris,
                               const tt_mesh_data* meshdata, uint32_t n_mesh, uint32_t mesh_index,
                               const float* vertices, uint32_t n_vertices, uint32_t vertex_stride,
                               const int32_t* indices, uint32_t n_mesh_tris, const int32_t* leaf_of_triangle,
                               const float* transform);

/* The R8 alpha atlas Cutout materials sample (see tt_scene_upload_alpha_atlas); NULL clears it.
 * Process-global (test infrastructure): set it before tracing a scene with Cutout materials. */
void tt_oracle_set_alpha_atlas(const uint8_t* texels, uint32_t width, uint32_t height);
/* _TextureAtlas as RGBA half texels (4 x uint16 per texel, row-major) for the stained-glass tint */
void tt_oracle_set_texture_atlas(const uint16_t* rgba_half, uint32_t width, uint32_t height);

#ifdef __cplusplus
}
#endif
#endif
