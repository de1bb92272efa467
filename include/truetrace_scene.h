/*
 * truetrace_scene.h — host-side producer of the buffers the trace kernel consumes.
 *
 * TrueTrace builds its acceleration structures on the CPU in C# (AssetManager /
 * ParentObject / BVH2Builder / BVH8Builder / CommonFunctions.Aggregate). No .NET runtime
 * exists in this environment, so this C++ library restates that pipeline (the reference's
 * host is compiled code) to produce byte-layout-identical buffers for tests and benches:
 *
 *   tt_blas_build      ParentObject.BuildTotal + Construct   ParentObject.cs:973-1111, 679-742
 *                        BVH2Builder (BLAS ctor)              BVH2Builder.cs:39-164
 *                        BVH8Builder (collapse)               BVH8Builder.cs:30-365
 *                        CommonFunctions.Aggregate            CommonVars.cs:662-688
 *   tt_scene_assemble  AssetManager.AccumulateData/UpdateTLAS AssetManager.cs:986-1138, 1610-1766
 *                        ConstructNewTLAS                     AssetManager.cs:1317-1421
 *
 * Divergences that cannot be pinned here (documented in DESIGN.md): .NET's Array.Sort tie
 * order is restated from the reference-source introsort; Mono float evaluation is assumed
 * IEEE single without contraction. Traversal parity does not depend on either: the trace
 * library consumes whatever node/triangle bytes it is given.
 */
#ifndef TRUETRACE_SCENE_H
#define TRUETRACE_SCENE_H
#include "truetrace_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One ParentObject's merged object-space mesh (ParentObject.LoadData output). */
typedef struct tt_mesh_input {
    const float* positions;   /* float3 per vertex, object space                          */
    uint32_t n_vertices;
    const float* normals;     /* float3 per vertex, nullable -> (0,1,0)                     */
    const float* tangents;    /* float4 per vertex, nullable -> (1,0,0,1)                   */
    const float* uvs;         /* float2 per vertex, nullable -> (0,0)                       */
    const int32_t* indices;   /* Unity index list, 3 per triangle                           */
    uint32_t n_indices;
    const int32_t* matdat;    /* per triangle MatDat (submesh material), nullable -> 0       */
    float lossy_scale[3];     /* transform.lossyScale: AABB padding 0.001/scale (:462-463)  */
} tt_mesh_input;

typedef struct tt_blas tt_blas;

typedef struct tt_blas_info {
    uint32_t n_nodes;         /* BVH.cwbvhnode_count                          */
    uint32_t n_tris;          /* AggTriangles.Length                          */
    uint32_t bvh2_depth;      /* deepest BVH2 leaf                            */
    float aabb_min[3];        /* aabb_untransformed (ConstructAABB :1143-1149) */
    float aabb_max[3];
    double build_seconds;
} tt_blas_info;

tt_status tt_blas_build(const tt_mesh_input* mesh, tt_blas** out);
/* The same build in three steps, so the BVH2 stage can run on the GPU (tt_bvh2_build_device in
 * truetrace_hip.h) with byte-identical results:
 *   tt_blas_prepare_aabbs   BuildTotal's triangle AABBs (n_indices / 3 x {BBMax[3], BBMin[3]}),
 *   tt_bvh2_presort         BVH2Builder's three centroid presorts (.NET Array.Sort), 3 x n indices,
 *   tt_blas_build_from_bvh2 Construct's BVH8 stage + Aggregate over a BVH2 as tt_bvh2_build writes it. */
tt_status tt_blas_prepare_aabbs(const tt_mesh_input* mesh, float* aabbs_maxmin);
tt_status tt_bvh2_presort(const float* aabbs_maxmin, uint32_t n, int32_t* presorted);
tt_status tt_blas_build_from_bvh2(const tt_mesh_input* mesh, const int32_t* final_indices, const float* node_aabbs,
                                  const int32_t* node_left, const uint32_t* node_count, uint32_t bvh2_depth,
                                  tt_blas** out);
/* ... or over finished CWBVH8 nodes + cwbvh_indices (tt_blas_build_device in truetrace_hip.h). */
tt_status tt_blas_build_from_cwbvh(const tt_mesh_input* mesh, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                                   const int32_t* cwbvh_indices, uint32_t bvh2_depth, tt_blas** out);
/* The same with the triangle preparation done once: tt_blas_prepare keeps BuildTotal's AggTriangles
 * (and writes the AABBs the device builder consumes); tt_blas_build_from_cwbvh_prepared then only
 * permutes them into leaf order. The handle is consumed (freed) by the build call on success and
 * on failure; tt_blas_prep_free releases one that is not built. */
typedef struct tt_blas_prep tt_blas_prep;
tt_status tt_blas_prepare(const tt_mesh_input* mesh, float* aabbs_maxmin, tt_blas_prep** out);
tt_status tt_blas_build_from_cwbvh_prepared(tt_blas_prep* prep, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                                            const int32_t* cwbvh_indices, uint32_t bvh2_depth, tt_blas** out);
void tt_blas_prep_free(tt_blas_prep* prep);
tt_status tt_blas_get_info(const tt_blas* b, tt_blas_info* info);
/* Copies the packed nodes (80 B) and the leaf-ordered triangles (88 B). */
tt_status tt_blas_copy(const tt_blas* b, tt_cwbvh_node* nodes, tt_cuda_triangle* tris);
/* CWBVHIndicesBufferInverted (ParentObject.cs:691-694): for each source triangle, its position in
 * the leaf-ordered triangle array — the map tt_blas_refit's Construct writes through. */
tt_status tt_blas_copy_leaf_order(const tt_blas* b, int32_t* leaf_of_triangle);
void tt_blas_free(tt_blas* b);

/* AssetManager aggregation. Order of meshes = RenderQue parents, then instances. */
typedef struct tt_parent_desc {
    const tt_blas* blas;
    float local_to_world[16];   /* transform.localToWorldMatrix (column-major)  */
    float world_to_local[16];   /* transform.worldToLocalMatrix (column-major)  */
    uint32_t material_count;    /* ParentObject.MatOffset                      */
} tt_parent_desc;

typedef struct tt_instance_desc {
    uint32_t instance_parent;   /* index into instance_parents[]                */
    float local_to_world[16];
    float world_to_local[16];
} tt_instance_desc;

typedef struct tt_scene_build tt_scene_build;

typedef struct tt_scene_build_info {
    uint32_t n_nodes;           /* AggNodeCount (TLAS region 2*(P+I) included) */
    uint32_t n_tris;
    uint32_t n_tlas_indices;    /* = number of meshes (P + I)                  */
    uint32_t n_mesh;
    uint32_t tlas_nodes;        /* TLASBVH8.cwbvhnode_count                    */
    uint32_t pad;
} tt_scene_build_info;

/* instance_parents are the InstanceData.RenderQue ParentObjects: their BLAS/triangles are
 * aggregated after the RenderQue parents but they get no MeshData of their own
 * (AssetManager.cs:1140-1185, 1704-1750). */
tt_status tt_scene_assemble(const tt_parent_desc* parents, uint32_t n_parents,
                            const tt_parent_desc* instance_parents, uint32_t n_instance_parents,
                            const tt_instance_desc* instances, uint32_t n_instances,
                            tt_scene_build** out);
tt_status tt_scene_build_get_info(const tt_scene_build* s, tt_scene_build_info* info);
tt_status tt_scene_build_copy(const tt_scene_build* s, tt_cwbvh_node* nodes,
                              tt_cuda_triangle* tris, int32_t* tlas_indices,
                              tt_mesh_data* meshdata);
/* The per-mesh world AABBs the TLAS was built over (AssetManager MeshAABBs, CreateAABB
 * :1239-1249), n_mesh x {BBMax[3], BBMin[3]} — the input tt_tlas_refit takes per frame. */
tt_status tt_scene_build_copy_mesh_aabbs(const tt_scene_build* s, float* out6);
void tt_scene_build_free(tt_scene_build* s);

/* Standalone pieces, exposed for unit tests. */
/* CommonFunctions.PackOctahedral (CommonVars.cs:816-833) */
uint32_t tt_pack_octahedral(float x, float y, float z);
/* BVH2 (BVH2Builder.cs): AABBs as {max xyz, min xyz} x n (the C# AABB field order).
 * Writes FinalIndices (n) and BVH2 nodes as {aabb(6 floats), left, count} (2n entries). */
tt_status tt_bvh2_build(const float* aabbs_maxmin, uint32_t n, int32_t* final_indices,
                        float* node_aabbs, int32_t* node_left, uint32_t* node_count);
/* .NET Framework IntrospectiveSort with a float-key Comparison (BVH2Builder.cs:137-147). */
void tt_dotnet_sort_by_key(int32_t* items, uint32_t n, const float* keys);

#ifdef __cplusplus
}
#endif
#endif
