/*
 * truetrace_hip.h — C ABI of the MI355X-native CWBVH8 closest-hit engine.
 *
 * This library replaces ONE dispatch of the TrueTrace path tracer:
 *
 *     cmd.DispatchCompute(IntersectionShader, TraceKernel, CurBounceInfoBuffer, 0)
 *         TrueTrace/Resources/RayTracingMaster.cs:964-970
 *     -> kernel_trace / IntersectBVH
 *         TrueTrace/Resources/MainCompute/IntersectionKernels.compute:60-260
 *
 * It consumes the exact buffers TrueTrace's AssetManager binds for that kernel
 * (AssetManager.SetMeshTraceBuffers, TrueTrace/Resources/AssetManager.cs:75-88):
 *
 *     cwbvh_nodes      80 B  BVHNode8Data            CommonData.cginc:174-181, CommonVars.cs:413-434
 *     AggTris          88 B  CudaTriangle            CommonData.cginc:63-77,   CommonVars.cs:436-456
 *     TLASBVH8Indices   4 B  int                     CommonData.cginc:160
 *     _MeshData        88 B  MyMeshDataCompacted     CommonData.cginc:162-172, CommonVars.cs:245-255
 *     _Materials      252 B  MaterialData            CommonData.cginc:215-258
 *
 * and the per-frame buffers RayTracingMaster binds (RayTracingMaster.cs:645-650):
 *
 *     GlobalRays           48 B RayData (hits written in place)   CommonData.cginc:100-107
 *     _PrimaryTriangleInfo 16 B uint4 per pixel                   IntersectionKernels.compute:11,229-238
 *     GlobalColors         64 B ColData (only Data.w is read)     CommonData.cginc:129-138
 *
 * Conventions: extern "C", cdecl, no exceptions cross the boundary, every call
 * returns tt_status. One host thread drives a context at a time (Unity issues
 * trace dispatches from its single render thread); one context per GPU.
 *
 * Numerics (pinned; the reference leaves them to DXC + the D3D driver):
 *   rcp(x) = IEEE 1.0f/x (correctly rounded); mad(a,b,c) = fmaf(a,b,c);
 *   dot(a,b) = fmaf(a.z,b.z, fmaf(a.y,b.y, a.x*b.x));
 *   cross(a,b).x = fmaf(a.y,b.z, -(a.z*b.y)) (cyclic);
 *   mul(M,v3).r = fmaf(m[r][2],v.z, fmaf(m[r][1],v.y, m[r][0]*v.x));
 *   mul(M,(o,1)).r = fmaf(m[r][2],o.z, fmaf(m[r][1],o.y, m[r][0]*o.x)) + m[r][3];
 *   min/max = IEEE minNum/maxNum (NaN-ignoring); no other contraction;
 *   fp32 denormals are preserved (no flush) on both the GPU and the oracle.
 */
#ifndef TRUETRACE_HIP_H
#define TRUETRACE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#define TT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define TT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

#define TT_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
typedef int32_t tt_status;
enum {
    TT_OK = 0,
    TT_ERR_INVALID_ARG = 1,
    TT_ERR_OOM = 2,
    TT_ERR_HIP = 3,
    TT_ERR_UNSUPPORTED = 4,     /* e.g. a Cutout material reachable by the trace kernel */
    TT_ERR_STACK_OVERFLOW = 5,  /* a ray needed more than TT_STACK_SIZE stack entries   */
    TT_ERR_NO_DEVICE = 6,
    TT_ERR_NO_SCENE = 7
};

/* Traversal stack depth of the reference: uint2 stack[16]
 * (IntersectionKernels.compute:65). */
#define TT_STACK_SIZE 16
/* Hard loop bound of the reference: while (Reps < 1000)
 * (IntersectionKernels.compute:155). On exhaustion no hit is written. */
#define TT_MAX_REPS 1000

/* ------------------------------------------------------ buffer layouts */
/* BVHNode8Data, 80 B (CommonData.cginc:174-181). */
typedef struct tt_cwbvh_node {
    float p[3];          /* node_0xyz: quantization origin                        */
    uint32_t e_imask;    /* node_0w: e_x | e_y<<8 | e_z<<16 | imask<<24             */
    uint32_t base_child; /* node_1.x                                             */
    uint32_t base_tri;   /* node_1.y                                             */
    uint32_t meta[2];    /* node_1.zw: 8 meta bytes                              */
    uint32_t qlo_x[2], qhi_x[2]; /* node_2 */
    uint32_t qlo_y[2], qhi_y[2]; /* node_3 */
    uint32_t qlo_z[2], qhi_z[2]; /* node_4 */
} tt_cwbvh_node;
TT_STATIC_ASSERT(sizeof(tt_cwbvh_node) == 80, "BVHNode8Data is 80 bytes");

/* CudaTriangle, 88 B (CommonData.cginc:63-77, CommonVars.cs:436-456). */
typedef struct tt_cuda_triangle {
    float pos0[3];
    float posedge1[3];
    float posedge2[3];
    uint32_t norms[3];   /* octahedral 16:16 (CommonVars.cs:816-833)       */
    uint32_t tans[3];
    float tex0[2];
    float texedge1[2];   /* raw vertex UV, not an edge (ParentObject.cs:1039-1041) */
    float texedge2[2];
    uint32_t MatDat;
} tt_cuda_triangle;
TT_STATIC_ASSERT(sizeof(tt_cuda_triangle) == 88, "CudaTriangle is 88 bytes");

/* MyMeshDataCompacted, 88 B (CommonData.cginc:162-172, CommonVars.cs:245-255).
 * W2L is Unity's worldToLocalMatrix, column-major: element (row r, col c) at W2L[c*4+r]. */
typedef struct tt_mesh_data {
    float W2L[16];
    int32_t TriOffset;            /* C#: AggIndexCount */
    int32_t NodeOffset;           /* C#: AggNodeCount  */
    int32_t MaterialOffset;
    int32_t mesh_data_bvh_offsets;/* BLAS root (& 0x7fffffff) */
    int32_t LightTriCount;
    int32_t LightNodeOffset;
} tt_mesh_data;
TT_STATIC_ASSERT(sizeof(tt_mesh_data) == 88, "MyMeshDataCompacted is 88 bytes");

/* MaterialData, 252 B (CommonData.cginc:215-258). Only the fields the trace kernel
 * reads are named; the rest is opaque to this library. */
typedef struct tt_material {
    int32_t AlbedoTex[2];
    int32_t NormalTex[2];
    int32_t EmissiveTex[2];
    int32_t MetallicTex[2];
    int32_t RoughnessTex[2];
    int32_t AlphaTex[2];         /* @40  */
    int32_t MatCapMask[2];
    int32_t MatCapTex[2];
    float surfaceColor[3];       /* @64  */
    float emmissive;
    float EmissionColor[3];
    uint32_t Tag;                /* @92: flag bits, Invisible = bit 7 (GlobalDefines.cginc:46) */
    float roughness;
    int32_t MatType;             /* @100: CutoutIndex = 2 (GlobalDefines.cginc:24) */
    float transmittanceColor[3];
    float ior;
    float metallic, sheen, sheenTint, specularTint, clearcoat, clearcoatGloss;
    float anisotropic, flatness, diffTrans;
    float specTrans;             /* @156 */
    float Specular, scatterDistance;
    float AlbedoTexScale[4];     /* @168 */
    float MetallicRemap[2];
    float RoughnessRemap[2];
    float AlphaCutoff;           /* @200 */
    float NormalStrength, Hue, Saturation, Contrast, Brightness;
    float BlendColor[3];
    float BlendFactor;
    float SecondaryTexScale[2];
    float Rotation;              /* @248 */
} tt_material;
TT_STATIC_ASSERT(sizeof(tt_material) == 252, "MaterialData is 252 bytes");

#define TT_MAT_CUTOUT_INDEX 2   /* GlobalDefines.cginc:24 */
#define TT_FLAG_INVISIBLE   7   /* GlobalDefines.cginc:46 */

/* RayData, 48 B (CommonData.cginc:100-107). hits = (mesh_id, triangle_id, asuint(t),
 * (uint)(u*65535) | (uint)(v*65535)<<16) — set(), CommonData.cginc:430-434. */
typedef struct tt_ray_data {
    float origin[3];
    uint32_t PixelIndex;
    float direction[3];
    float last_pdf;
    uint32_t hits[4];
} tt_ray_data;
TT_STATIC_ASSERT(sizeof(tt_ray_data) == 48, "RayData is 48 bytes");

/* ColData, 64 B (CommonData.cginc:129-138); the trace kernel reads Data.w only. */
typedef struct tt_col_data {
    float throughput[3];
    float Direct[3];
    float Indirect[3];
    uint32_t PrimaryNEERay, Flags, MetRoughIsSpec;
    float Data[4];
} tt_col_data;
TT_STATIC_ASSERT(sizeof(tt_col_data) == 64, "ColData is 64 bytes");

/* ShadowRayData, 48 B (CommonData.cginc:116-123). t > 0 / t < 0 selects the Direct vs
 * PrimaryNEERay/Indirect accumulation in the reference; max distance = |t|; t is set to 0 in
 * place when the ray is occluded (IntersectionKernels.compute:449-454). */
typedef struct tt_shadow_ray {
    float origin[3];
    float LuminanceIncomming;
    float direction[3];
    float t;
    float illumination[3];
    uint32_t PixelIndex;
} tt_shadow_ray;
TT_STATIC_ASSERT(sizeof(tt_shadow_ray) == 48, "ShadowRayData is 48 bytes");

#define TT_FLAG_IS_BACKGROUND 5 /* GlobalDefines.cginc:41 */
#define TT_FLAG_SHADOW_CASTER 6 /* GlobalDefines.cginc:42 */

/* --------------------------------------------------------- context */
typedef struct tt_ctx tt_ctx;

typedef struct tt_config {
    int32_t device;        /* HIP device ordinal                                 */
    uint32_t flags;        /* reserved, 0                                        */
    uint64_t max_rays;     /* capacity of the staging ray buffer for host-pointer
                              traces (2*W*H for a wavefront ray buffer); 0 = none */
    void* stream;          /* hipStream_t to issue on; NULL = a library-owned BLOCKING
                              stream (it orders with the legacy NULL stream in both
                              directions, so a caller that writes device buffers on the
                              NULL stream, e.g. PyTorch's default stream, needs no extra
                              synchronisation before or after a call) */
} tt_config;

/* Create / destroy a per-GPU context. */
tt_status tt_ctx_create(const tt_config* cfg, tt_ctx** out);
tt_status tt_ctx_destroy(tt_ctx* ctx);
/* Last error message of this context (never NULL). */
const char* tt_last_error(const tt_ctx* ctx);
int32_t tt_abi_version(void);
/* Number of visible HIP devices (0 on a machine without a GPU). */
int32_t tt_device_count(void);

/* A non-blocking hipStream_t on a hardware queue of its own, for the concurrent launch streams of
 * one frame (parts / frame slots / the hit-record gather). Plain hipStreamCreate streams share a
 * process's few HW queues round-robin: two persistent trace grids whose streams land on one queue
 * run back to back instead of overlapping each other's drain (measured: a 2-part step then takes
 * the time of both launches, 0.45 vs 0.25 ms at an 8-GPU shard; profiles/r04/streams/). The stream is
 * made with hipExtStreamCreateWithCUMask and every CU enabled, which gives it a dedicated queue.
 * The reference has no equivalent (Unity issues one command buffer); a host that records its
 * dispatches on several queues (RayTracingMaster.cs:954-1007 per camera) would use one per queue.
 * The calling thread's current device is left unchanged. Destroy with tt_stream_destroy (it
 * synchronises the stream first). */
tt_status tt_stream_create(int32_t device, void** stream);
/* Synchronises and destroys a stream tt_stream_create made; TT_ERR_INVALID_ARG for any other handle
 * (or one destroyed already). Streams still alive when the process exits are synchronised and
 * destroyed by the library before the HIP runtime's own teardown (a CU-mask queue alive at that point
 * crashes the exit, SIGSEGV in __cxa_finalize): from the main thread's thread_local destructors (armed by
 * the first launch on such a stream, so they also run ahead of a profiler's per-thread state, e.g. under
 * rocprofv3) and, for launches made only from other threads, from an atexit handler (which runs the teardown on a
 * fresh thread: the exiting thread's per-thread profiler state is gone by then). A host that exits without
 * tt_stream_destroy -- or a Unity domain reload that skips it -- ends cleanly. A context whose stream the teardown
 * (or tt_shutdown) destroyed refuses launches with TT_ERR_INVALID_ARG and tt_ctx_destroy skips its stream sync, so
 * a host's static destructors may still destroy contexts after it. Note the main thread's teardown also runs when
 * the main thread ends with pthread_exit while other threads go on: their launches on library streams are then
 * refused -- such hosts destroy their streams themselves or call tt_shutdown. */
tt_status tt_stream_destroy(void* stream);
/* Streams made by tt_stream_create and not destroyed yet. */
uint32_t tt_stream_live_count(void);

/* ---------------------------------------------------------- scene */
/* Replaces AssetManager.SetMeshTraceBuffers (AssetManager.cs:75-88): copies the
 * aggregated buffers into HBM (the host keeps ownership of its arrays). Any previous
 * scene of the context is released. n_mat may be 0 (no material checks). */
tt_status tt_scene_upload(tt_ctx* ctx,
                          const tt_cwbvh_node* nodes, uint32_t n_nodes,
                          const tt_cuda_triangle* tris, uint32_t n_tris,
                          const int32_t* tlas_indices, uint32_t n_tlas_indices,
                          const tt_mesh_data* meshdata, uint32_t n_mesh,
                          const tt_material* materials, uint32_t n_mat);
/* The structural check tt_scene_upload runs (no GPU needed): every node, triangle, TLAS slot,
 * mesh record and (when any material is Invisible) material index reachable by IntersectBVH's
 * index arithmetic (IntersectionKernels.compute:157-213) is in range. why (nullable) receives
 * the first violation. Returns TT_OK, TT_ERR_INVALID_ARG or TT_ERR_UNSUPPORTED (Cutout). */
tt_status tt_scene_validate(const tt_cwbvh_node* nodes, uint32_t n_nodes,
                            const tt_cuda_triangle* tris, uint32_t n_tris,
                            const int32_t* tlas_indices, uint32_t n_tlas_indices,
                            const tt_mesh_data* meshdata, uint32_t n_mesh,
                            const tt_material* materials, uint32_t n_mat,
                            char* why, uint32_t why_len);
/* Per-frame TLAS refit region rewrite (BVH8AggregatedBuffer.SetData at
 * AssetManager.cs:1760 / GPU refit AssetManager.cs:1821-1822). */
tt_status tt_scene_update_nodes(tt_ctx* ctx, uint32_t first, uint32_t count,
                                const tt_cwbvh_node* nodes);
/* Per-frame transform update (MeshDataBuffer.SetData, AssetManager.cs:1825). */
tt_status tt_scene_update_meshdata(tt_ctx* ctx, uint32_t first, uint32_t count,
                                   const tt_mesh_data* meshdata);
/* _AlphaAtlas (AssetManager.cs:260-262, :309): the R8 alpha atlas Cutout materials sample
 * (IntersectionKernels.compute:35-40 with my_linear_clamp_sampler; CommonData.cginc:616 with
 * my_point_clamp_sampler in the shadow path). texels: width*height bytes, row 0 = v in [0, 1/height)
 * (the sampling orientation, i.e. D3D texture rows). Copied to HBM; replaces any previous atlas.
 * Without an atlas, a scene with Cutout materials traces with TT_ERR_UNSUPPORTED.
 * Filtering is pinned (the reference leaves it to the texture unit): point = texel
 * clamp(floor(uv*size)); linear = taps at floor(uv*size - 0.5) and +1, clamped, weights
 * f = x - floor(x), lerp(a,b,f) = a*(1-f) + b*f in x then y, texel value = byte / 255.0f. */
tt_status tt_scene_upload_alpha_atlas(tt_ctx* ctx, const uint8_t* texels, uint32_t width, uint32_t height);
/* _TextureAtlas (AssetManager.cs:82, :275; declared Texture2D<half4>, CommonData.cginc:272): the
 * albedo atlas, BC6H in the reference, handed over DECODED as RGBA half texels (4 x uint16 IEEE
 * binary16 per texel, row-major, same row orientation as the alpha atlas). The any-hit kernel reads
 * it for the stained-glass shadow tint (triangle_intersect_shadow, CommonData.cginc:613-625 with
 * IgnoreGlassShadow + StainedGlassShadows, GlobalDefines.cginc:3,8): a glass surface (specTrans == 1)
 * never occludes; it multiplies the ray's throughput by surfaceColor * (texel.xyz + 2) / 3, texel =
 * point-clamp sample at AlignUV(BaseUv, AlbedoTexScale, AlbedoTex). Copied to HBM; replaces any
 * previous atlas. Without it, tt_trace_shadow on a scene with glass materials returns
 * TT_ERR_UNSUPPORTED. */
tt_status tt_scene_upload_texture_atlas(tt_ctx* ctx, const uint16_t* rgba_half, uint32_t width, uint32_t height);

/* Per-frame TLAS refit on the GPU: AssetManager.RefitTLAS
 * (AssetManager.cs:1473-1548) with BVHRefitter.compute's RefitBVHLayer / NodeUpdate / NodeCompress
 * (:220-371). Re-quantizes p, e and the child boxes of the uploaded nodes [0, n_tlas_nodes) from
 * per-mesh world AABBs (mesh_aabbs: n_mesh x {BBMax[3], BBMin[3]}, the reference's AABB order,
 * indexed like _MeshData). The TLAS topology (meta, imask, base indices) is the uploaded one; its
 * NodePair / layer plan (ConstructNewTLAS, :1256-1390) is rebuilt on the host only when the scene
 * or its nodes change. Runs on the context stream: a later trace sees the refit TLAS. Numerics
 * pinned: e = 2^ceil(log2(extent * 0.003921569f)) exactly, float -> uint as D3D (NaN -> 0,
 * saturating). flags: TT_TRACE_DEVICE_PTRS (mesh_aabbs in HBM), TT_TRACE_ASYNC. */
tt_status tt_tlas_refit(tt_ctx* ctx, uint32_t n_tlas_nodes, const float* mesh_aabbs, uint32_t n_mesh,
                        uint32_t flags);

/* Per-frame BLAS refit of a deforming or skinned mesh (row f4), replacing ParentObject.RefitMesh
 * (ParentObject.cs:750-917): Construct (BVHRefitter.compute:72-120) re-derives each triangle of the
 * mesh from the current vertex buffer — positions and normals transformed by `transform`, AABB
 * padded by 1e-6 where flat, pos0 / posedge1 / posedge2 / packed normals written to AggTris at
 * TriOffset + leaf_of_triangle[t] — then NodeInitializer, RefitLayer (:177-212, deepest layer
 * first), NodeUpdate and NodeCompress re-quantize the mesh's CWBVH8 nodes in HBM (the plan of
 * ParentObject.Construct, :679-730, is built once per scene and cached per mesh).
 *   vertices: n_vertices x vertex_stride floats, position at +0 and normal at +3 (the raw
 *             GraphicsBuffer of SkinnedMeshRenderer.GetVertexBuffer / Mesh.GetVertexBuffer(0)),
 *   indices: 3 per triangle in Unity order (sharedMesh.triangles; submeshes concatenated, the
 *            triangle is (i0, i2, i1) as everywhere in TrueTrace),
 *   leaf_of_triangle: CWBVHIndicesBufferInverted (source triangle -> leaf-order position),
 *                     from tt_blas_copy_leaf_order.
 * Numerics pinned where the HLSL leaves them to DXC: mul as fmaf(m2, z, fmaf(m1, y, m0 * x)) (+ m3),
 * normalize(v) = v * (1 / sqrt(dot)), octahedral round = round-half-to-even. Out-of-range vertex
 * reads return zeros and out-of-range leaf writes are dropped (D3D semantics); host arrays are
 * also validated up front. The caller refits the TLAS afterwards (the mesh's bounds changed).
 * flags: TT_TRACE_DEVICE_PTRS (all three arrays in HBM), TT_TRACE_ASYNC. */
typedef struct tt_blas_refit_params {
    uint32_t mesh_index;     /* _MeshData record: its TriOffset, NodeOffset and BLAS root          */
    uint32_t n_tris;         /* triangles of the mesh (= its BLAS's triangle count)               */
    uint32_t n_vertices;
    uint32_t vertex_stride;  /* floats per vertex (Unity vertex buffer stride / 4), >= 6           */
    float transform[16];     /* "Transform", column-major (Unity Matrix4x4)                        */
    uint32_t flags;
} tt_blas_refit_params;
tt_status tt_blas_refit(tt_ctx* ctx, const tt_blas_refit_params* p, const float* vertices, const int32_t* indices,
                        const int32_t* leaf_of_triangle);

/* BLAS builder, BVH2 stage, on the GPU (row f4's builder half): BVH2Builder (BVH2Builder.cs:9-217)
 * restated level by level -- segmented AABB.Extend scans, the full-sweep SAH with the reference's
 * tie rules, stable partitions -- with outputs identical to the sequential C# recursion and to
 * tt_bvh2_build (include/truetrace_scene.h), which takes the same arguments minus the presort.
 *   aabbs:      n x {BBMax[3], BBMin[3]} primitive boxes (host),
 *   presorted:  3 x n primitive indices, axis x, y, z, each sorted by centroid with .NET's
 *               Array.Sort (tt_bvh2_presort in truetrace_scene.h: the introsort's tie order decides
 *               trees, so the sort stays on the host),
 *   final_indices (n), node_aabbs (2n x 6), node_left (2n), node_count (2n): BVH2Nodes and
 *               FinalIndices as BVH2Builder leaves them; max_depth: BuildRecursive's deepest level.
 * Synchronous on the context stream. TT_ERR_UNSUPPORTED if some node has no finite SAH split. */
tt_status tt_bvh2_build_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                               int32_t* final_indices, float* node_aabbs, int32_t* node_left, uint32_t* node_count,
                               uint32_t* max_depth);

/* The whole BLAS build after the host's presort on the GPU (row f4's builder half): the BVH2 stage
 * above, then BVH8Builder (BVH8Builder.cs:30-392) -- the cost pass bottom up over the BVH2's levels,
 * get_children / order_children / collapse top down over the CWBVH8's levels with the sequential
 * depth-first node and triangle numbering recovered from per-subtree counts -- and Aggregate
 * (CommonVars.cs:662-688). Outputs are byte-identical to tt_blas_build's: the 80-B nodes (capacity
 * max_nodes >= n - 1 suffices), their count, cwbvh_indices (n: leaf position -> source triangle)
 * and the BVH2 depth; tt_blas_build_from_cwbvh (truetrace_scene.h) assembles the tt_blas.
 * TT_ERR_UNSUPPORTED where the reference's BVH8Builder.build fails. */
/* BVH2Builder's three centroid presorts (.NET Array.Sort: IntrospectiveSort with the float-key
 * Comparison, BVH2Builder.cs:137-147) on the GPU, with the same output as tt_bvh2_presort -- the
 * unstable sort's exact swap sequence replayed level by level (median of three, the two-pointer
 * partition in closed form, insertion sort <= 16, heapsort at the depth limit). TT_ERR_UNSUPPORTED
 * (use tt_bvh2_presort) for n <= 16, non-finite centroids, or a depth-exhausted partition above
 * 65536 elements. aabbs: n x {BBMax[3], BBMin[3]} (host); presorted: 3 x n (host). */
tt_status tt_bvh2_presort_device(tt_ctx* ctx, const float* aabbs, uint32_t n, int32_t* presorted);

tt_status tt_blas_build_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                               tt_cwbvh_node* nodes, uint32_t max_nodes, uint32_t* n_nodes, int32_t* cwbvh_indices,
                               uint32_t* bvh2_depth);

/* Copies AggTris [first, first+count) back from HBM (e.g. after tt_blas_refit). */
tt_status tt_scene_read_tris(tt_ctx* ctx, uint32_t first, uint32_t count, tt_cuda_triangle* out);

/* Copies nodes [first, first+count) of the scene in HBM back to the host (e.g. the TLAS after
 * tt_tlas_refit; the reference reads its refit TLAS back for nothing, but editors and tests do).
 * On a frame-slot context (tt_ctx_share_blas) nodes [0, n_tlas_nodes) are its own TLAS.
 * Synchronizes the context stream. */
tt_status tt_scene_read_nodes(tt_ctx* ctx, uint32_t first, uint32_t count, tt_cwbvh_node* out);

/* Makes `dst` trace `src`'s scene: no copy, the device buffers of src's last tt_scene_upload (and its
 * atlases) are read by dst's launches on dst's own stream. For several contexts tracing one scene
 * concurrently (e.g. a frame's tile-interleaved parts, one context and stream each): one cache
 * footprint instead of one per context. Scene updates (tt_scene_update_*, tt_tlas_refit,
 * tt_blas_refit) go through src and are seen by dst, ordered by the library in call order across
 * the two streams, with no host synchronization: a dst launch (trace, shadow, resolve, enqueue,
 * scene read) waits on the GPU for every src mutation called before it, and a src mutation waits
 * for every dst launch called before it (HIP events; the reference's per-frame "rewrite the TLAS
 * and _MeshData, then dispatch", AssetManager.cs:1821-1825, needs no caller-side ordering). While
 * borrowers exist, src refuses tt_scene_upload / the atlas uploads and
 * tt_ctx_destroy (destroy the borrowers first); dst refuses every scene-mutating call. Same device;
 * src must not itself borrow. Synchronizes both streams. */
tt_status tt_ctx_share_scene(tt_ctx* dst, tt_ctx* src);

/* Makes `dst` a frame slot over `src`'s scene: dst traces src's BLAS nodes, triangles, materials and
 * atlases (no copy, as tt_ctx_share_scene) but has a TLAS of its own -- a copy of the TLAS nodes
 * [0, n_tlas_nodes) (the refit's count, AssetManager.cs:995: the TLAS region at the front of the node
 * array), of TLASBVH8Indices and of _MeshData, taken from src's device buffers as they are now. The
 * reference refits the TLAS and rewrites every _MeshData record each frame before it traces
 * (AssetManager.cs:1767-1826); with one scene shared by frames in flight those writes would have to
 * wait for every in-flight frame's traces. On dst, tt_tlas_refit, tt_scene_update_meshdata and
 * tt_scene_update_nodes (its TLAS nodes only) change dst's TLAS alone and are ordered only on dst's
 * stream: no wait on src or on other slots, and neither src nor other slots see them. src's own
 * TLAS-side updates (tt_tlas_refit, tt_scene_update_meshdata, TLAS-only node rewrites) are not seen by
 * dst and do not wait for it; src's BLAS-side updates (tt_blas_refit) are seen by dst and ordered
 * against its launches as with tt_ctx_share_scene, and a BLAS-side node rewrite through
 * tt_scene_update_nodes is refused while frame slots exist (TT_ERR_UNSUPPORTED). The TLAS copy lives
 * in one of 8 regions src's upload reserved behind its nodes (8 x the TLAS region; TT_ERR_UNSUPPORTED
 * when all are in use). Precondition: every node the TLAS walk reaches lies in [0, n_tlas_nodes)
 * (TT_ERR_INVALID_ARG otherwise). dst refuses tt_blas_refit and uploads. Same device; src must not
 * itself borrow. Synchronizes both streams. */
tt_status tt_ctx_share_blas(tt_ctx* dst, tt_ctx* src, uint32_t n_tlas_nodes);

/* Bytes of HBM the scene occupies (device copies + derived traversal layouts). */
tt_status tt_scene_bytes(const tt_ctx* ctx, uint64_t* bytes);

/* ---------------------------------------------------------- trace */
enum {
    TT_TRACE_DEVICE_PTRS = 1u << 0,  /* ray/info/colors pointers are HIP device memory */
    TT_TRACE_USE_RESTIRGI = 1u << 1, /* uniform UseReSTIRGI (RayTracingMaster.cs:558)   */
    TT_TRACE_USE_ASVGF = 1u << 2,    /* uniform UseASVGF    (RayTracingMaster.cs:562)   */
    TT_TRACE_STATS = 1u << 3,        /* count node visits / tri tests into tt_stats     */
    TT_TRACE_ASYNC = 1u << 4,        /* device pointers only: return without syncing    */
    /* The reference's compile-time trace variants (GlobalDefines.cginc:4,11; both off there by
     * default), tested in IntersectTriangle after the Cutout alpha test:
     *   IgnoreGlassMain  (IntersectionKernels.compute:42-44): a candidate whose material has
     *                    specTrans == 1 is skipped;
     *   IgnoreBackfacing (:45-47): at bounce 0, a candidate whose material has specTrans != 1
     *                    (out-of-range materials read as zeros, so they count) is skipped when
     *                    dot(normalize(cross(normalize(posedge1), normalize(posedge2))), dir) <= 0,
     *                    dir = the ray in the space the triangle is tested in; normalize(v) pinned
     *                    as v * (1 / sqrt(dot(v, v))), cross / dot as in the numerics contract. */
    TT_TRACE_IGNORE_GLASS = 1u << 5,
    TT_TRACE_IGNORE_BACKFACING = 1u << 6,
    /* Adaptive dequeue order (tt_trace_closest only; ignored with TT_TRACE_STATS and by
     * tt_trace_closest_indirect). The launch records, per 64-ray chunk (the 8x8 pixel tile of a
     * full-frame batch, else 64 consecutive records), the largest Reps count of its rays, and the
     * next flagged launch with the same bounce index and screen size on this context dequeues its
     * chunks longest-first within each of the scheduler's segments, so long rays start early instead
     * of forming the launch's tail. Pays on scenes whose long rays are latency-bound chains (the
     * Bistro-shaped C4: -18% primary launch time with the previous, differently jittered frame's
     * costs); neutral to slightly negative on small, L2-resident scenes. Which lane traces which ray
     * changes, what is written does not: results are identical to an unflagged launch. The
     * reference pops rays in InterlockedAdd order (IntersectionKernels.compute:79-81), so no order
     * is part of its contract. */
    TT_TRACE_ADAPTIVE_ORDER = 1u << 7
};

typedef struct tt_trace_params {
    uint32_t n_rays;         /* BufferSizes[CurBounce].tracerays                     */
    int32_t bounce;          /* CurBounce; odd bounces read GlobalRays[W*H + i]      */
    float far_plane;         /* FarPlane (miss t)                                    */
    uint32_t screen_width;   /* screen_width  (ping-pong offset, pixel decode)       */
    uint32_t screen_height;  /* screen_height                                        */
    uint32_t flags;          /* TT_TRACE_*                                            */
} tt_trace_params;

typedef struct tt_stats {
    uint64_t rays;           /* rays traced                                           */
    uint64_t node_visits;    /* internal node tests (Reps increments)                  */
    uint64_t tri_tests;      /* IntersectTriangle calls                                */
    uint64_t blas_entries;   /* TLAS -> BLAS switches                                  */
    uint64_t hits;           /* rays whose final t < FarPlane                          */
    uint64_t reps_exhausted; /* rays that hit the Reps >= 1000 bound (no write)        */
    uint64_t stack_overflows;/* rays that would have pushed a 17th stack entry        */
    uint64_t accepts;        /* candidates that passed 0 < t < best.t                  */
    float kernel_ms;         /* trace kernel time (HIP events), sync traces only       */
    uint32_t pad;
} tt_stats;

/* kernel_trace replacement (IntersectionKernels.compute:60-260).
 *   global_rays    : RayData[2*W*H] (or at least bounce-half + n_rays); hits written
 *                    in place into GlobalRays[i].hits.
 *   primary_info   : nullable uint4[W*H] (_PrimaryTriangleInfo).
 *   global_colors  : ColData[W*H]; required when primary_info != NULL and bounce > 0.
 *   stats          : nullable; counters require TT_TRACE_STATS. */
tt_status tt_trace_closest(tt_ctx* ctx, const tt_trace_params* p, tt_ray_data* global_rays,
                           uint32_t* primary_info, const tt_col_data* global_colors,
                           tt_stats* stats);
/* tt_trace_closest that also writes each ray's 16-byte hit record contiguously: ray i of the launch
 * (GlobalRays[offset + i]) -> hits_out[4 i .. 4 i + 3], the same bytes as its RayData.hits. The hit
 * records of a tile-sharded frame are what the multi-GPU path gathers; written by
 * the trace itself they need no strided copy out of GlobalRays before the collective. Requires
 * TT_TRACE_DEVICE_PTRS; hits_out is 16-byte-aligned device memory of n_rays records. Everything
 * else (flags, stats, synchronization) is tt_trace_closest's. */
tt_status tt_trace_closest_hits(tt_ctx* ctx, const tt_trace_params* p, tt_ray_data* global_rays,
                                uint32_t* primary_info, const tt_col_data* global_colors, uint32_t* hits_out);
/* kernel_trace dispatched indirectly (the reference keeps BufferSizes[CurBounce].tracerays on the
 * GPU; TransferKernel turns it into DispatchIndirect arguments, RayTracingShader.compute:736-747,
 * RayTracingMaster.cs:964-970): the launch traces min(*n_rays_dev, p->n_rays) rays, the count read
 * on the device when the kernel starts, so a bounce chain (trace -> enqueue -> trace ...) runs on the
 * context stream with no host round trip. p->n_rays is the capacity (e.g. W*H); n_rays_dev is a
 * device uint32 written by an earlier operation on the stream (tt_enqueue_diffuse_bounce_indirect,
 * or the caller's own kernel / copy). Requires TT_TRACE_DEVICE_PTRS, implies TT_TRACE_ASYNC, and
 * rejects TT_TRACE_STATS. Results are identical to tt_trace_closest with the same count. */
tt_status tt_trace_closest_indirect(tt_ctx* ctx, const tt_trace_params* p, const uint32_t* n_rays_dev,
                                    tt_ray_data* global_rays, uint32_t* primary_info,
                                    const tt_col_data* global_colors);

/* The per-chunk costs the last TT_TRACE_ADAPTIVE_ORDER launch of bounce index `bounce` recorded on this
 * context (one uint32 per 64-ray chunk: the chunk's largest Reps count, 0 when every ray of the chunk
 * stayed below 32 node steps). A full-frame launch (n_rays == W*H, W and H multiples of 8) indexes
 * chunks by 8x8 pixel tile, (y / 8) * (W / 8) + x / 8; otherwise chunk i holds rays [64 i, 64 i + 64)
 * of the launch. Copies min(max, chunks) values and sets *n to that count (0 before any flagged
 * launch). Synchronizes the context stream. Hosts use it to balance screen tiles over GPUs by the
 * previous frame's cost (bench.py's strong-scaling deal). */
tt_status tt_trace_chunk_costs(tt_ctx* ctx, int32_t bounce, uint32_t* costs, uint32_t max, uint32_t* n);
/* Per-call GPU durations (HIP events on the context stream, in issue order) since the last
 * tt_timing_reset (ring of 256 entries). One entry per call of tt_trace_closest and
 * tt_trace_shadow (the trace kernel alone), tt_generate_primary (the generate kernel),
 * tt_enqueue_diffuse_bounce (counter reset + enqueue kernel), tt_tlas_refit and tt_blas_refit
 * (the whole device-side refit). Host<->device staging copies are never inside an entry.
 * Synchronizes. */
tt_status tt_timing_reset(tt_ctx* ctx);
tt_status tt_timing_read(tt_ctx* ctx, float* ms, uint32_t max, uint32_t* n);
/* Per-call timing on (default) or off. Off: asynchronous calls (TT_TRACE_ASYNC, device-resident counts)
 * record no HIP events and add no entry; synchronous trace calls still time their kernel (stats->kernel_ms).
 * Each timed call puts two stream-ordered event markers around its kernel, which costs little beside a
 * whole-frame launch but ~15-20% of a strong-scaled rank's small launches (profiles/r05/events/): a host
 * with several frames in flight keeps timing on for the one context it measures, if any. */
tt_status tt_ctx_set_timing(tt_ctx* ctx, int32_t enabled);
/* Several frames traced as one batch on a screen B times as tall (frame j's rays carry PixelIndex + j *
 * frame_pixels, so each frame keeps its own _PrimaryTriangleInfo / GlobalColors texels): with frame_pixels
 * = W * H of one frame, tt_enqueue_diffuse_bounce(_indirect) draws the bounce direction of a ray with
 * PixelIndex p from pixel p mod frame_pixels at frames + p / frame_pixels -- frame j's bounce rays are those
 * of the same pixels traced alone with frames_accumulated = frames + j (RayTracingShader.compute:52-84's
 * random(1, pixel) per frame). 0 (the default): PixelIndex as-is, the reference's form. */
tt_status tt_ctx_set_frame_pixels(tt_ctx* ctx, uint32_t frame_pixels);

/* SIMD-efficiency diagnostics of the last synchronous TT_TRACE_STATS launch: wave loop
 * iterations, iterations with node-phase work, node-phase lanes, iterations with triangle-phase
 * work, triangle-phase lanes, active lanes (sums over waves), node-phase lanes visiting the
 * same node as the wave's first node-phase lane, wave-uniform node phases. */
tt_status tt_trace_diagnostics(const tt_ctx* ctx, uint64_t* out8);

/* Self-test of the fast reciprocal the kernels use for rcp() (numerics contract: correctly
 * rounded 1.0f/x): evaluates it and the full IEEE division for all 2^32 fp32 bit patterns on the
 * context's device and returns the number of inputs whose results differ (bitwise, NaN == NaN) in
 * *mismatches; 0 is required. Synchronous, a few milliseconds. */
tt_status tt_selftest_rcp(tt_ctx* ctx, uint64_t* mismatches);

/* Wait for all work issued on the context's stream. */
tt_status tt_sync(tt_ctx* ctx);
/* Stack overflows (rays that would have pushed a 17th entry and were dropped) of every trace and
 * any-hit launch since the previous call, TT_TRACE_ASYNC launches included: synchronizes, writes
 * the count (nullable) and resets it. Returns TT_ERR_STACK_OVERFLOW when it is non-zero. */
tt_status tt_async_overflows(tt_ctx* ctx, uint64_t* count);
/* The hipStream_t the context issues on. */
void* tt_ctx_stream(tt_ctx* ctx);

/* --------------------------------------- any-hit visibility */
/* PropogatedCacheData, 48 B (CommonData.cginc:1621-1627, PropDepth 4 at :1493): the radiance-cache
 * record per pixel; the any-hit kernel updates CurrentIlluminance only. */
typedef struct tt_cache_data {
    uint32_t samples[4][2];
    uint32_t throughput;
    uint32_t pathLength;
    uint32_t CurrentIlluminance; /* @40: EncodeRGB log-luminance colour */
    uint32_t Norm;
} tt_cache_data;
TT_STATIC_ASSERT(sizeof(tt_cache_data) == 48, "PropogatedCacheData is 48 bytes");

/* tt_shadow_params.flags beyond TT_TRACE_DEVICE_PTRS / _STATS / _ASYNC / _USE_RESTIRGI: */
enum {
    /* the reference's RadianceCache define (GlobalDefines.cginc:15, on in its shipped define set):
     * selects the #ifdef RadianceCache accumulations of IntersectionKernels.compute:463-482 */
    TT_SHADOW_RADIANCE_CACHE = 1u << 7,
    /* VisabilityCheckCompute semantics (CommonData.cginc:710-819): the same any-hit traversal with
     * max distance = t as given (not |t|); visibility = (1,1,1,1) when no occluder is found -- the
     * Reps bound included -- else (0,0,0,0); nothing else is written */
    TT_SHADOW_VISIBILITY_CHECK = 1u << 8
};

typedef struct tt_shadow_params {
    uint32_t n_rays;         /* BufferSizes[CurBounce].shadow_rays                      */
    int32_t bounce;          /* CurBounce                                               */
    uint32_t screen_width;   /* NEEPosA pixel decode                                    */
    uint32_t screen_height;
    uint32_t flags;          /* TT_TRACE_DEVICE_PTRS | TT_TRACE_STATS | TT_TRACE_ASYNC  */
} tt_shadow_params;

/* Replaces one kernel_shadow dispatch (IntersectionKernels.compute:264-505, HardwareRT off,
 * AdvancedAlphaMapped / IgnoreGlassShadow / StainedGlassShadows on): any-hit CWBVH8 traversal of
 * shadow_rays[0, n_rays) against max distance |t|, skipping IsBackground / ShadowCaster
 * materials (triangle_intersect_shadow, CommonData.cginc:593-634). Outputs:
 *   shadow_rays    : t = 0 in place for occluded rays (as the reference);
 *   visibility     : nullable float4[n_rays] = (throughput.xyz, 1) for rays that reached |t|,
 *                    (0,0,0,0) occluded, (0,0,0,-1) Reps bound hit (the reference writes nothing);
 *   global_colors  : nullable ColData[W*H]; at bounce 0, for unoccluded rays with t >= 0,
 *                    Direct += illumination * throughput (:466-470);
 *   nee_pos        : nullable float4[W*H]; at bounce 0, unoccluded rays write
 *                    (origin + direction * |t|, 0) to NEEPosA[pixel] (:461).
 * tt_trace_shadow_ex (below) adds the radiance-cache, PrimaryNEERay and bounce > 0 Indirect
 * accumulations (RGBE / log-luminance encodings). Scenes with Cutout materials need the
 * alpha atlas and scenes with glass (specTrans == 1, stained-glass tint) the texture atlas;
 * without them the call returns TT_ERR_UNSUPPORTED. throughput = product of the glass tints of the
 * surfaces crossed, in traversal order (IEEE: t *= (c * (x + 2)) / 3 per component). */
tt_status tt_trace_shadow(tt_ctx* ctx, const tt_shadow_params* p, tt_shadow_ray* shadow_rays, float* visibility,
                          tt_col_data* global_colors, float* nee_pos, tt_stats* stats);
/* The full kernel_shadow output contract of a ray that reaches |t| (IntersectionKernels.compute:
 * 457-485, TerrainExists false), beyond tt_trace_shadow's Direct / NEEPosA, pixel = PixelIndex
 * (writes to pixels >= W*H are dropped):
 *   TT_SHADOW_RADIANCE_CACHE set (the reference's define set):
 *     cache_buffer[pixel].CurrentIlluminance = EncodeRGB(DecodeRGB(it) + illumination * throughput
 *         * ((!UseReSTIRGI || t >= 0) ? 1 : unpackRGBE(asuint(LuminanceIncomming))))  (cache nullable);
 *     t >= 0: bounce 0: Direct += illumination * throughput;
 *     t <  0: bounce != 0 && (UseReSTIRGI || Data.w == bounce):
 *                 Indirect += illumination * throughput * (UseReSTIRGI ? unpackRGBE(Lum..) : 1)
 *             else PrimaryNEERay = packRGBE(pow(unpackRGBE(PrimaryNEERay), 2.2f)
 *                                           + pow(illumination, rcp(2.2f)) * throughput);
 *   flag clear (#ifndef RadianceCache):
 *     t >= 0: bounce 0: Direct += illumination * throughput, else Indirect += the same;
 *     t <  0: bounce != 0 && !UseReSTIRGI && Data.w == -1: Indirect += illumination * throughput,
 *             else the PrimaryNEERay update above.
 * UseReSTIRGI = TT_TRACE_USE_RESTIRGI. The encoders and HLSL pow are pinned (driver-defined in the
 * reference): log2 / exp2 evaluated in double with a fixed series and rounded once to float, exact
 * floor(log2) / pow(2, n), round-half-to-even, D3D float -> uint; see csrc/tt_encode.h. One shadow
 * ray per pixel per launch (the reference's updates are not atomic either). */
tt_status tt_trace_shadow_ex(tt_ctx* ctx, const tt_shadow_params* p, tt_shadow_ray* shadow_rays, float* visibility,
                             tt_col_data* global_colors, float* nee_pos, tt_cache_data* cache_buffer,
                             tt_stats* stats);
/* tt_trace_shadow_ex dispatched indirectly (BufferSizes[CurBounce].shadow_rays on the GPU,
 * TransferKernel Type 1): traces min(*n_rays_dev, p->n_rays) shadow rays; as
 * tt_trace_closest_indirect (device pointers, asynchronous, no stats). */
tt_status tt_trace_shadow_ex_indirect(tt_ctx* ctx, const tt_shadow_params* p, const uint32_t* n_rays_dev,
                                      tt_shadow_ray* shadow_rays, float* visibility, tt_col_data* global_colors,
                                      float* nee_pos, tt_cache_data* cache_buffer);

/* ------------------------------------------------- attribute resolve */
/* Parity aid for "normals within 1e-5": per hit, the interpolated shading normal
 * (GetTriangleNormal, CommonData.cginc:904-911) with Inverse = transpose of W2L's
 * 3x3 (RayTracingShader.compute:99-118) and the geometric normal. Out: float[6] per
 * ray (shading xyz, geometric xyz); misses write zeros. */
tt_status tt_resolve_normals(tt_ctx* ctx, const tt_trace_params* p,
                             const tt_ray_data* global_rays, float* normals6);

/* ------------------------------------------- ray producers */
/* Camera for Generate (RayGenKernels.compute:40-57) + CreateCameraRay (CommonData.cginc:511-567),
 * UseDoF off. Matrices are Unity's cameraToWorldMatrix and projectionMatrix.inverse,
 * column-major (m[c*4+r]). */
typedef struct tt_camera {
    float cam_to_world[16];
    float cam_inv_proj[16];
    float near_plane;
    float far_plane;
    uint32_t width;
    uint32_t height;
    int32_t jitter;             /* 1: random(0,pixel)-0.5 sub-pixel jitter (the !UseReCur path) */
    int32_t frames_accumulated; /* random() seed inputs (non-ASVGF branch)                      */
    int32_t max_bounce;
    uint32_t flags;             /* TT_TRACE_DEVICE_PTRS [| TT_TRACE_ASYNC]                      */
} tt_camera;

/* Writes W*H RayData (hits = (0,0,asuint(FarPlane),0)) into GlobalRays[pixel]. With device rays and
 * TT_TRACE_ASYNC the call returns without waiting (the camera is staged through pinned memory), so a
 * whole frame -- Generate, trace, enqueue, indirect trace -- is issued with no host synchronization. */
tt_status tt_generate_primary(tt_ctx* ctx, const tt_camera* cam, tt_ray_data* global_rays);

/* Diffuse-lobe next-bounce enqueue for the rays traced at p->bounce (the subset of kernel_shade
 * in RayTracingShader.compute:52-84, 99-122, 293, 498-506 that produces the next ray): hits
 * spawn a cosine-weighted ray about the shading normal, offset 1e-4 along the geometric normal;
 * misses terminate. Survivors are compacted into the other half of the ping-pong buffer in
 * source order (a stable single-pass scan: 4096-ray tiles, block ballot / LDS prefix, decoupled
 * look-back over the preceding tiles' counts; the reference's InterlockedAdd order,
 * RayTracingShader.compute:500, is whatever its atomics serialise to); *n_next receives their
 * count. */
tt_status tt_enqueue_diffuse_bounce(tt_ctx* ctx, const tt_trace_params* p, tt_ray_data* global_rays,
                                    int32_t frames_accumulated, int32_t max_bounce, uint32_t* n_next);
/* The same enqueue with device-resident counts: reads the traced count from n_rays_dev (nullable:
 * p->n_rays; otherwise p->n_rays is the capacity) and writes the survivor count to the device uint32
 * n_next_dev (BufferSizes[CurBounce + 1].tracerays) instead of returning it: no synchronization, so
 * it chains with tt_trace_closest_indirect. Requires TT_TRACE_DEVICE_PTRS. */
tt_status tt_enqueue_diffuse_bounce_indirect(tt_ctx* ctx, const tt_trace_params* p, const uint32_t* n_rays_dev,
                                             tt_ray_data* global_rays, int32_t frames_accumulated,
                                             int32_t max_bounce, uint32_t* n_next_dev);

/* ------------------------------- multi-GPU tile-sharded frames */
/* The reference traces a frame with one dispatch per bounce on one GPU
 * (RayTracingMaster.cs:954-1007: Generate, then kernel_trace / kernel_shade per bounce). A group
 * traces a frame over several MI355X: the scene is replicated per device, the screen is cut into
 * tile x tile pixel tiles dealt round-robin (tile t to rank t % world), every member generates and
 * traces the primary rays of its tiles on its own device and streams, and the 16-B primary hit
 * records go to rank 0 with ONE RCCL gather (ncclSend / ncclRecv in a single group), where they are
 * scattered back to screen order: hits_out[pixel] holds exactly the RayData.hits tt_generate_primary
 * + tt_trace_closest write at GlobalRays[pixel]. Optionally each member then continues its own rays
 * (bounce 1: tt_enqueue_diffuse_bounce_indirect + tt_trace_closest_indirect on its stream) -- the
 * bounce chain never leaves the device.
 *
 * Two ways to form a group, one code path after that:
 *   tt_group_create       one process drives n devices (ncclCommInitAll): the C# / Unity host shape;
 *   tt_group_create_rank  one process per device (ncclCommInitRank over a tt_group_unique_id that
 *                         the host distributes), the shape of bench.py under torch.distributed.run.
 * RCCL is loaded at run time (dlopen "librccl.so.1": the copy a process already has, e.g. PyTorch's,
 * or the system ROCm one); TT_GROUP_COPY_GATHER gathers with device-to-device copies instead (one
 * process only; lets several members share one device, for tests on a one-GPU machine).
 * Frames are asynchronous when TT_TRACE_ASYNC is set: frame k uses slot k % slots (its own rays,
 * contexts and dedicated streams per member), so a member's next frame overlaps the previous one's
 * drain and gather; tt_group_sync waits for everything. */
typedef struct tt_group tt_group;

enum {
    TT_GROUP_COPY_GATHER = 1u << 0, /* gather with hipMemcpyAsync instead of RCCL (tt_group_create only)   */
    TT_GROUP_BOUNCE = 1u << 1,      /* each member traces bounce 1 of its primary hits (diffuse enqueue)  */
    TT_GROUP_INFO = 1u << 2         /* gather the bounce-0 _PrimaryTriangleInfo texels too (info_out)      */
};

typedef struct tt_group_config {
    uint32_t width, height; /* the screen (hits_out holds width * height records)                      */
    uint32_t tile;          /* tile edge in pixels, a multiple of 8 (0: 64)                               */
    uint32_t slots;         /* frames in flight per member (0: 2; at most 8)                              */
    uint32_t flags;         /* TT_GROUP_*                                                                 */
    uint32_t batch;         /* frames per call, B (0: 1; at most 16): a call traces frames_accumulated + b,
                               b < B, of one camera as ONE screen B frames tall (frame b's PixelIndex + b W H,
                               tt_ctx_set_frame_pixels): a launch's ramp-up and drain and every per-frame call
                               are paid once per B frames -- for progressive accumulation of a still view (the
                               next B samples' pose is known); B = 1 for a moving camera                  */
} tt_group_config;

/* One process, n devices (devices[i] is member i's HIP ordinal; member 0 is rank 0 and receives the
 * gather). Without TT_GROUP_COPY_GATHER the devices must be distinct. */
tt_status tt_group_create(const int32_t* devices, uint32_t n, const tt_group_config* cfg, tt_group** out);
/* The 128-byte RCCL unique id for tt_group_create_rank (rank 0 makes it; the host broadcasts it). */
tt_status tt_group_unique_id(uint8_t id[128]);
/* One member per process: this process is rank `rank` of `world` and drives HIP device `device`.
 * Every rank calls it concurrently (RCCL's init is collective). */
tt_status tt_group_create_rank(const uint8_t id[128], uint32_t world, uint32_t rank, int32_t device,
                               const tt_group_config* cfg, tt_group** out);
/* Synchronizes, tears the communicators, contexts and streams down. */
tt_status tt_group_destroy(tt_group* g);
const char* tt_group_last_error(const tt_group* g);
/* Members this process drives (n for tt_group_create, 1 for tt_group_create_rank). */
uint32_t tt_group_local_members(const tt_group* g);
/* Member m's scene context (slot 0's; the other slots share its scene, tt_ctx_share_scene): scene
 * updates (tt_scene_update_*, tt_tlas_refit, tt_blas_refit) go through it, and every slot sees them
 * in call order. NULL for m out of range. */
tt_ctx* tt_group_member_ctx(tt_group* g, uint32_t m);
/* tt_scene_upload on every local member (the scene replicated per device). */
tt_status tt_group_scene_upload(tt_group* g, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                                const tt_cuda_triangle* tris, uint32_t n_tris,
                                const int32_t* tlas_indices, uint32_t n_tlas_indices,
                                const tt_mesh_data* meshdata, uint32_t n_mesh,
                                const tt_material* materials, uint32_t n_mat);
/* tt_scene_upload_alpha_atlas / tt_scene_upload_texture_atlas on every local member (after the scene upload:
 * a scene with Cutout materials needs the alpha atlas before it is traced). */
tt_status tt_group_scene_upload_alpha_atlas(tt_group* g, const uint8_t* texels, uint32_t width, uint32_t height);
tt_status tt_group_scene_upload_texture_atlas(tt_group* g, const uint16_t* rgba_half, uint32_t width, uint32_t height);
/* Per-frame scene updates on every local member, between frames (AssetManager.cs:1760-1825 on each device):
 * tt_scene_update_meshdata / tt_scene_update_nodes / tt_tlas_refit of each member's scene context. The frame slots
 * borrow that scene, and the library orders each update after the traces already issued and before later ones, so
 * no synchronisation is needed. tt_group_tlas_refit takes host AABBs (flags: TT_TRACE_ASYNC). */
tt_status tt_group_scene_update_meshdata(tt_group* g, uint32_t first, uint32_t count, const tt_mesh_data* meshdata);
tt_status tt_group_scene_update_nodes(tt_group* g, uint32_t first, uint32_t count, const tt_cwbvh_node* nodes);
tt_status tt_group_tlas_refit(tt_group* g, uint32_t n_tlas_nodes, const float* mesh_aabbs, uint32_t n_mesh,
                              uint32_t flags);
/* One frame: Generate (cam: width / height must be the group's; TT_TRACE_DEVICE_PTRS implied) on every
 * member for its tiles, the primary trace, the gather to rank 0 and, with TT_GROUP_BOUNCE, bounce 1 on
 * every member. hits_out: on the process holding rank 0, a 16-byte-aligned buffer of batch * width * height uint4
 * records (frame b's screen-order records at [b W H, (b + 1) W H)) -- device memory of rank 0's device, or host
 * memory (then the frame must be
 * synchronous: the records are staged on rank 0's device and copied back); ignored (may be NULL) elsewhere.
 * info_out (TT_GROUP_INFO; else ignored): batch * width * height uint4 _PrimaryTriangleInfo texels, as hits_out, the
 * bounce-0 form tt_trace_closest writes (IntersectionKernels.compute:229-238), same kind of memory as hits_out;
 * each member packs its texels behind its hit records, so they travel in the same RCCL group.
 * flags: TT_TRACE_ASYNC (return without waiting; device hits_out only). */
tt_status tt_group_trace_frame(tt_group* g, const tt_camera* cam, uint32_t* hits_out, uint32_t* info_out,
                               uint32_t flags);
/* Waits for every frame issued so far (all members, all slots, the gathers). */
tt_status tt_group_sync(tt_group* g);
/* Of the latest call, member m: its primary ray count (batch x its pixels), its bounce-1 ray count (0 without
 * TT_GROUP_BOUNCE) and the device pointer of its ray buffer (RayData[batch * width * height + primary]: primary
 * rays at [0, primary) -- frame b's at [b n, (b + 1) n) --, bounce-1 rays at [batch * width * height, + bounce),
 * each frame's survivors after the previous frame's). Synchronizes. Any output may be NULL. */
tt_status tt_group_frame_rays(tt_group* g, uint32_t m, uint32_t* n_primary, uint32_t* n_bounce,
                              tt_ray_data** rays_dev);
/* The shard arithmetic (host only, no GPU): the pixels rank `rank` of `world` traces, in trace order --
 * its tiles t = rank, rank + world, ... (row-major tile ids over ceil(W / tile) x ceil(H / tile)), inside a
 * tile 8 x 8 pixel blocks in row-major block order, pixels row-major inside a block (so the 64 rays a
 * wave dequeues together are one 8 x 8 screen patch). world == 1 is the identity (pixel i = ray i, the
 * full-frame order the trace kernel swizzles itself). Writes min(count, max) indices, sets *n to count. */
tt_status tt_group_tile_pixels(uint32_t width, uint32_t height, uint32_t tile, uint32_t world, uint32_t rank,
                               uint32_t* pixels, uint32_t max, uint32_t* n);

/* ------------------------------------------------------------- shutdown */
/* Synchronizes and destroys every stream tt_stream_create made that is still alive. For hosts that
 * trace from a thread other than the main one (Unity's render thread): call it before the process or
 * the domain goes down (OnApplicationQuit / AppDomain.DomainUnload), after the last launch. Contexts
 * still alive keep their own streams; a context on a destroyed library stream refuses further launches
 * (TT_ERR_INVALID_ARG). Idempotent. */
tt_status tt_shutdown(void);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* TRUETRACE_HIP_H */
