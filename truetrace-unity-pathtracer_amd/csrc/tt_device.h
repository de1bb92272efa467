// tt_device.h — device-side layouts derived at tt_scene_upload from the reference buffers,
// and the launch-argument blocks shared by tt_trace.hip and tt_api.cpp.
#ifndef TT_DEVICE_H
#define TT_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/truetrace_hip.h"

// rcp(x) of the reference (IntersectionKernels.compute:22,145,214), pinned to the correctly rounded
// IEEE 1.0f / x (numerics contract, include/truetrace_hip.h). v_rcp_f32 plus one FMA Newton step
// (e = fma(-a, r, 1), r' = fma(e, r, r)) equals the correctly rounded quotient for every input whose
// biased exponent is 1..252 -- checked exhaustively over all 2^32 inputs on gfx950
// (tt_selftest_rcp, tests/test_gpu_parity.py) -- so only zeros, denormals, |a| >= 2^126 (denormal
// result), infinities and NaNs take the compiler's full division sequence (v_div_scale/fmas/fixup).
#ifndef TT_FAST_RCP
#define TT_FAST_RCP 1  // 0: always the full division sequence (A/B measurement)
#endif
__device__ __forceinline__ float rcp_rn(float a) {
    if (!TT_FAST_RCP) return 1.0f / a;
    const uint32_t e = (__float_as_uint(a) >> 23) & 0xffu;
    if (__builtin_expect(e - 1u < 252u, 1)) {
        const float r = __builtin_amdgcn_rcpf(a);
        return __builtin_fmaf(__builtin_fmaf(-a, r, 1.0f), r, r);
    }
    return 1.0f / a;
}

// Byte stride of the node array the kernels read (tt_traverse.h node_offset): 80 = the reference's
// cwbvh_nodes as uploaded; 128 = a derived copy, one node per 128-B line (tt_api.hip keeps it in step).
#ifndef TT_NODE_STRIDE
#define TT_NODE_STRIDE 80
#endif

// Traversal-layout triangle, 48 B: the 36 B of positions the Moller-Trumbore test reads
// (CudaTriangle pos0/posedge1/posedge2, CommonData.cginc:63-66) + MatDat, padded so one
// triangle is three 16-B loads. Built from AggTris at upload; AggTris itself also stays in
// HBM for the attribute resolve.
struct TriPos {
    float p0x, p0y, p0z, e1x;
    float e1y, e1z, e2x, e2y;
    float e2z;
    uint32_t matdat;
    uint32_t pad0, pad1;
};
static_assert(sizeof(TriPos) == 48, "TriPos size");

// Traversal-layout mesh record, 64 B: W2L rows 0-2 (row-major, 12 floats) + the four offsets
// IntersectBVH reads on a TLAS->BLAS switch (IntersectionKernels.compute:197-213).
struct MeshGpu {
    float m[12];      // m[r*4+c] = W2L(r, c)
    int32_t TriOffset;
    int32_t NodeOffset;
    int32_t MaterialOffset;
    int32_t root;     // mesh_data_bvh_offsets & 0x7fffffff
};
static_assert(sizeof(MeshGpu) == 64, "MeshGpu is 64 bytes");

// The mesh record of TLASBVH8Indices[i], stored at i (80 B): a TLAS leaf reaches its instance's
// transform and offsets with one round of independent loads instead of the dependent
// TLASBVH8Indices -> _MeshData pair (IntersectionKernels.compute:197-213). Rebuilt whenever the
// mesh records or the TLAS indices change.
struct LeafMesh {
    MeshGpu m;
    int32_t mesh_id;     // TLASBVH8Indices[i]
    int32_t pad[3];
};
static_assert(sizeof(LeafMesh) == 80, "LeafMesh is 80 bytes");

// Control block, zeroed by hipMemsetAsync before every trace launch.
struct TraceControl {
    uint32_t seg_ticket[8 * 32];  // per-segment dequeue tickets, one 128-B line each
    uint32_t err_overflow;    // rays that overflowed the 16-entry stack
    uint32_t err_unsupported; // cutout material reached (never with a validated scene)
    uint32_t pad[2];
    unsigned long long stats[8];  // rays, nodes, tris, blas, hits, reps_exhausted, overflow, accepts
    unsigned long long diag[8];   // STATS-build SIMD diagnostics: wave iterations, node-phase iterations,
                                  // node-phase lanes, tri-phase iterations, tri-phase lanes, active lanes,
                                  // node lanes sharing the first lane's node, wave-uniform node phases
};

// Per-material record for the Cutout alpha test (row f3), 32 B; only uploaded when a Cutout
// material exists. The per-material word in mat_tag carries MaterialData.Tag plus bit 31 = Cutout.
struct CutoutMat {
    int32_t alpha_tex[2];   // MaterialData.AlphaTex (atlas rectangle, 15-bit fixed point)
    float cutoff;           // MaterialData.AlphaCutoff
    uint32_t pad;
    float scale[4];         // MaterialData.AlbedoTexScale
};
static_assert(sizeof(CutoutMat) == 32, "CutoutMat is 32 bytes");
#define TT_MATWORD_CUTOUT 31u
#define TT_MATWORD_GLASS 30u  // specTrans == 1 (stained-glass shadow tint, any-hit kernel)

// Per-material record for the stained-glass shadow tint (row f1), 48 B; only uploaded when a
// material has specTrans == 1.
struct GlassMat {
    int32_t albedo_tex[2];  // MaterialData.AlbedoTex (atlas rectangle, 15-bit fixed point)
    float color[3];         // MaterialData.surfaceColor
    float pad0;
    float scale[4];         // MaterialData.AlbedoTexScale
    float pad1[2];
};
static_assert(sizeof(GlassMat) == 48, "GlassMat is 48 bytes");

// Everything the material checks of the triangle tests read (IntersectionKernels.compute:35-48,
// CommonData.cginc:611-617).
struct MatView {
    const uint32_t* word;         // Tag | Cutout << 31 | Glass << 30, per material
    const CutoutMat* cut;         // per material (nullptr without Cutout materials)
    const tt_cuda_triangle* raw;  // AggTris (raw UVs for the cutout sample)
    const uint8_t* atlas;         // _AlphaAtlas, R8
    uint32_t n_mat, atlas_w, atlas_h;
    const GlassMat* glass;        // per material (nullptr without glass materials)
    const uint2* tex;             // _TextureAtlas, RGBA half texels (8 B)
    uint32_t tex_w, tex_h;
};

#include "tt_fastdiv.h"

// A ray that overflows the 16-entry stack: counted in the launch's control block (reported by
// synchronous calls) and in the context's sticky counter (tt_async_overflows), which launches never
// reset, so overflows inside TT_TRACE_ASYNC chains are not lost when a later launch zeroes the block.
#define TT_REPORT_OVERFLOW(A)                          \
    do {                                               \
        atomicAdd(&(A).ctl->err_overflow, 1u);         \
        if ((A).sticky_overflow) atomicAdd((A).sticky_overflow, 1u); \
    } while (0)

// TT_ROOT_LEAF: the TLAS root (node 0) of a one-leaf TLAS -- no internal child and exactly one
// non-empty child slot, a leaf: the TLAS the reference builds for a scene of one ParentObject instance,
// such as an imported OBJ (C2, C3, C5). Its node step (IntersectionKernels.compute:157-187, the first of
// every ray, at t_max = FarPlane) is then that one child's slab test (tt_trace.hip root_leaf_hit, the
// node test's arithmetic for that child), so hits, Reps and stats are unchanged. Derived on the host
// from the node-0 bytes the device holds (tt_api.hip: known after an upload or a node update; a device
// refit of the TLAS turns it off until the next update), passed as a kernel argument (SGPRs).
#ifndef TT_ROOT_LEAF
#define TT_ROOT_LEAF 1
#endif
struct RootLeaf {
    uint32_t ok;                          // node 0 qualifies
    uint32_t qlo, qhi;                    // the child's quantized planes: bytes 0-2 = x, y, z
    uint32_t e;                           // node 0's exponent bytes (x, y, z) = node_0w & 0xffffff
    float px, py, pz;                     // node origin
    uint32_t base_child, base_tri, bits;  // node 0's base indices; the leaf's hit bits (child_bits << low5)
};
__host__ __device__ inline uint32_t rl_byte(uint32_t w, uint32_t k) { return (w >> (k * 8u)) & 0xffu; }
// w: node 0's 20 words (the 80-B layout)
__host__ __device__ inline RootLeaf root_leaf_of(const uint32_t* w) {
    RootLeaf R{};
    uint32_t count = 0, slot = 0, inner = 0;
    for (uint32_t j = 0; j < 8u; j++) {
        const uint32_t meta = rl_byte(w[6 + (j >> 2)], j & 3u);
        if (meta >> 5) {
            count++;
            slot = j;
            inner |= (meta & (meta << 1) & 0x10u) ? 1u : 0u;  // node_intersect's inner-child test
        }
    }
    const uint32_t h = slot >> 2, k = slot & 3u;
    R.ok = (w[3] >> 24) == 0u && count == 1u && inner == 0u;
    R.qlo = rl_byte(w[8 + h], k) | rl_byte(w[12 + h], k) << 8 | rl_byte(w[16 + h], k) << 16;
    R.qhi = rl_byte(w[10 + h], k) | rl_byte(w[14 + h], k) << 8 | rl_byte(w[18 + h], k) << 16;
    R.e = w[3] & 0xffffffu;
    uint32_t p[3] = {w[0], w[1], w[2]};
    R.px = __builtin_bit_cast(float, p[0]);
    R.py = __builtin_bit_cast(float, p[1]);
    R.pz = __builtin_bit_cast(float, p[2]);
    R.base_child = w[4];
    R.base_tri = w[5];
    const uint32_t meta = rl_byte(w[6 + h], k);
    R.bits = (meta >> 5) << (meta & 0x1fu);
    return R;
}

struct TraceArgs {
    const uint4* nodes;          // 80 B nodes as 5 x uint4
    uint32_t n_nodes;
    const TriPos* tris;          // traversal-layout triangles
    uint32_t n_tris;
    const int32_t* tlas;         // TLASBVH8Indices
    const MeshGpu* mesh;         // traversal-layout mesh records
    const LeafMesh* leaf;        // mesh record per TLAS index position
    const uint32_t* mat_tag;     // MaterialData.Tag per material (n_mat entries)
    uint32_t n_mat;
    MatView mat;                 // material checks (Invisible, Cutout)
    tt_ray_data* rays;           // GlobalRays
    uint32_t* info;              // _PrimaryTriangleInfo (uint4 per pixel), nullable
    const tt_col_data* colors;   // GlobalColors (bounce > 0 with info)
    TraceControl* ctl;
    uint32_t* sticky_overflow;   // stack overflows since the last tt_async_overflows (never reset by launches)
    uint2* spill;                // traversal-stack entries beyond TT_LDS_STACK, [entry][thread]
    unsigned long long* diag_times;  // TT_DIAG_TIMES builds: per wave (start, end, rays)
    uint32_t n_rays;             // rays to trace; with n_rays_dev: the capacity
    const uint32_t* n_rays_dev;  // nullable: device-resident count (BufferSizes[CurBounce].tracerays),
                                 // traced = min(*n_rays_dev, n_rays) -- the reference's DispatchIndirect
    uint32_t ray_offset;         // W*H on odd bounces
    uint32_t width, height;
    uint32_t n_pixels;           // width * height (< 2^31, checked by the API)
    float far_plane;
    int32_t bounce;
    uint32_t flags;              // TT_TRACE_*
    uint32_t tile_swizzle;       // 1: work index -> 8x8 screen tiles (n_rays == W*H, W,H % 8 == 0)
    TraceControl* ctl_next;      // the other control block: zeroed by this launch for the next one
    FastDiv div_width;           // n / width (pixel decode of finished rays)
    FastDiv div_tiles;           // n / (width / 8) (8x8 tile swizzle in the refill)
    // TT_TRACE_ADAPTIVE_ORDER (tt_trace_kernel_ord only)
    const uint32_t* order;       // nullable: work chunk -> ray chunk (64 rays), from tt_order_kernel
    uint32_t* chunk_cost;        // per ray chunk: max Reps of its rays (atomicMax, rays with Reps >= TT_ORDER_MIN_REPS)
    uint4* hits_out;             // nullable (tt_trace_closest_hits): ray i's hit record also at hits_out[i]
    RootLeaf root;               // TT_ROOT_LEAF: node 0 as a one-leaf TLAS root (root.ok = 0: the generic path)
    uint32_t tlas_base;          // node index of the context's TLAS node 0: 0, or its frame-slot overlay region
                                 // (tt_ctx_share_blas); the TLAS-level NodeOffset
};

// Adaptive-order builder (tt_order.hip): one block per scheduler segment sorts the segment's
// chunks by the previous launch's chunk costs, longest first.
struct OrderArgs {
    const uint32_t* cost;        // previous launch's per-chunk costs
    uint32_t* cost_clear;        // the map this launch's trace fills: zeroed here ([0, n_chunks))
    uint32_t n_rays, n_chunks;
    uint32_t hot;                // chunks costing less than this keep their natural order (0: sort all)
    uint32_t* order;             // out: n_chunks entries
};
hipError_t tt_launch_order(const OrderArgs& a, hipStream_t st);

// Any-hit visibility launch (tt_shadow.hip, kernel_shadow replacement).
struct ShadowArgs {
    const uint4* nodes;
    uint32_t n_nodes;
    const TriPos* tris;
    uint32_t n_tris;
    const int32_t* tlas;
    const MeshGpu* mesh;
    const LeafMesh* leaf;
    const uint32_t* mat_tag;     // MaterialData.Tag per material (n_mat entries)
    uint32_t n_mat;
    MatView mat;                 // material checks (IsBackground / ShadowCaster, Cutout)
    tt_shadow_ray* rays;         // ShadowRaysBuffer (t = 0 written for occluded rays)
    float4* visibility;          // nullable, per ray
    tt_col_data* colors;         // nullable, GlobalColors (Direct += at bounce 0)
    float4* nee_pos;             // nullable, NEEPosA (bounce 0)
    tt_cache_data* cache;        // nullable, CacheBuffer (TT_SHADOW_RADIANCE_CACHE)
    TraceControl* ctl;
    uint32_t* sticky_overflow;
    uint2* spill;
    uint32_t n_rays;             // rays to trace; with n_rays_dev: the capacity
    const uint32_t* n_rays_dev;  // nullable: device-resident count (BufferSizes[CurBounce].shadow_rays)
    uint32_t width, height;
    int32_t bounce;
    uint32_t flags;
    uint32_t tlas_base;          // as TraceArgs::tlas_base
};

// The launch's ray count: the host value, or the device-resident count clamped to it (a wave-uniform
// load of a word an earlier operation on the stream wrote).
template <class Args>
__device__ __forceinline__ uint32_t launch_ray_count(const Args& A) {
    return A.n_rays_dev ? min(*A.n_rays_dev, A.n_rays) : A.n_rays;
}

#endif
