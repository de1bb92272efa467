// tt_refit.hip — per-frame BVH refit on the GPU:
//  * TLAS: the reference's AssetManager.RefitTLAS (AssetManager.cs:1473-1548) driving
//    BVHRefitter.compute (NodeInitializer :386-394, RefitBVHLayer :220-252, NodeUpdate :277-317,
//    NodeCompress :344-371) over the NodePair / ForwardStack / layer structures of
//    ConstructNewTLAS (:1256-1390);
//  * BLAS of a deforming / skinned mesh: ParentObject.RefitMesh (ParentObject.cs:750-917) —
//    Construct (BVHRefitter.compute:72-120) re-derives the triangles and their boxes from the
//    current vertex buffer, then the same NodeInitializer / RefitLayer (:177-212) / NodeUpdate /
//    NodeCompress over the plan ParentObject.Construct builds (:679-730).
//
// MI355X shape: the refit is a few thousand tiny records per frame, latency- not bandwidth-bound,
// so it is ONE launch (not the reference's one dispatch per depth level, AssetManager.cs:1531-1567):
// a thread per leaf NodePair computes its box, then climbs. Each NodePair has an arrival counter;
// the thread whose arrival completes a parent's 8 slots computes that parent's box (the same union
// loop over the same 8 entries as RefitBVHLayer), then NodeUpdate of the parent's 8 child slots and
// NodeCompress of the BVH node the parent documents -- in registers, straight into the 80-B node --
// and climbs on. Boxes are handed between threads (and XCDs) with write-through sc1 stores, a
// vmcnt(0) drain and an agent-scope atomic; the completing thread reads them with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility). The counters are reset by the thread that
// completed them, so consecutive refits need no memset. On the context stream, so a trace
// enqueued after it sees the new nodes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "tt_refit.h"

namespace {

constexpr int kBlock = 256;

// pow(2, ceil(log2(x))) pinned exactly (the reference's HLSL pow/log2 are driver-defined)
__device__ __forceinline__ float pow2_ceil_log2(float x) {
    if (isnan(x) || x < 0.0f) return __int_as_float(0x7fc00000);
    if (x == 0.0f) return 0.0f;
    if (isinf(x)) return x;
    int k;
    const float m = frexpf(x, &k);
    return ldexpf(1.0f, m == 0.5f ? k - 1 : k);
}

// HLSL float -> uint (D3D: NaN -> 0, saturating)
__device__ __forceinline__ uint32_t ftou_d3d(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

// NodePair boxes for the cross-thread hand-off: 32 B {BBMax, BBMin.x | BBMin.yz, pad}, written
// through (sc1, aux 16) and read L1-bypassing (sc1) as two 16-B buffer accesses.
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_box(__amdgpu_buffer_rsrc_t bb, int32_t id, const float v[6]) {
    const uint32_t off = (uint32_t)id * 32u;
    __builtin_amdgcn_raw_buffer_store_b128(f32x4{v[0], v[1], v[2], v[3]}, bb, off, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(f32x4{v[4], v[5], 0.0f, 0.0f}, bb, off + 16u, 0, 16);
}
__device__ __forceinline__ void ld_box(__amdgpu_buffer_rsrc_t bb, int32_t id, float v[6]) {
    const uint32_t off = (uint32_t)id * 32u;
    const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bb, off, 0, 16));
    const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bb, off + 16u, 0, 16));
    v[0] = a.x;
    v[1] = a.y;
    v[2] = a.z;
    v[3] = a.w;
    v[4] = b.x;
    v[5] = b.y;
}

// RefitLayer (BLAS: leaf ranges are triangle boxes in leaf order, box_idx == nullptr) /
// RefitBVHLayer (TLAS: leaf ranges index the boxes through TLASCWBVHIndices) for a leaf NodePair:
// the union of its row's entries, in slot order, from the accumulators the reference starts with.
__device__ __forceinline__ void leaf_union(int32_t id, const int32_t* __restrict__ fwd, const int32_t* __restrict__ box_idx,
                                           const float* __restrict__ boxes, float o[6]) {
    float mx0 = -99999999.0f, mx1 = -99999999.0f, mx2 = -99999999.0f;
    float mn0 = 99999999.0f, mn1 = 99999999.0f, mn2 = 99999999.0f;
    for (int k = 0; k < 8; k++) {
        const int32_t leaf = fwd[8 * id + k];
        if (leaf <= 0) continue;  // a leaf NodePair's row holds no NodePair entries
        const int32_t v = leaf - 1;
        const int32_t start = v / 24, end = start + v % 24;
        for (int32_t i4 = start; i4 < end; i4++) {
            const float* b = boxes + 6 * (size_t)(box_idx ? box_idx[i4] : i4);  // AABB {BBMax, BBMin}
            mx0 = fmaxf(mx0, b[0]);
            mx1 = fmaxf(mx1, b[1]);
            mx2 = fmaxf(mx2, b[2]);
            mn0 = fminf(mn0, b[3]);
            mn1 = fminf(mn1, b[4]);
            mn2 = fminf(mn2, b[5]);
        }
    }
    o[0] = mx0;
    o[1] = mx1;
    o[2] = mx2;
    o[3] = mn0;
    o[4] = mn1;
    o[5] = mn2;
}

// An internal NodePair `p` (all 8 children NodePairs complete): its box is the union of the
// children's boxes in slot order (RefitBVHLayer / RefitLayer), then NodeUpdate of the 8 child
// slots against it and NodeCompress of the BVH node it documents: full uints shifted and OR-ed, as
// the reference packs them (out-of-range quantized values spill into the neighbouring bytes there
// too). The 8 children boxes are loaded once, all in flight together.
__device__ __forceinline__ void internal_pair(int32_t p, const int32_t* __restrict__ fwd, __amdgpu_buffer_rsrc_t bb,
                                              tt_cwbvh_node* __restrict__ node, float par[6]) {
    float cb[8][6];
#pragma unroll
    for (int k = 0; k < 8; k++) ld_box(bb, -fwd[8 * p + k] - 1, cb[k]);
    float mx0 = -99999999.0f, mx1 = -99999999.0f, mx2 = -99999999.0f;
    float mn0 = 99999999.0f, mn1 = 99999999.0f, mn2 = 99999999.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        mx0 = fmaxf(mx0, cb[k][0]);
        mx1 = fmaxf(mx1, cb[k][1]);
        mx2 = fmaxf(mx2, cb[k][2]);
        mn0 = fminf(mn0, cb[k][3]);
        mn1 = fminf(mn1, cb[k][4]);
        mn2 = fminf(mn2, cb[k][5]);
    }
    par[0] = mx0;
    par[1] = mx1;
    par[2] = mx2;
    par[3] = mn0;
    par[4] = mn1;
    par[5] = mn2;
    float P[3], e[3];
    uint32_t E[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        e[a] = pow2_ceil_log2((par[a] - par[3 + a]) * 0.003921569f);
        P[a] = par[3 + a];
        E[a] = __float_as_uint(e[a]) >> 23;
    }
    uint32_t words[6][2] = {};
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float tmx[3] = {cb[k][0], cb[k][1], cb[k][2]};
        float tmn[3] = {cb[k][3], cb[k][4], cb[k][5]};
        if (tmx[0] < -10000.0f)
            for (int a = 0; a < 3; a++) tmx[a] = tmn[a] = par[3 + a];
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const uint32_t hi = ftou_d3d(ceilf((tmx[a] - P[a]) / e[a]));
            const uint32_t lo = ftou_d3d(floorf((tmn[a] - P[a]) / e[a]));
            words[2 * a][k >> 2] |= lo << (8 * (k & 3));
            words[2 * a + 1][k >> 2] |= hi << (8 * (k & 3));
        }
    }
    const uint32_t imask = node->e_imask >> 24;
    node->p[0] = P[0];
    node->p[1] = P[1];
    node->p[2] = P[2];
    node->e_imask = E[0] | (E[1] << 8) | (E[2] << 16) | (imask << 24);
    uint32_t* dst[6] = {node->qlo_x, node->qhi_x, node->qlo_y, node->qhi_y, node->qlo_z, node->qhi_z};
#pragma unroll
    for (int w = 0; w < 6; w++) {
        dst[w][0] = words[w][0];
        dst[w][1] = words[w][1];
    }
}

struct RefitTreeArgs {
    const int32_t* starts;  // leaf NodePairs (rows without NodePair entries)
    uint32_t n_starts;
    const int32_t* fwd;     // ForwardStack rows, 8 per NodePair
    const int32_t* parent;  // parent NodePair
    const int32_t* node_of; // BVH node an internal NodePair documents (-1: leaf NodePair)
    uint32_t* arrive;       // arrival counters (0 between refits)
    float* bb;              // NodePair boxes, 32 B each (st_box / ld_box)
    uint32_t n_pairs;
    const float* boxes;     // primitive boxes (instances or triangles)
    const int32_t* box_idx; // TLASCWBVHIndices (TLAS) or nullptr (BLAS)
    tt_cwbvh_node* nodes;
};

__global__ void refit_tree(RefitTreeArgs t) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= t.n_starts) return;
    const __amdgpu_buffer_rsrc_t bb = __builtin_amdgcn_make_buffer_rsrc(t.bb, 0, (int)(t.n_pairs * 32u), 0x00020000);
    int32_t id = t.starts[s];
    float box[6];
    leaf_union(id, t.fwd, t.box_idx, t.boxes, box);
    while (id != 0) {  // the root pair completes the tree
        st_box(bb, id, box);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the box has left this CU before the arrival
        const int32_t p = t.parent[id];
        const uint32_t prev = __hip_atomic_fetch_add(t.arrive + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev != 7u) return;  // not the last of the parent's 8 slots
        // the other 7 boxes were stored sc1 by threads of other workgroups (often other CUs / XCDs):
        // one agent-scope acquire before reading them (MI355X_MICROARCH.md, inter-workgroup
        // visibility: with several workgroups per CU the sc1-loads-only hand-off is outside the
        // measured table, so the acquire stays), then wait for its invalidate to complete
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(t.arrive + p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        id = p;
        internal_pair(id, t.fwd, bb, t.nodes + t.node_of[id], box);
    }
}

// ------------------------------------------------------------------ Construct (BLAS refit)
// The reference leaves normalize / round / the mul association to DXC; pinned here and in the
// oracle: mul rows as fmaf(m2, z, fmaf(m1, y, m0 * x)) (+ m3), normalize(v) = v * (1 / sqrt(dot))
// with dot = fmaf(z, z, fmaf(y, y, x * x)), round = round-half-to-even, no other contraction.
__device__ __forceinline__ float3 ld_vec3(const BlasConstructArgs& a, int32_t idx, uint32_t off) {
    if (idx < 0 || (uint32_t)idx >= a.n_vertices) return make_float3(0.0f, 0.0f, 0.0f);  // D3D: OOB reads 0
    const float* v = a.vertices + (size_t)idx * a.vertex_stride + off;
    return make_float3(v[0], v[1], v[2]);
}
__device__ __forceinline__ float M(const float* m, int r, int c) { return m[c * 4 + r]; }
__device__ __forceinline__ float3 xform_point(const float* m, float3 p) {
    return make_float3(__builtin_fmaf(M(m, 0, 2), p.z, __builtin_fmaf(M(m, 0, 1), p.y, M(m, 0, 0) * p.x)) + M(m, 0, 3),
                       __builtin_fmaf(M(m, 1, 2), p.z, __builtin_fmaf(M(m, 1, 1), p.y, M(m, 1, 0) * p.x)) + M(m, 1, 3),
                       __builtin_fmaf(M(m, 2, 2), p.z, __builtin_fmaf(M(m, 2, 1), p.y, M(m, 2, 0) * p.x)) + M(m, 2, 3));
}
__device__ __forceinline__ float3 xform_normal(const float* m, float3 n) {
    const float3 v = make_float3(__builtin_fmaf(M(m, 0, 2), n.z, __builtin_fmaf(M(m, 0, 1), n.y, M(m, 0, 0) * n.x)),
                                 __builtin_fmaf(M(m, 1, 2), n.z, __builtin_fmaf(M(m, 1, 1), n.y, M(m, 1, 0) * n.x)),
                                 __builtin_fmaf(M(m, 2, 2), n.z, __builtin_fmaf(M(m, 2, 1), n.y, M(m, 2, 0) * n.x)));
    const float inv = 1.0f / sqrtf(__builtin_fmaf(v.z, v.z, __builtin_fmaf(v.y, v.y, v.x * v.x)));
    return make_float3(v.x * inv, v.y * inv, v.z * inv);
}
// octahedral_32 — BVHRefitter.compute:62-68
__device__ __forceinline__ uint32_t octahedral_32(float3 n) {
    const float s = (fabsf(n.x) + fabsf(n.y)) + fabsf(n.z);
    float x = n.x / s, y = n.y / s;
    if (!(n.z >= 0.0f)) {
        const float sx = (x >= 0.0f) ? 1.0f : -1.0f, sy = (y >= 0.0f) ? 1.0f : -1.0f;
        const float ox = x;
        x = (1.0f - fabsf(y)) * sx;
        y = (1.0f - fabsf(ox)) * sy;
    }
    const uint32_t dx = (uint32_t)rintf(32767.5f + x * 32767.5f), dy = (uint32_t)rintf(32767.5f + y * 32767.5f);
    return dx | (dy << 16);
}

__global__ void blas_construct(BlasConstructArgs a) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= a.n_tris) return;
    const int32_t i0 = a.indices[3 * t], i1 = a.indices[3 * t + 1], i2 = a.indices[3 * t + 2];
    // vidx = Load3(...).xzy: p from i0, p2 from i2, p3 from i1
    const float3 p = xform_point(a.m, ld_vec3(a, i0, 0)), p2 = xform_point(a.m, ld_vec3(a, i2, 0)),
                 p3 = xform_point(a.m, ld_vec3(a, i1, 0));
    const float3 n1 = xform_normal(a.m, ld_vec3(a, i0, 3)), n2 = xform_normal(a.m, ld_vec3(a, i2, 3)),
                 n3 = xform_normal(a.m, ld_vec3(a, i1, 3));
    const int32_t leaf = a.leaf_of[t];
    if (leaf < 0 || (uint32_t)leaf >= a.n_tris) return;  // D3D drops out-of-range writes
    float mx[3] = {fmaxf(fmaxf(p.x, p2.x), p3.x), fmaxf(fmaxf(p.y, p2.y), p3.y), fmaxf(fmaxf(p.z, p2.z), p3.z)};
    float mn[3] = {fminf(fminf(p.x, p2.x), p3.x), fminf(fminf(p.y, p2.y), p3.y), fminf(fminf(p.z, p2.z), p3.z)};
    for (int k = 0; k < 3; k++)
        if (mx[k] - mn[k] < 0.000001f) {
            mn[k] -= 0.000001f;
            mx[k] += 0.000001f;
        }
    float* b = a.boxes + 6 * (size_t)leaf;
    b[0] = mx[0];
    b[1] = mx[1];
    b[2] = mx[2];
    b[3] = mn[0];
    b[4] = mn[1];
    b[5] = mn[2];
    const float3 e1 = make_float3(p2.x - p.x, p2.y - p.y, p2.z - p.z), e2 = make_float3(p3.x - p.x, p3.y - p.y, p3.z - p.z);
    tt_cuda_triangle& T = a.tris88[leaf];
    T.pos0[0] = p.x;
    T.pos0[1] = p.y;
    T.pos0[2] = p.z;
    T.posedge1[0] = e1.x;
    T.posedge1[1] = e1.y;
    T.posedge1[2] = e1.z;
    T.posedge2[0] = e2.x;
    T.posedge2[1] = e2.y;
    T.posedge2[2] = e2.z;
    T.norms[0] = octahedral_32(n1);
    T.norms[1] = octahedral_32(n2);
    T.norms[2] = octahedral_32(n3);
    TriPos& q = a.tripos[leaf];
    q.p0x = p.x;
    q.p0y = p.y;
    q.p0z = p.z;
    q.e1x = e1.x;
    q.e1y = e1.y;
    q.e1z = e1.z;
    q.e2x = e2.x;
    q.e2y = e2.y;
    q.e2z = e2.z;
}

inline uint32_t grid_of(uint32_t n) { return (n + kBlock - 1) / kBlock; }

}  // namespace

// ------------------------------------------------------------------ host-side structure build
// DocumentNodes (AssetManager.cs:1257-1297) and the ForwardStack / LayerStack construction
// (:1364-1390), from the TLAS region of the uploaded nodes. Returned as flat arrays.
static void document_nodes(const tt_cwbvh_node* nodes, RefitPlan& R, int current, int parent, int next_bvh8,
                           bool is_leaf, int recur) {
    R.depth[current] = recur;
    R.parent[current] = parent;
    if (!is_leaf) {
        R.to_bvh[next_bvh8] = current;
        R.leaf[current] = 0;
        const tt_cwbvh_node& node = nodes[next_bvh8];
        for (int i = 0; i < 8; i++) {
            R.pair_bvh.push_back(next_bvh8);
            R.pair_slot.push_back(i);
            R.leaf.push_back(0);
            R.depth.push_back(0);
            R.parent.push_back(0);
            const int me = (int)R.pair_bvh.size() - 1;
            const uint32_t m = (node.meta[i >> 2] >> (8 * (i & 3))) & 0xffu;
            if ((m & 0x1fu) < 24u) {
                document_nodes(nodes, R, me, current, -1, true, recur + 1);
            } else {
                const int child = (int)node.base_child + (int)(m & 31u) - 24;
                if (child < 0 || (uint32_t)child >= R.n_tlas || recur > 256) {
                    R.ok = false;
                    return;
                }
                document_nodes(nodes, R, me, current, child, false, recur + 1);
            }
        }
    } else {
        R.leaf[current] = 1;
    }
}

bool tt_refit_build_plan(const tt_cwbvh_node* nodes, uint32_t n_tlas_nodes, RefitPlan& R) {
    R = RefitPlan();
    R.n_tlas = n_tlas_nodes;
    R.to_bvh.assign(n_tlas_nodes, 0);
    R.pair_bvh.push_back(0);
    R.pair_slot.push_back(0);
    R.leaf.push_back(0);
    R.depth.push_back(0);
    R.parent.push_back(0);
    document_nodes(nodes, R, 0, 0, 0, false, 0);
    if (!R.ok) return false;
    const size_t N = R.pair_bvh.size();
    R.fwd.assign(N * 8, 0);
    int max_depth = 0;
    for (size_t i = 0; i < N; i++) {
        const tt_cwbvh_node& node = nodes[R.pair_bvh[i]];
        const int slot = R.pair_slot[i];
        if (R.leaf[i]) {
            const uint32_t m = (node.meta[slot >> 2] >> (8 * (slot & 3))) & 0xffu;
            const int nb = __builtin_popcount(m >> 5), first = (int)node.base_tri + (int)(m & 0x1fu);
            R.fwd[i * 8 + slot] = nb + first * 24 + 1;
            if (nb) R.leaf_end = std::max(R.leaf_end, first + nb);
        } else {
            R.fwd[i * 8 + slot] = -(int)i - 1;
        }
        R.fwd[(size_t)R.parent[i] * 8 + slot] = -(int)i - 1;
        max_depth = std::max(max_depth, R.depth[i]);
    }
    R.layers.assign((size_t)max_depth + 1, {});
    for (size_t i = 0; i < N; i++) R.layers[R.depth[i]].push_back((int32_t)i);
    return true;
}

void tt_refit_free(RefitDev& d) {
    for (void* p : {(void*)d.starts, (void*)d.fwd, (void*)d.parent, (void*)d.node_of, (void*)d.arrive, (void*)d.bb})
        if (p) (void)hipFree(p);
    d = RefitDev();
}

template <class T>
static hipError_t up(T** dst, const std::vector<T>& v) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), std::max<size_t>(1, v.size()) * sizeof(T));
    if (e != hipSuccess) return e;
    return v.empty() ? hipSuccess : hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

hipError_t tt_refit_prepare(const RefitPlan& R, const tt_cwbvh_node* host_nodes, uint32_t n_tlas_nodes, RefitDev& d) {
    (void)host_nodes;
    tt_refit_free(d);
    const size_t N = R.pair_bvh.size();
    d.n_pairs = (uint32_t)N;
    d.n_nodes = n_tlas_nodes;
    std::vector<int32_t> starts, node_of(N, -1);
    for (size_t i = 0; i < N; i++)
        if (R.leaf[i]) starts.push_back((int32_t)i);
    for (uint32_t n = 0; n < n_tlas_nodes; n++)
        if (n == 0 || R.to_bvh[n] != 0) node_of[(size_t)R.to_bvh[n]] = (int32_t)n;
    d.n_starts = (uint32_t)starts.size();
    hipError_t e;
    if ((e = up(&d.starts, starts)) != hipSuccess || (e = up(&d.fwd, R.fwd)) != hipSuccess ||
        (e = up(&d.parent, R.parent)) != hipSuccess || (e = up(&d.node_of, node_of)) != hipSuccess)
        return e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&d.arrive), sizeof(uint32_t) * N)) != hipSuccess) return e;
    if ((e = hipMemset(d.arrive, 0, sizeof(uint32_t) * N)) != hipSuccess) return e;
    return hipMalloc(reinterpret_cast<void**>(&d.bb), 8 * sizeof(float) * N);
}

// One frame: primitive boxes (device) -> the nodes of `nodes` the plan covers. One launch.
hipError_t tt_refit_run(RefitDev& d, const float* boxes, const int32_t* box_index, tt_cwbvh_node* nodes, hipStream_t st) {
    if (!d.n_starts) return hipSuccess;
    RefitTreeArgs t{d.starts, d.n_starts, d.fwd, d.parent, d.node_of, d.arrive, d.bb, d.n_pairs, boxes, box_index, nodes};
    hipLaunchKernelGGL(refit_tree, dim3(grid_of(d.n_starts)), dim3(kBlock), 0, st, t);
    return hipGetLastError();
}

hipError_t tt_blas_construct(const BlasConstructArgs& a, hipStream_t st) {
    if (!a.n_tris) return hipSuccess;
    hipLaunchKernelGGL(blas_construct, dim3(grid_of(a.n_tris)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}
