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
// MI355X shape: the refit is a few thousand tiny records per frame, latency- not bandwidth-bound;
// it runs as one short launch per BVH depth level on the context stream (no host sync), so a
// trace enqueued after it on the same stream sees the new TLAS nodes.
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

__global__ void refit_init(float* __restrict__ bb, uint32_t n) {  // NodeInitializer
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    for (int a = 0; a < 3; a++) {
        bb[6 * i + a] = -9999999999.0f;     // BBMax
        bb[6 * i + 3 + a] = 9999999999.0f;  // BBMin
    }
}

// RefitBVHLayer (TLAS: leaf ranges index the boxes through TLASCWBVHIndices) / RefitLayer (BLAS:
// leaf ranges are triangle boxes in leaf order, box_idx == nullptr): one NodePair per thread
__global__ void refit_layer(const int32_t* __restrict__ layer, uint32_t n, const int32_t* __restrict__ fwd,
                            const int32_t* __restrict__ box_idx, const float* __restrict__ boxes,
                            float* __restrict__ bb) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= n) return;
    const int32_t id = layer[t];
    float mx0 = -99999999.0f, mx1 = -99999999.0f, mx2 = -99999999.0f;
    float mn0 = 99999999.0f, mn1 = 99999999.0f, mn2 = 99999999.0f;
    for (int k = 0; k < 8; k++) {
        const int32_t leaf = fwd[8 * id + k];
        if (leaf == 0) continue;
        if (leaf < 0) {
            const float* c = bb + 6 * (size_t)(-leaf - 1);
            mx0 = fmaxf(mx0, c[0]);
            mx1 = fmaxf(mx1, c[1]);
            mx2 = fmaxf(mx2, c[2]);
            mn0 = fminf(mn0, c[3]);
            mn1 = fminf(mn1, c[4]);
            mn2 = fminf(mn2, c[5]);
        } else {
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
    }
    float* o = bb + 6 * (size_t)id;
    o[0] = mx0;
    o[1] = mx1;
    o[2] = mx2;
    o[3] = mn0;
    o[4] = mn1;
    o[5] = mn2;
}

// NodeUpdate: NodePair id (>= 1) re-quantizes its slot of its BVH8 node against the node's bounds
__global__ void refit_update(uint32_t n_pairs, const int32_t* __restrict__ pair_bvh, const int32_t* __restrict__ pair_slot,
                             const int32_t* __restrict__ to_bvh, const float* __restrict__ bb, float* __restrict__ P,
                             uint32_t* __restrict__ E, uint32_t* __restrict__ Q) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n_pairs || i == 0) return;
    const int32_t node = pair_bvh[i], slot = pair_slot[i];
    const float* par = bb + 6 * (size_t)to_bvh[node];
    const float* me = bb + 6 * (size_t)i;
    float tmx[3] = {me[0], me[1], me[2]}, tmn[3] = {me[3], me[4], me[5]};
    if (tmx[0] < -10000.0f)
        for (int a = 0; a < 3; a++) tmx[a] = tmn[a] = par[3 + a];
    for (int a = 0; a < 3; a++) {
        const float e = pow2_ceil_log2((par[a] - par[3 + a]) * 0.003921569f);
        const float p = par[3 + a];
        P[3 * node + a] = p;
        E[3 * node + a] = __float_as_uint(e) >> 23;
        Q[48 * node + 8 * (2 * a + 1) + slot] = ftou_d3d(ceilf((tmx[a] - p) / e));
        Q[48 * node + 8 * (2 * a) + slot] = ftou_d3d(floorf((tmn[a] - p) / e));
    }
}

// NodeCompress: pack the fixed layout into 80-B nodes (full uints shifted and OR-ed, as the reference)
__global__ void refit_compress(uint32_t n_nodes, const float* __restrict__ P, const uint32_t* __restrict__ E,
                               const uint32_t* __restrict__ Q, tt_cwbvh_node* __restrict__ nodes) {
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= n_nodes) return;
    tt_cwbvh_node& o = nodes[n];
    const uint32_t imask = o.e_imask >> 24;
    o.p[0] = P[3 * n];
    o.p[1] = P[3 * n + 1];
    o.p[2] = P[3 * n + 2];
    o.e_imask = E[3 * n] | (E[3 * n + 1] << 8) | (E[3 * n + 2] << 16) | (imask << 24);
    uint32_t* words[6] = {o.qlo_x, o.qhi_x, o.qlo_y, o.qhi_y, o.qlo_z, o.qhi_z};
    for (int w = 0; w < 6; w++)
        for (int h = 0; h < 2; h++) {
            const uint32_t* q = Q + 48 * n + 8 * w + 4 * h;
            words[w][h] = q[0] | (q[1] << 8) | (q[2] << 16) | (q[3] << 24);
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
    for (void* p : {(void*)d.pair_bvh, (void*)d.pair_slot, (void*)d.to_bvh, (void*)d.fwd, (void*)d.layers, (void*)d.bb,
                    (void*)d.P, (void*)d.boxes, (void*)d.E, (void*)d.Q})
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
    tt_refit_free(d);
    d.n_pairs = (uint32_t)R.pair_bvh.size();
    d.n_nodes = n_tlas_nodes;
    std::vector<int32_t> flat;
    for (const auto& l : R.layers) {
        d.layer_off.push_back((uint32_t)flat.size());
        d.layer_n.push_back((uint32_t)l.size());
        flat.insert(flat.end(), l.begin(), l.end());
    }
    // fixed-layout node state, seeded from the current node bytes (NodeUpdate rewrites all of it)
    std::vector<float> P(3 * (size_t)n_tlas_nodes);
    std::vector<uint32_t> E(3 * (size_t)n_tlas_nodes), Q(48 * (size_t)n_tlas_nodes);
    for (uint32_t n = 0; n < n_tlas_nodes; n++) {
        const tt_cwbvh_node& s = host_nodes[n];
        for (int a = 0; a < 3; a++) {
            P[3 * n + a] = s.p[a];
            E[3 * n + a] = (s.e_imask >> (8 * a)) & 0xffu;
        }
        const uint32_t* words[6] = {s.qlo_x, s.qhi_x, s.qlo_y, s.qhi_y, s.qlo_z, s.qhi_z};
        for (int w = 0; w < 6; w++)
            for (int k = 0; k < 8; k++) Q[48 * n + 8 * w + k] = (words[w][k >> 2] >> (8 * (k & 3))) & 0xffu;
    }
    hipError_t e;
    if ((e = up(&d.pair_bvh, R.pair_bvh)) != hipSuccess || (e = up(&d.pair_slot, R.pair_slot)) != hipSuccess ||
        (e = up(&d.to_bvh, R.to_bvh)) != hipSuccess || (e = up(&d.fwd, R.fwd)) != hipSuccess ||
        (e = up(&d.layers, flat)) != hipSuccess || (e = up(&d.P, P)) != hipSuccess || (e = up(&d.E, E)) != hipSuccess ||
        (e = up(&d.Q, Q)) != hipSuccess)
        return e;
    return hipMalloc(reinterpret_cast<void**>(&d.bb), 6 * sizeof(float) * d.n_pairs);
}

// One frame: boxes (device, n_mesh x 6 floats) -> TLAS nodes [0, n_nodes) of `nodes`.
hipError_t tt_refit_run(RefitDev& d, const float* boxes, const int32_t* box_index, tt_cwbvh_node* nodes, hipStream_t st) {
    hipLaunchKernelGGL(refit_init, dim3(grid_of(d.n_pairs)), dim3(kBlock), 0, st, d.bb, d.n_pairs);
    for (int l = (int)d.layer_n.size() - 1; l >= 0; l--) {
        if (!d.layer_n[l]) continue;
        hipLaunchKernelGGL(refit_layer, dim3(grid_of(d.layer_n[l])), dim3(kBlock), 0, st, d.layers + d.layer_off[l],
                           d.layer_n[l], d.fwd, box_index, boxes, d.bb);
    }
    hipLaunchKernelGGL(refit_update, dim3(grid_of(d.n_pairs)), dim3(kBlock), 0, st, d.n_pairs, d.pair_bvh, d.pair_slot,
                       d.to_bvh, d.bb, d.P, d.E, d.Q);
    hipLaunchKernelGGL(refit_compress, dim3(grid_of(d.n_nodes)), dim3(kBlock), 0, st, d.n_nodes, d.P, d.E, d.Q, nodes);
    return hipGetLastError();
}

hipError_t tt_blas_construct(const BlasConstructArgs& a, hipStream_t st) {
    if (!a.n_tris) return hipSuccess;
    hipLaunchKernelGGL(blas_construct, dim3(grid_of(a.n_tris)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}
