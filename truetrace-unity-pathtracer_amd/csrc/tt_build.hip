// tt_build.hip — the BLAS builder's BVH2 stage on the GPU (builder half):
// BVH2Builder (BVH2Builder.cs:9-217) restated level by level, producing the SAME nodes and the
// same FinalIndices as the sequential C# recursion (and as host/tt_scene.cpp's restatement).
//
// The reference builds depth first: per node, a full SAH sweep over the node's primitives in each
// axis' presorted order (left-to-right running unions -> sah[i] = SA(left) * i, then right-to-left
// unions -> cost = sah[i] + SA(right) * (count - i), `cost <= best` so ties go to the lowest i and,
// across axes x, y, z, to the later axis), then a stable partition of the other two axes' index
// lists. Nothing in a node depends on its siblings, and a subtree of k primitives takes 2(k - 1)
// node slots of the depth-first numbering, so every node's slot is known when its parent splits.
// Here all nodes of one depth are split at once:
//  * the running unions are segmented scans (rocPRIM scan-by-key, one segment per node) whose
//    operator is AABB.Extend itself -- `if (b.min < a.min) a.min = b.min` keeps the EARLIER value
//    on ties (signed zeros included), which is associative, so the scan reproduces the sequential
//    unions bit for bit; NaN components never win an Extend, so they enter as the identity;
//  * the SAH cost is evaluated per position with the reference's expression (no contraction), and
//    the per-node argmin packs (order-preserving cost bits, position) into one 64-bit atomic min;
//  * the partition is a segmented exclusive count of left-going primitives (stable by construction).
// The three per-axis presorts (.NET's unstable introsort, whose tie order decides trees) stay on
// the host (tt_dotnet_sort_by_key); this file takes their output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "../../include/truetrace_hip.h"

extern "C" hipStream_t tt_ctx_stream_of(tt_ctx* c);  // tt_api.hip (C linkage there)

namespace {

struct Box {
    float mx[3];  // BBMax (C# field order: BBMax then BBMin)
    float mn[3];  // BBMin
};

__host__ __device__ inline Box box_init() {
    Box b;
    for (int i = 0; i < 3; i++) {
        b.mx[i] = -FLT_MAX;  // float.MinValue
        b.mn[i] = FLT_MAX;
    }
    return b;
}

// CommonVars.AABB.Extend(AABB) (CommonVars.cs:304-402): `a` is the union so far, `b` the next box.
struct ExtendOp {
    __device__ Box operator()(const Box& a, const Box& b) const {
        Box r;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            r.mn[i] = b.mn[i] < a.mn[i] ? b.mn[i] : a.mn[i];
            r.mx[i] = b.mx[i] > a.mx[i] ? b.mx[i] : a.mx[i];
        }
        return r;
    }
};

// surface_area (BVH2Builder.cs): s = BBMax - BBMin; 2 * (s.x*s.y + s.x*s.z + s.y*s.z)
__device__ inline float surface_area(const Box& a) {
    const float sx = a.mx[0] - a.mn[0], sy = a.mx[1] - a.mn[1], sz = a.mx[2] - a.mn[2];
    return 2.0f * ((sx * sy) + (sx * sz) + (sy * sz));
}

// A primitive box as Extend sees it: a NaN component never replaces the running value, i.e. it acts
// like the identity's component.
__device__ inline Box prim_box(const Box& p) {
    Box b;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        b.mx[i] = p.mx[i] == p.mx[i] ? p.mx[i] : -FLT_MAX;
        b.mn[i] = p.mn[i] == p.mn[i] ? p.mn[i] : FLT_MAX;
    }
    return b;
}

struct Seg {
    int nodesi;      // BVH2Nodes slot of this node
    int node_index;  // first slot of its children's subtree (BuildRecursive's node_index)
    int first, count;
};

// position p -> the box of the primitive at p in axis order `idx` (identity outside live segments)
struct FwdBox {
    const int* idx;
    const Box* prims;
    const int* seg;
    __device__ Box operator()(int p) const { return seg[p] < 0 ? box_init() : prim_box(prims[idx[p]]); }
};
struct RevBox {
    const int* idx;
    const Box* prims;
    const int* seg;
    int n;
    __device__ Box operator()(int q) const {
        const int p = n - 1 - q;
        return seg[p] < 0 ? box_init() : prim_box(prims[idx[p]]);
    }
};
struct RevKey {
    const int* seg;
    int n;
    __device__ int operator()(int q) const { return seg[n - 1 - q]; }
};
// left-going flag of position p in axis d for segments that split on another axis (else 0)
struct LeftFlag {
    const int* idx;
    const int* seg;
    const int* dim;
    const unsigned char* going_left;
    int d;
    __device__ int operator()(int p) const {
        const int s = seg[p];
        return (s >= 0 && dim[s] != d) ? (int)going_left[idx[p]] : 0;
    }
};

__device__ inline uint32_t ordered_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float from_ordered(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

constexpr int kBlock = 256;

// SAH cost of every split position of every live segment for one axis; per-segment argmin (lowest
// cost, then lowest relative index) by a 64-bit atomic min. pre[p] = union of the segment's
// positions [first, p]; sufr[n - 1 - p] = union of [p, end] (the reverse scan's output order).
__global__ void k_cost(int n, const int* __restrict__ seg, const Seg* __restrict__ segs, const Box* __restrict__ pre,
                       const Box* __restrict__ sufr, unsigned long long* __restrict__ best) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    int s = -1;
    unsigned long long key = ~0ull;
    if (p < n) {
        s = seg[p];
        if (s >= 0) {
            const Seg g = segs[s];
            const int rel = p - g.first;
            if (rel >= 1) {
                float cost = surface_area(pre[p - 1]) * (float)rel + surface_area(sufr[n - 1 - p]) * (float)(g.count - rel);
                if (cost <= FLT_MAX) {  // `cost <= split.cost` from float.MaxValue: +inf / NaN never split
                    if (cost == 0.0f) cost = 0.0f;  // -0 == +0 for the reference's compare
                    key = ((unsigned long long)ordered_bits(cost) << 32) | (uint32_t)rel;
                }
            }
        }
    }
    // one atomic per wave when the wave is inside one segment (the common case near the root)
    const int s0 = __builtin_amdgcn_readfirstlane(s);
    if (__ballot(s != s0) == 0ull) {
        if (s0 < 0) return;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(key, off, 64);
            key = o < key ? o : key;
        }
        if ((threadIdx.x & 63) == 0 && key != ~0ull) atomicMin(best + s0, key);
    } else if (s >= 0 && key != ~0ull) {
        atomicMin(best + s, key);
    }
}

// the best split of axis d of every segment: its cost, position and both unions
__global__ void k_candidate(int S, int n, const Seg* __restrict__ segs, const unsigned long long* __restrict__ best,
                            const Box* __restrict__ pre, const Box* __restrict__ sufr, float* __restrict__ c_cost,
                            int* __restrict__ c_pos, Box* __restrict__ c_left, Box* __restrict__ c_right) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const unsigned long long k = best[s];
    if (k == ~0ull) {
        c_pos[s] = -1;
        return;
    }
    const int p = segs[s].first + (int)(uint32_t)k;
    c_cost[s] = from_ordered((uint32_t)(k >> 32));
    c_pos[s] = p;
    c_left[s] = pre[p - 1];
    c_right[s] = sufr[n - 1 - p];
}

struct SplitOut {
    int split;  // first position of the right child, -1: no valid split (error)
    int dim;
    int n_next; // live children (count >= 2)
};

// partition_sah's axis choice (x, y, z in turn, `cost <= best`) and BuildRecursive's node writes:
// the node's child slots and boxes, leaf children (count 1) written at once.
__global__ void k_split(int S, const Seg* __restrict__ segs, const float* __restrict__ c_cost, const int* __restrict__ c_pos,
                        const Box* __restrict__ c_left, const Box* __restrict__ c_right, SplitOut* __restrict__ out,
                        Box* __restrict__ node_box, int* __restrict__ node_left, uint32_t* __restrict__ node_count,
                        int* __restrict__ err) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    float cost = FLT_MAX;
    int split = -1, dim = -1;
    Box L = box_init(), R = box_init();
    for (int d = 0; d < 3; d++) {
        const int pos = c_pos[d * S + s];
        if (pos >= 0 && c_cost[d * S + s] <= cost) {
            cost = c_cost[d * S + s];
            split = pos;
            dim = d;
            L = c_left[d * S + s];
            R = c_right[d * S + s];
        }
    }
    SplitOut o{split, dim, 0};
    if (split < 0) {
        atomicOr(err, 1);
        out[s] = o;
        return;
    }
    const Seg g = segs[s];
    node_left[g.nodesi] = g.node_index;
    node_box[g.node_index] = L;
    node_box[g.node_index + 1] = R;
    const int n_left = split - g.first, n_right = g.first + g.count - split;
    if (n_left == 1) {
        node_left[g.node_index] = g.first;
        node_count[g.node_index] = 1u;
    }
    if (n_right == 1) {
        node_left[g.node_index + 1] = split;
        node_count[g.node_index + 1] = 1u;
    }
    o.n_next = (n_left >= 2 ? 1 : 0) + (n_right >= 2 ? 1 : 0);
    out[s] = o;
}

// next level's segments (children with >= 2 primitives, in parent order: left then right)
__global__ void k_children(int S, const Seg* __restrict__ segs, const SplitOut* __restrict__ so,
                           const int* __restrict__ base, Seg* __restrict__ next, int2* __restrict__ child_id) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const Seg g = segs[s];
    const SplitOut o = so[s];
    int b = base[s];
    const int n_left = o.split - g.first, n_right = g.first + g.count - o.split;
    int2 id = make_int2(-1, -1);
    if (n_left >= 2) {
        next[b] = Seg{g.node_index, g.node_index + 2, g.first, n_left};
        id.x = b++;
    }
    if (n_right >= 2) {
        next[b] = Seg{g.node_index + 1, g.node_index + 2 + 2 * (n_left - 1), o.split, n_right};
        id.y = b;
    }
    child_id[s] = id;
}

// indices_going_left[prim] = position < split, from the split axis' order
__global__ void k_flags(int n, const int* __restrict__ i0, const int* __restrict__ i1, const int* __restrict__ i2,
                        const int* __restrict__ seg, const SplitOut* __restrict__ so, unsigned char* __restrict__ going_left) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    if (s < 0) return;
    const SplitOut o = so[s];
    const int* idx = o.dim == 0 ? i0 : (o.dim == 1 ? i1 : i2);
    going_left[idx[p]] = p < o.split ? 1 : 0;
}

// stable partition of axis d inside every segment that split on another axis
__global__ void k_scatter(int n, int d, const int* __restrict__ idx, const int* __restrict__ seg,
                          const Seg* __restrict__ segs, const SplitOut* __restrict__ so,
                          const unsigned char* __restrict__ going_left, const int* __restrict__ lrank,
                          int* __restrict__ out) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    const int v = idx[p];
    if (s < 0 || so[s].dim == d) {
        out[p] = v;
        return;
    }
    const int first = segs[s].first, split = so[s].split;
    const int r = lrank[p];
    out[going_left[v] ? first + r : split + (p - first - r)] = v;
}

__global__ void k_reseg(int n, int* __restrict__ seg, const SplitOut* __restrict__ so, const int2* __restrict__ child_id) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int s = seg[p];
    if (s < 0) return;
    const int2 id = child_id[s];
    seg[p] = p < so[s].split ? id.x : id.y;
}

__global__ void k_dim_of(int S, const SplitOut* __restrict__ so, int* __restrict__ dim) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s < S) dim[s] = so[s].dim;
}

template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t k) {
        n = k;
        return hipMalloc(&p, std::max<size_t>(k, 1) * sizeof(T));
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};

inline unsigned grid_of(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

// exclusive-scan input: live children per segment (0 past the last segment, so base[S] = total)
struct NextCount {
    const SplitOut* so;
    int S;
    __device__ int operator()(int q) const { return q < S ? so[q].n_next : 0; }
};

#define TT_BH(x)                                  \
    do {                                          \
        const hipError_t e_ = (x);                \
        if (e_ != hipSuccess) return TT_ERR_HIP;  \
    } while (0)

extern "C" tt_status tt_bvh2_build_device(tt_ctx* ctx, const float* aabbs, uint32_t n_u, const int32_t* presorted,
                                          int32_t* final_indices, float* node_aabbs, int32_t* node_left,
                                          uint32_t* node_count, uint32_t* max_depth) {
    if (!ctx || !aabbs || !n_u || !presorted || !final_indices || n_u >= (1u << 30)) return TT_ERR_INVALID_ARG;
    const int n = (int)n_u;
    hipStream_t st = tt_ctx_stream_of(ctx);
    for (size_t i = 0; i < 3 * (size_t)n; i++)
        if (presorted[i] < 0 || presorted[i] >= n) return TT_ERR_INVALID_ARG;

    // root box: Extend over the primitives in index order (BVH2Builder.cs: BVH2Nodes[0].aabb)
    Box root = box_init();
    for (int i = 0; i < n; i++) {
        const float* b = aabbs + 6 * (size_t)i;
        for (int k = 0; k < 3; k++) {
            if (b[3 + k] < root.mn[k]) root.mn[k] = b[3 + k];
            if (b[k] > root.mx[k]) root.mx[k] = b[k];
        }
    }
    const size_t n2 = 2 * (size_t)n;
    uint32_t depth = 0;
    if (n == 1) {
        if (node_aabbs) {
            std::memset(node_aabbs, 0, n2 * sizeof(Box));
            std::memcpy(node_aabbs, &root, sizeof(Box));
        }
        if (node_left) std::memset(node_left, 0, n2 * sizeof(int32_t));
        if (node_count) {
            std::memset(node_count, 0, n2 * sizeof(uint32_t));
            node_count[0] = 1u;
        }
        final_indices[0] = presorted[0];
        if (max_depth) *max_depth = 0;
        return TT_OK;
    }
    DBuf<Box> prims, pre, sufr, box, c_left, c_right;
    DBuf<int> idxb[4], seg, lrank, nleft, c_pos, dimv, base, err;
    DBuf<uint32_t> ncount;
    DBuf<unsigned char> going_left;
    DBuf<Seg> segs, next;
    DBuf<SplitOut> so;
    DBuf<unsigned long long> best;
    DBuf<float> c_cost;
    DBuf<int2> child_id;
    const size_t smax = (size_t)n / 2 + 1;  // live segments per level (>= 2 primitives each)
    TT_BH(prims.alloc(n));
    TT_BH(pre.alloc(n));
    TT_BH(sufr.alloc(n));
    TT_BH(box.alloc(n2));
    TT_BH(nleft.alloc(n2));
    TT_BH(ncount.alloc(n2));
    for (auto& b : idxb) TT_BH(b.alloc(n));
    TT_BH(seg.alloc(n));
    TT_BH(lrank.alloc(n));
    TT_BH(going_left.alloc(n));
    TT_BH(segs.alloc(smax));
    TT_BH(next.alloc(smax));
    TT_BH(so.alloc(smax));
    TT_BH(best.alloc(3 * smax));
    TT_BH(c_cost.alloc(3 * smax));
    TT_BH(c_pos.alloc(3 * smax));
    TT_BH(c_left.alloc(3 * smax));
    TT_BH(c_right.alloc(3 * smax));
    TT_BH(dimv.alloc(smax));
    TT_BH(base.alloc(smax + 1));
    TT_BH(child_id.alloc(smax));
    TT_BH(err.alloc(1));
    int* idx[3] = {idxb[0].p, idxb[1].p, idxb[2].p};
    int* tmp = idxb[3].p;
    static_assert(sizeof(Box) == 24, "Box is BBMax xyz, BBMin xyz");
    TT_BH(hipMemcpyAsync(prims.p, aabbs, (size_t)n * sizeof(Box), hipMemcpyHostToDevice, st));
    for (int d = 0; d < 3; d++)
        TT_BH(hipMemcpyAsync(idx[d], presorted + (size_t)d * n, (size_t)n * sizeof(int), hipMemcpyHostToDevice, st));
    TT_BH(hipMemsetAsync(box.p, 0, n2 * sizeof(Box), st));  // NativeArrayOptions.ClearMemory
    TT_BH(hipMemcpyAsync(box.p, &root, sizeof(Box), hipMemcpyHostToDevice, st));
    TT_BH(hipMemsetAsync(nleft.p, 0, n2 * sizeof(int), st));
    TT_BH(hipMemsetAsync(ncount.p, 0, n2 * sizeof(uint32_t), st));
    TT_BH(hipMemsetAsync(seg.p, 0, (size_t)n * sizeof(int), st));  // every position in segment 0 (the root)
    TT_BH(hipMemsetAsync(err.p, 0, sizeof(int), st));
    const Seg root_seg{0, 2, 0, n};
    TT_BH(hipMemcpyAsync(segs.p, &root_seg, sizeof(Seg), hipMemcpyHostToDevice, st));

    // rocPRIM temporary storage: the largest of the scans used per level (sizes depend on n only)
    auto cnt = rocprim::make_counting_iterator<int>(0);
    size_t tb = 0;
    {
        size_t t1 = 0;
        auto fwd = rocprim::make_transform_iterator(cnt, FwdBox{idx[0], prims.p, seg.p});
        TT_BH(rocprim::inclusive_scan_by_key(nullptr, t1, seg.p, fwd, pre.p, (size_t)n, ExtendOp(),
                                             rocprim::equal_to<int>(), st));
        tb = std::max(tb, t1);
        auto rk = rocprim::make_transform_iterator(cnt, RevKey{seg.p, n});
        auto rb = rocprim::make_transform_iterator(cnt, RevBox{idx[0], prims.p, seg.p, n});
        TT_BH(rocprim::inclusive_scan_by_key(nullptr, t1, rk, rb, sufr.p, (size_t)n, ExtendOp(),
                                             rocprim::equal_to<int>(), st));
        tb = std::max(tb, t1);
        auto fl = rocprim::make_transform_iterator(cnt, LeftFlag{idx[0], seg.p, dimv.p, going_left.p, 0});
        TT_BH(rocprim::exclusive_scan_by_key(nullptr, t1, seg.p, fl, lrank.p, 0, (size_t)n, rocprim::plus<int>(),
                                             rocprim::equal_to<int>(), st));
        tb = std::max(tb, t1);
        auto nc = rocprim::make_transform_iterator(cnt, NextCount{so.p, 1});
        TT_BH(rocprim::exclusive_scan(nullptr, t1, nc, base.p, 0, smax + 1, rocprim::plus<int>(), st));
        tb = std::max(tb, t1);
    }
    DBuf<unsigned char> tstore;
    TT_BH(tstore.alloc(tb));

    int S = 1;
    while (S > 0) {
        depth++;  // the children created at this level sit one deeper (BuildRecursive's depth + 1)
        TT_BH(hipMemsetAsync(best.p, 0xff, 3 * (size_t)S * sizeof(unsigned long long), st));
        for (int d = 0; d < 3; d++) {
            size_t t = tb;
            auto fwd = rocprim::make_transform_iterator(cnt, FwdBox{idx[d], prims.p, seg.p});
            TT_BH(rocprim::inclusive_scan_by_key(tstore.p, t, seg.p, fwd, pre.p, (size_t)n, ExtendOp(),
                                                 rocprim::equal_to<int>(), st));
            t = tb;
            auto rk = rocprim::make_transform_iterator(cnt, RevKey{seg.p, n});
            auto rb = rocprim::make_transform_iterator(cnt, RevBox{idx[d], prims.p, seg.p, n});
            TT_BH(rocprim::inclusive_scan_by_key(tstore.p, t, rk, rb, sufr.p, (size_t)n, ExtendOp(),
                                                 rocprim::equal_to<int>(), st));
            hipLaunchKernelGGL(k_cost, dim3(grid_of(n)), dim3(kBlock), 0, st, n, seg.p, segs.p, pre.p, sufr.p,
                               best.p + (size_t)d * S);
            hipLaunchKernelGGL(k_candidate, dim3(grid_of(S)), dim3(kBlock), 0, st, S, n, segs.p, best.p + (size_t)d * S,
                               pre.p, sufr.p, c_cost.p + (size_t)d * S, c_pos.p + (size_t)d * S,
                               c_left.p + (size_t)d * S, c_right.p + (size_t)d * S);
        }
        hipLaunchKernelGGL(k_split, dim3(grid_of(S)), dim3(kBlock), 0, st, S, segs.p, c_cost.p, c_pos.p, c_left.p,
                           c_right.p, so.p, box.p, nleft.p, ncount.p, err.p);
        size_t t = tb;
        auto nc = rocprim::make_transform_iterator(cnt, NextCount{so.p, S});
        TT_BH(rocprim::exclusive_scan(tstore.p, t, nc, base.p, 0, (size_t)S + 1, rocprim::plus<int>(), st));
        int h[2] = {0, 0};
        TT_BH(hipMemcpyAsync(&h[0], base.p + S, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipMemcpyAsync(&h[1], err.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipStreamSynchronize(st));
        if (h[1]) return TT_ERR_UNSUPPORTED;  // a node without a finite SAH split (the C# recursion misbehaves there too)
        hipLaunchKernelGGL(k_children, dim3(grid_of(S)), dim3(kBlock), 0, st, S, segs.p, so.p, base.p, next.p,
                           child_id.p);
        hipLaunchKernelGGL(k_dim_of, dim3(grid_of(S)), dim3(kBlock), 0, st, S, so.p, dimv.p);
        hipLaunchKernelGGL(k_flags, dim3(grid_of(n)), dim3(kBlock), 0, st, n, idx[0], idx[1], idx[2], seg.p, so.p,
                           going_left.p);
        for (int d = 0; d < 3; d++) {
            size_t t2 = tb;
            auto fl = rocprim::make_transform_iterator(cnt, LeftFlag{idx[d], seg.p, dimv.p, going_left.p, d});
            TT_BH(rocprim::exclusive_scan_by_key(tstore.p, t2, seg.p, fl, lrank.p, 0, (size_t)n, rocprim::plus<int>(),
                                                 rocprim::equal_to<int>(), st));
            hipLaunchKernelGGL(k_scatter, dim3(grid_of(n)), dim3(kBlock), 0, st, n, d, idx[d], seg.p, segs.p, so.p,
                               going_left.p, lrank.p, tmp);
            std::swap(idx[d], tmp);
        }
        hipLaunchKernelGGL(k_reseg, dim3(grid_of(n)), dim3(kBlock), 0, st, n, seg.p, so.p, child_id.p);
        TT_BH(hipGetLastError());
        std::swap(segs.p, next.p);
        S = h[0];
    }
    TT_BH(hipMemcpyAsync(final_indices, idx[0], (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st));
    if (node_aabbs) TT_BH(hipMemcpyAsync(node_aabbs, box.p, n2 * sizeof(Box), hipMemcpyDeviceToHost, st));
    if (node_left) TT_BH(hipMemcpyAsync(node_left, nleft.p, n2 * sizeof(int), hipMemcpyDeviceToHost, st));
    if (node_count) TT_BH(hipMemcpyAsync(node_count, ncount.p, n2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    TT_BH(hipStreamSynchronize(st));
    if (max_depth) *max_depth = depth;
    return TT_OK;
}
