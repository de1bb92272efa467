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
#include <cstdio>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "../../include/truetrace_hip.h"

extern "C" hipStream_t tt_ctx_stream_of(tt_ctx* c);  // tt_api.hip (C linkage there)
extern "C" hipError_t tt_ctx_bind_device(tt_ctx* c);  // hipSetDevice(the context's device)
extern "C" void tt_ctx_set_error(tt_ctx* c, const char* msg);

namespace {
thread_local char g_err[256];  // the failing step of the current build, for tt_last_error
}

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

// ------------------------------------------------------------------------------- BVH8 stage
// BVH8Builder (BVH8Builder.cs:30-392) restated for the GPU: the cost pass bottom up over the BVH2's
// depth levels, the collapse top down over the CWBVH8's levels. The sequential collapse numbers the
// nodes and the leaf triangles with two running counters in depth-first order; here each CWBVH8 node
// first learns how many nodes (A) and triangles (T) its subtree allocates (bottom up), then its
// counters on entry (top down), so every node is written independently with the reference's numbers.

__device__ inline float surface_area_h(const Box& a) { return surface_area(a); }

// BFS of the BVH2 from the root: lvl_out gets the internal children of the frontier's internal nodes
__global__ void k_bvh2_level(int m, const int* __restrict__ frontier, const int* __restrict__ left,
                             const uint32_t* __restrict__ count, int* __restrict__ next, int* __restrict__ n_next,
                             int cap) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= m) return;
    const int v = frontier[t];
    if (count[v] > 0) return;
    const int l = left[v];
    const int o = atomicAdd(n_next, 2);
    if (o + 1 >= cap) return;  // not a tree: the host sees the count and fails
    next[o] = l;
    next[o + 1] = l + 1;
}

struct Dec {
    int8_t type, dl, dr;  // 0 LEAF, 1 INTERNAL, 2 DISTRIBUTE
};

// calculate_cost (BVH8Builder.cs) of one BVH2 node whose children are done; nprim / firstpos: the
// subtree's primitive count and first leaf position (count_primitives' range)
__global__ void k_cost8(int m, const int* __restrict__ nodes_lvl, const Box* __restrict__ box, const int* __restrict__ left,
                        const uint32_t* __restrict__ count, float* __restrict__ cost, Dec* __restrict__ dec,
                        int* __restrict__ nprim, int* __restrict__ firstpos, int* __restrict__ err) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= m) return;
    const int v = nodes_lvl[t];
    const Box a = box[v];
    if (count[v] > 0) {
        const int np = (int)count[v];
        nprim[v] = np;
        firstpos[v] = left[v];
        if (np != 1) {
            atomicOr(err, 2);
            return;
        }
        const float cl = surface_area(a) * (float)np;
        for (int i = 0; i < 7; i++) {
            cost[(size_t)v * 7 + i] = cl;
            dec[(size_t)v * 7 + i] = Dec{0, 0, 0};
        }
        return;
    }
    const int l = left[v], r = l + 1;
    const int np = nprim[l] + nprim[r];
    nprim[v] = np;
    firstpos[v] = firstpos[l];
    const float cost_leaf = np <= 3 ? (float)np * surface_area(a) : FLT_MAX;
    float cost_distribute = FLT_MAX;
    int dist_left = -1, dist_right = -1;
    for (int k = 0; k < 7; k++) {
        const float c = cost[(size_t)l * 7 + k] + cost[(size_t)r * 7 + 6 - k];
        if (c < cost_distribute) {
            cost_distribute = c;
            dist_left = k;
            dist_right = 6 - k;
        }
    }
    const float cost_internal = cost_distribute + surface_area(a);
    Dec d0;
    if (cost_leaf < cost_internal) {
        cost[(size_t)v * 7] = cost_leaf;
        d0.type = 0;
    } else {
        cost[(size_t)v * 7] = cost_internal;
        d0.type = 1;
    }
    d0.dl = (int8_t)dist_left;
    d0.dr = (int8_t)dist_right;
    dec[(size_t)v * 7] = d0;
    Dec prev = d0;
    for (int i = 1; i < 7; i++) {
        float cd = cost[(size_t)v * 7 + i - 1];
        int dl = -1, dr = -1;
        for (int k = 0; k < i; k++) {
            const float c = cost[(size_t)l * 7 + k] + cost[(size_t)r * 7 + i - k - 1];
            if (c < cd) {
                cd = c;
                dl = k;
                dr = i - k - 1;
            }
        }
        cost[(size_t)v * 7 + i] = cd;
        if (dl != -1) prev = Dec{2, (int8_t)dl, (int8_t)dr};
        dec[(size_t)v * 7 + i] = prev;
    }
}

struct Rec8 {
    int bvh2;       // the BVH2 node this CWBVH8 node collapses
    int child[8];   // BVH2 children by slot (order_children), -1 empty
    int crec[8];    // records of the internal children by internal rank
    int k, t;       // internal children, triangles of the leaf children
    int A, T;       // CWBVH8 nodes / triangles the subtree's collapse allocates
    int idx, C, Ct; // node index, node and triangle counters on entry to collapse()
};

// get_children + order_children + the child checks of collapse() for one CWBVH8 node; appends its
// internal children as records of the next level.
__global__ void k_expand8(int lo, int hi, int cap, Rec8* __restrict__ rec, int* __restrict__ n_rec, const Box* __restrict__ box,
                          const int* __restrict__ left, const uint32_t* __restrict__ count, const Dec* __restrict__ dec,
                          const int* __restrict__ nprim, int* __restrict__ err) {
    const int x = lo + blockIdx.x * kBlock + threadIdx.x;
    if (x >= hi) return;
    Rec8& R = rec[x];
    const int N = R.bvh2;
    int children[8];
    int cc = 0;
    bool ok = true;
    if (count[N] > 0) {
        children[cc++] = N;
    } else {
        int stn[24], sti[24], sp = 0;  // pending (node, i) expansions, processed depth first
        stn[sp] = N;
        sti[sp] = 0;
        sp++;
        bool root = true;
        while (sp > 0 && ok) {
            sp--;
            const int v = stn[sp], i = sti[sp];
            if (!root && dec[(size_t)v * 7 + i].type != 2) {  // a plain child
                if (cc >= 8) { ok = false; break; }
                children[cc++] = v;
                continue;
            }
            root = false;
            const Dec d = dec[(size_t)v * 7 + i];
            if (!(d.dl >= 0 && d.dl < 7) || !(d.dr >= 0 && d.dr < 7) || cc >= 8) { ok = false; break; }
            const int l = left[v];
            stn[sp] = l + 1; sti[sp] = d.dr; sp++;  // right after left
            stn[sp] = l; sti[sp] = d.dl; sp++;
        }
    }
    if (!ok) { atomicOr(err, 4); return; }
    // order_children: greedy slot assignment by octant direction costs
    const Box nb = box[N];
    const float px = (nb.mx[0] + nb.mn[0]) / 2.0f, py = (nb.mx[1] + nb.mn[1]) / 2.0f, pz = (nb.mx[2] + nb.mn[2]) / 2.0f;
    float cost2[8][8];
    for (int c = 0; c < cc; c++) {
        const Box ca = box[children[c]];
        const float dx = (ca.mx[0] + ca.mn[0]) / 2.0f - px, dy = (ca.mx[1] + ca.mn[1]) / 2.0f - py,
                    dz = (ca.mx[2] + ca.mn[2]) / 2.0f - pz;
        for (int s = 0; s < 8; s++) {
            const float sx = ((s >> 2) & 1) ? -1.0f : 1.0f, sy = ((s >> 1) & 1) ? -1.0f : 1.0f, sz = (s & 1) ? -1.0f : 1.0f;
            cost2[c][s] = dx * sx + dy * sy + dz * sz;
        }
    }
    int assignment[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    bool slot_filled[8] = {false, false, false, false, false, false, false, false};
    while (true) {
        float min_cost = FLT_MAX;
        int min_slot = -1, min_index = -1;
        for (int c = 0; c < cc; c++) {
            if (assignment[c] != -1) continue;
            for (int s = 0; s < 8; s++) {
                if (!slot_filled[s] && cost2[c][s] < min_cost) {
                    min_cost = cost2[c][s];
                    min_slot = s;
                    min_index = c;
                }
            }
        }
        if (min_slot == -1) break;
        slot_filled[min_slot] = true;
        assignment[min_index] = min_slot;
    }
    int slots[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    for (int c = 0; c < cc; c++) {
        if (assignment[c] < 0) { atomicOr(err, 8); return; }  // a child no slot could take (NaN boxes)
        slots[assignment[c]] = children[c];
    }
    int k = 0, t = 0;
    for (int s = 0; s < 8; s++) {
        R.child[s] = slots[s];
        const int c = slots[s];
        if (c < 0) continue;
        const int ty = dec[(size_t)c * 7].type;
        if (ty == 0) {
            const int tc = nprim[c];
            if (!(tc > 0 && tc <= 3)) { atomicOr(err, 16); return; }
            t += tc;
            if (t > 24) { atomicOr(err, 16); return; }
        } else if (ty == 1) {
            const int o = atomicAdd(n_rec, 1);
            if (o >= cap) { atomicOr(err, 128); return; }
            rec[o].bvh2 = c;
            R.crec[k++] = o;
        } else {
            atomicOr(err, 32);
            return;
        }
    }
    R.k = k;
    R.t = t;
}

__global__ void k_up8(int lo, int hi, Rec8* __restrict__ rec) {
    const int x = lo + blockIdx.x * kBlock + threadIdx.x;
    if (x >= hi) return;
    Rec8& R = rec[x];
    int A = R.k, T = R.t;
    for (int r = 0; r < R.k; r++) {
        A += rec[R.crec[r]].A;
        T += rec[R.crec[r]].T;
    }
    R.A = A;
    R.T = T;
}

__global__ void k_down8(int lo, int hi, Rec8* __restrict__ rec) {
    const int x = lo + blockIdx.x * kBlock + threadIdx.x;
    if (x >= hi) return;
    const Rec8& R = rec[x];
    int C = R.C + R.k, Ct = R.Ct + R.t;
    for (int r = 0; r < R.k; r++) {
        Rec8& c = rec[R.crec[r]];
        c.idx = R.C + r;
        c.C = C;
        c.Ct = Ct;
        C += c.A;
        Ct += c.T;
    }
}

// Mathf.Log2 / Ceil / Floor / Pow: float wrappers over System.Math (double)
__device__ inline float mathf_log2(float f) { return (float)(log((double)f) / log(2.0)); }
__device__ inline float mathf_ceil(float f) { return (float)ceil((double)f); }
__device__ inline float mathf_floor(float f) { return (float)floor((double)f); }
__device__ inline float mathf_pow2(float p) { return (float)pow(2.0, (double)p); }
// (byte)(uint)x of a C# float (unchecked): truncate toward zero, wrap to 8 bits
__device__ inline uint32_t to_byte(float x) {
    if (!(x == x)) return 0u;
    if (x <= -1.0f || x >= 4294967296.0f) return 0u;
    return (uint32_t)x & 0xffu;
}

// collapse()'s node body + Aggregate (CommonVars.cs:662-688): the 80-B node at R.idx, and the leaf
// children's primitives (count_primitives) at cwbvh_indices[R.Ct ...]
__global__ void k_fill8(int m, const Rec8* __restrict__ rec, const Box* __restrict__ box, const Dec* __restrict__ dec,
                        const int* __restrict__ nprim, const int* __restrict__ firstpos, const int* __restrict__ final_idx,
                        tt_cwbvh_node* __restrict__ out, int* __restrict__ cwbvh_indices, int* __restrict__ err) {
    const int x = blockIdx.x * kBlock + threadIdx.x;
    if (x >= m) return;
    const Rec8& R = rec[x];
    const Box a = box[R.bvh2];
    const float denom = 1.0f / (float)((1 << 8) - 1);
    const float ex = mathf_pow2(mathf_ceil(mathf_log2((a.mx[0] - a.mn[0]) * denom)));
    const float ey = mathf_pow2(mathf_ceil(mathf_log2((a.mx[1] - a.mn[1]) * denom)));
    const float ez = mathf_pow2(mathf_ceil(mathf_log2((a.mx[2] - a.mn[2]) * denom)));
    const float ox = 1.0f / ex, oy = 1.0f / ey, oz = 1.0f / ez;
    const uint32_t ux = __float_as_uint(ex), uy = __float_as_uint(ey), uz = __float_as_uint(ez);
    if ((ux & 0x807FFFFFu) || (uy & 0x807FFFFFu) || (uz & 0x807FFFFFu)) {
        atomicOr(err, 64);
        return;
    }
    uint32_t meta[2] = {0u, 0u}, qlx[2] = {0u, 0u}, qhx[2] = {0u, 0u}, qly[2] = {0u, 0u}, qhy[2] = {0u, 0u},
             qlz[2] = {0u, 0u}, qhz[2] = {0u, 0u};
    uint32_t imask = 0;
    int internal = 0, tri = 0;
    for (int s = 0; s < 8; s++) {
        const int c = R.child[s];
        if (c < 0) continue;
        const Box ca = box[c];
        const int w = s >> 2, sh = (s & 3) * 8;
        qlx[w] |= to_byte(mathf_floor((ca.mn[0] - a.mn[0]) * ox)) << sh;
        qly[w] |= to_byte(mathf_floor((ca.mn[1] - a.mn[1]) * oy)) << sh;
        qlz[w] |= to_byte(mathf_floor((ca.mn[2] - a.mn[2]) * oz)) << sh;
        qhx[w] |= to_byte(mathf_ceil((ca.mx[0] - a.mn[0]) * ox)) << sh;
        qhy[w] |= to_byte(mathf_ceil((ca.mx[1] - a.mn[1]) * oy)) << sh;
        qhz[w] |= to_byte(mathf_ceil((ca.mx[2] - a.mn[2]) * oz)) << sh;
        uint32_t mb;
        if (dec[(size_t)c * 7].type == 0) {
            const int tc = nprim[c], f = firstpos[c];
            mb = 0u;
            for (int j = 0; j < tc; j++) {
                mb |= 1u << (j + 5);
                cwbvh_indices[R.Ct + tri + j] = final_idx[f + j];
            }
            mb |= (uint32_t)tri;
            tri += tc;
        } else {
            mb = (uint32_t)((internal + 24) | 0x20);
            imask |= (1u << internal) & 0xffu;
            internal++;
        }
        meta[w] |= (mb & 0xffu) << sh;
    }
    tt_cwbvh_node o;
    o.p[0] = a.mn[0];
    o.p[1] = a.mn[1];
    o.p[2] = a.mn[2];
    o.e_imask = (ux >> 23) | ((uy >> 23) << 8) | ((uz >> 23) << 16) | (imask << 24);
    o.base_child = (uint32_t)R.C;
    o.base_tri = (uint32_t)R.Ct;
    o.meta[0] = meta[0]; o.meta[1] = meta[1];
    o.qlo_x[0] = qlx[0]; o.qlo_x[1] = qlx[1]; o.qhi_x[0] = qhx[0]; o.qhi_x[1] = qhx[1];
    o.qlo_y[0] = qly[0]; o.qlo_y[1] = qly[1]; o.qhi_y[0] = qhy[0]; o.qhi_y[1] = qhy[1];
    o.qlo_z[0] = qlz[0]; o.qlo_z[1] = qlz[1]; o.qhi_z[0] = qhz[0]; o.qhi_z[1] = qhz[1];
    out[R.idx] = o;
}

// ------------------------------------------------------------------------ presort (introsort)
// .NET Framework's ArraySortHelper IntrospectiveSort with BVH2Builder's float-key Comparison
// (BVH2Builder.cs:137-147; host restatement DotNetSort in host/tt_scene.cpp), run level by level.
// The sort is unstable, so its output order of equal keys is whatever its exact sequence of swaps
// produces -- the GPU must replay that sequence, not just sort. Partitions of one recursion level are
// disjoint and independent, so they run together; within a partition, PickPivotAndPartition's
// two-pointer scan is replayed in closed form: after the median-of-three and the pivot parked at
// hi - 1, the k-th stop of the left pointer is the k-th position (from lo + 1) whose key is >= the
// pivot's (a_k), the k-th stop of the right pointer the k-th position (from hi - 2 down) whose key
// is <= it (b_k); pairs k < K swap, where K is the first k with a_k >= b_k, and the pivot lands at
// min(a_K, b_(K-1)) (b_0 = hi - 1). Small partitions (<= 16) and partitions whose depth limit ran
// out (heapsort) are finished by one thread each, exactly as the sequential code does them.
struct SortPart {
    int lo, hi, depth;
};

__device__ inline int key_cmp(const float* __restrict__ k, int a, int b) {  // KeyCmp
    const float sign = k[a] - k[b];
    return sign < 0 ? -1 : (sign == 0 ? 0 : 1);
}
// position p of the 3n-long index array -> the axis it sorts (keys of axis d at cent + d * n)
__device__ inline const float* axis_keys(const float* cent, int n, int p) { return cent + (size_t)(p / n) * n; }

__device__ void swap_if_greater(int* it, const float* k, int a, int b) {
    if (a != b && key_cmp(k, it[a], it[b]) > 0) {
        const int t = it[a];
        it[a] = it[b];
        it[b] = t;
    }
}
__device__ void small_sort(int* it, const float* k, int lo, int hi) {  // IntroSort's <= 16 branch
    const int size = hi - lo + 1;
    if (size <= 1) return;
    if (size == 2) {
        swap_if_greater(it, k, lo, hi);
        return;
    }
    if (size == 3) {
        swap_if_greater(it, k, lo, hi - 1);
        swap_if_greater(it, k, lo, hi);
        swap_if_greater(it, k, hi - 1, hi);
        return;
    }
    for (int i = lo; i < hi; i++) {  // InsertionSort
        int j = i;
        const int t = it[i + 1];
        while (j >= lo && key_cmp(k, t, it[j]) < 0) {
            it[j + 1] = it[j];
            j--;
        }
        it[j + 1] = t;
    }
}
__device__ void down_heap(int* it, const float* k, int i, int n, int lo) {
    const int d = it[lo + i - 1];
    while (i <= n / 2) {
        int child = 2 * i;
        if (child < n && key_cmp(k, it[lo + child - 1], it[lo + child]) < 0) child++;
        if (!(key_cmp(k, d, it[lo + child - 1]) < 0)) break;
        it[lo + i - 1] = it[lo + child - 1];
        i = child;
    }
    it[lo + i - 1] = d;
}
__device__ void heap_sort(int* it, const float* k, int lo, int hi) {
    const int n = hi - lo + 1;
    for (int i = n / 2; i >= 1; i--) down_heap(it, k, i, n, lo);
    for (int i = n; i > 1; i--) {
        const int t = it[lo];
        it[lo] = it[lo + i - 1];
        it[lo + i - 1] = t;
        down_heap(it, k, 1, i - 1, lo);
    }
}

// median of three, the pivot parked at hi - 1; pk = the pivot item
__global__ void k_pivot(int P, const SortPart* __restrict__ parts, int* __restrict__ it, const float* __restrict__ cent,
                        int n, int* __restrict__ pk) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= P) return;
    const SortPart q = parts[s];
    const float* k = axis_keys(cent, n, q.lo);
    const int middle = q.lo + ((q.hi - q.lo) >> 1);
    swap_if_greater(it, k, q.lo, middle);
    swap_if_greater(it, k, q.lo, q.hi);
    swap_if_greater(it, k, middle, q.hi);
    const int pivot = it[middle];
    if (middle != q.hi - 1) {
        it[middle] = it[q.hi - 1];
        it[q.hi - 1] = pivot;
    }
    pk[s] = pivot;
}

// left-pointer stops (ge: key >= pivot, over [lo+1, hi-1]) and right-pointer stops (le: key <=
// pivot, over [lo, hi-2]) as 0/1 flags
struct GeFlag {
    const int* it;
    const int* part;
    const SortPart* parts;
    const int* pk;
    const float* cent;
    int n;
    __device__ int operator()(int p) const {
        const int s = part[p];
        if (s < 0) return 0;
        const SortPart q = parts[s];
        if (p < q.lo + 1 || p > q.hi - 1) return 0;
        const float* k = axis_keys(cent, n, p);
        return key_cmp(k, it[p], pk[s]) < 0 ? 0 : 1;
    }
};
struct LeFlagRev {  // indexed by q = 3n - 1 - p (the right pointer's direction)
    const int* it;
    const int* part;
    const SortPart* parts;
    const int* pk;
    const float* cent;
    int n, n3;
    __device__ int operator()(int qi) const {
        const int p = n3 - 1 - qi;
        const int s = part[p];
        if (s < 0) return 0;
        const SortPart q = parts[s];
        if (p < q.lo || p > q.hi - 2) return 0;
        const float* k = axis_keys(cent, n, p);
        return key_cmp(k, pk[s], it[p]) < 0 ? 0 : 1;
    }
};
struct PartKeyRev {
    const int* part;
    int n3;
    __device__ int operator()(int qi) const { return part[n3 - 1 - qi]; }
};

// aList[lo + k] = k-th left stop, bList[lo + k] = k-th right stop (k from 0)
__global__ void k_stops(int n3, const int* __restrict__ part, const SortPart* __restrict__ parts, const int* __restrict__ it,
                        const int* __restrict__ pk, const float* __restrict__ cent, int n, const int* __restrict__ gerank,
                        const int* __restrict__ lerank_rev, int* __restrict__ alist, int* __restrict__ blist) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n3) return;
    const int s = part[p];
    if (s < 0) return;
    const SortPart q = parts[s];
    const float* k = axis_keys(cent, n, p);
    if (p >= q.lo + 1 && p <= q.hi - 1 && key_cmp(k, it[p], pk[s]) >= 0) alist[q.lo + gerank[p]] = p;
    if (p >= q.lo && p <= q.hi - 2 && key_cmp(k, pk[s], it[p]) >= 0) blist[q.lo + lerank_rev[n3 - 1 - p]] = p;
}

// K (first k with a_k >= b_k) by binary search; the swap count K - 1 and the pivot's final slot
__global__ void k_crossing(int P, const SortPart* __restrict__ parts, const int* __restrict__ gerank,
                           const int* __restrict__ lerank_rev, const int* __restrict__ alist, const int* __restrict__ blist,
                           int n3, int2* __restrict__ res) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= P) return;
    const SortPart q = parts[s];
    const int cnt_ge = gerank[q.hi - 1] + 1;       // hi - 1 (the pivot) is always a stop
    const int cnt_le = lerank_rev[n3 - 1 - q.lo] + 1;  // lo (<= pivot after the median of three) is too
    auto pred = [&](int K) {  // a_K >= b_K (1-based K); b_K = -1 past the last right stop
        const int a = alist[q.lo + K - 1];
        const int b = K <= cnt_le ? blist[q.lo + K - 1] : -1;
        return a >= b;
    };
    int lo = 1, hi = cnt_ge;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pred(mid)) hi = mid;
        else lo = mid + 1;
    }
    const int K = lo;
    const int aK = alist[q.lo + K - 1];
    const int bK1 = K >= 2 ? blist[q.lo + K - 2] : q.hi - 1;
    res[s] = make_int2(K - 1, aK < bK1 ? aK : bK1);
}

__global__ void k_pswap(int n3, const int* __restrict__ part, const SortPart* __restrict__ parts, const int2* __restrict__ res,
                        const int* __restrict__ alist, const int* __restrict__ blist, int* __restrict__ it) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n3) return;
    const int s = part[p];
    if (s < 0) return;
    const int kk = p - parts[s].lo;
    if (kk >= res[s].x) return;
    const int a = alist[p], b = blist[p];
    const int t = it[a];
    it[a] = it[b];
    it[b] = t;
}

// the pivot into its slot; children: finished here (<= 16, or heapsort at depth 0) or the next level
__global__ void k_children_sort(int P, const SortPart* __restrict__ parts, const int2* __restrict__ res, int* __restrict__ it,
                                const float* __restrict__ cent, int n, SortPart* __restrict__ next, int* __restrict__ n_next,
                                int2* __restrict__ child, int* __restrict__ err) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= P) return;
    const SortPart q = parts[s];
    const int left = res[s].y;
    if (left != q.hi - 1) {
        const int t = it[left];
        it[left] = it[q.hi - 1];
        it[q.hi - 1] = t;
    }
    const float* k = axis_keys(cent, n, q.lo);
    const int d = q.depth - 1;
    int2 id = make_int2(-1, -1);
    const int bounds[2][2] = {{q.lo, left - 1}, {left + 1, q.hi}};
    for (int c = 0; c < 2; c++) {
        const int lo = bounds[c][0], hi = bounds[c][1];
        const int size = hi - lo + 1;
        if (size <= 16) {
            small_sort(it, k, lo, hi);
        } else if (d == 0) {
            if (size > 65536) atomicOr(err, 1);  // left to the host: one thread would take too long
            else heap_sort(it, k, lo, hi);
        } else {
            const int o = atomicAdd(n_next, 1);
            next[o] = SortPart{lo, hi, d};
            if (c == 0) id.x = o;
            else id.y = o;
        }
    }
    child[s] = id;
}

__global__ void k_repart(int n3, int* __restrict__ part, const int2* __restrict__ res, const int2* __restrict__ child) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n3) return;
    const int s = part[p];
    if (s < 0) return;
    const int left = res[s].y;
    part[p] = p < left ? child[s].x : (p > left ? child[s].y : -1);
}

// BVH2Builder's centroids, (max - min) / 2 + min per axis, axis-major; flags non-finite keys
__global__ void k_centroids(int n, const Box* __restrict__ prims, float* __restrict__ cent, int* __restrict__ it,
                            int* __restrict__ bad) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const Box b = prims[i];
    for (int d = 0; d < 3; d++) {
        const float c = (b.mx[d] - b.mn[d]) / 2.0f + b.mn[d];
        cent[(size_t)d * n + i] = c;
        it[(size_t)d * n + i] = i;
        if (!(c - c == 0.0f)) atomicOr(bad, 1);  // NaN or infinity: the comparator is not an order there
    }
}

// exclusive-scan input: live children per segment (0 past the last segment, so base[S] = total)
struct NextCount {
    const SplitOut* so;
    int S;
    __device__ int operator()(int q) const { return q < S ? so[q].n_next : 0; }
};

#define TT_BH(x)                                                                                  \
    do {                                                                                          \
        const hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                                   \
            std::snprintf(g_err, sizeof(g_err), "%s: %s", #x, hipGetErrorString(e_));             \
            return e_ == hipErrorOutOfMemory ? TT_ERR_OOM : TT_ERR_HIP;                            \
        }                                                                                         \
    } while (0)
#define TT_BFAIL(status, msg)                                  \
    do {                                                       \
        std::snprintf(g_err, sizeof(g_err), "%s", msg);        \
        return status;                                         \
    } while (0)

// The BVH2 stage's result, left on the device for the BVH8 stage: BVH2Nodes (boxes, left, count; 2n
// slots) and FinalIndices.
struct Bvh2Dev {
    DBuf<Box> box;
    DBuf<int> left, final_idx;
    DBuf<uint32_t> count;
    uint32_t depth = 0;
};

static tt_status bvh2_stage(hipStream_t st, const float* aabbs, int n, const int32_t* presorted, Bvh2Dev& R) {

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
    TT_BH(R.box.alloc(n2));
    TT_BH(R.left.alloc(n2));
    TT_BH(R.count.alloc(n2));
    TT_BH(R.final_idx.alloc(n));
    if (n == 1) {  // BuildRecursive(0, 2, 0, 1, 0): the root is a leaf
        const uint32_t one = 1u;
        TT_BH(hipMemsetAsync(R.box.p, 0, n2 * sizeof(Box), st));
        TT_BH(hipMemcpyAsync(R.box.p, &root, sizeof(Box), hipMemcpyHostToDevice, st));
        TT_BH(hipMemsetAsync(R.left.p, 0, n2 * sizeof(int), st));
        TT_BH(hipMemsetAsync(R.count.p, 0, n2 * sizeof(uint32_t), st));
        TT_BH(hipMemcpyAsync(R.count.p, &one, sizeof(uint32_t), hipMemcpyHostToDevice, st));
        TT_BH(hipMemcpyAsync(R.final_idx.p, presorted, sizeof(int), hipMemcpyHostToDevice, st));
        TT_BH(hipStreamSynchronize(st));
        R.depth = 0;
        return TT_OK;
    }
    DBuf<Box> prims, pre, sufr, c_left, c_right;
    DBuf<int> idxb[4], seg, lrank, c_pos, dimv, base, err;
    Box* box_p = R.box.p;
    int* nleft_p = R.left.p;
    uint32_t* ncount_p = R.count.p;
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
    TT_BH(hipMemsetAsync(box_p, 0, n2 * sizeof(Box), st));  // NativeArrayOptions.ClearMemory
    TT_BH(hipMemcpyAsync(box_p, &root, sizeof(Box), hipMemcpyHostToDevice, st));
    TT_BH(hipMemsetAsync(nleft_p, 0, n2 * sizeof(int), st));
    TT_BH(hipMemsetAsync(ncount_p, 0, n2 * sizeof(uint32_t), st));
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
                           c_right.p, so.p, box_p, nleft_p, ncount_p, err.p);
        size_t t = tb;
        auto nc = rocprim::make_transform_iterator(cnt, NextCount{so.p, S});
        TT_BH(rocprim::exclusive_scan(tstore.p, t, nc, base.p, 0, (size_t)S + 1, rocprim::plus<int>(), st));
        int h[2] = {0, 0};
        TT_BH(hipMemcpyAsync(&h[0], base.p + S, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipMemcpyAsync(&h[1], err.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipStreamSynchronize(st));
        if (h[1]) TT_BFAIL(TT_ERR_UNSUPPORTED, "BVH2 stage: a node has no finite SAH split");  // the C# misbehaves too
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
    TT_BH(hipMemcpyAsync(R.final_idx.p, idx[0], (size_t)n * sizeof(int), hipMemcpyDeviceToDevice, st));
    TT_BH(hipStreamSynchronize(st));
    R.depth = depth;
    return TT_OK;
}

static tt_status check_inputs(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted) {
    if (!ctx || !aabbs || !n || !presorted || n >= (1u << 30)) return TT_ERR_INVALID_ARG;
    for (size_t i = 0; i < 3 * (size_t)n; i++)
        if (presorted[i] < 0 || (uint32_t)presorted[i] >= n) return TT_ERR_INVALID_ARG;
    return TT_OK;
}

extern "C" tt_status tt_bvh2_build_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                                          int32_t* final_indices, float* node_aabbs, int32_t* node_left,
                                          uint32_t* node_count, uint32_t* max_depth) {
    tt_status s = check_inputs(ctx, aabbs, n, presorted);
    if (s != TT_OK || !final_indices) return s != TT_OK ? s : TT_ERR_INVALID_ARG;
    TT_BH(tt_ctx_bind_device(ctx));  // allocations and launches on the context's GPU
    hipStream_t st = tt_ctx_stream_of(ctx);
    Bvh2Dev R;
    if ((s = bvh2_stage(st, aabbs, (int)n, presorted, R)) != TT_OK) {
        tt_ctx_set_error(ctx, g_err);
        return s;
    }
    const size_t n2 = 2 * (size_t)n;
    TT_BH(hipMemcpyAsync(final_indices, R.final_idx.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st));
    if (node_aabbs) TT_BH(hipMemcpyAsync(node_aabbs, R.box.p, n2 * sizeof(Box), hipMemcpyDeviceToHost, st));
    if (node_left) TT_BH(hipMemcpyAsync(node_left, R.left.p, n2 * sizeof(int), hipMemcpyDeviceToHost, st));
    if (node_count) TT_BH(hipMemcpyAsync(node_count, R.count.p, n2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    TT_BH(hipStreamSynchronize(st));
    if (max_depth) *max_depth = R.depth;
    return TT_OK;
}

static tt_status blas_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                             tt_cwbvh_node* nodes, uint32_t max_nodes, uint32_t* n_nodes, int32_t* cwbvh_indices,
                             uint32_t* bvh2_depth);

extern "C" tt_status tt_blas_build_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                                          tt_cwbvh_node* nodes, uint32_t max_nodes, uint32_t* n_nodes,
                                          int32_t* cwbvh_indices, uint32_t* bvh2_depth) {
    g_err[0] = 0;
    const tt_status s = blas_device(ctx, aabbs, n, presorted, nodes, max_nodes, n_nodes, cwbvh_indices, bvh2_depth);
    if (s != TT_OK) tt_ctx_set_error(ctx, g_err[0] ? g_err : "tt_blas_build_device: invalid argument");
    return s;
}

static tt_status blas_device(tt_ctx* ctx, const float* aabbs, uint32_t n, const int32_t* presorted,
                             tt_cwbvh_node* nodes, uint32_t max_nodes, uint32_t* n_nodes, int32_t* cwbvh_indices,
                             uint32_t* bvh2_depth) {
    tt_status s = check_inputs(ctx, aabbs, n, presorted);
    if (s != TT_OK) return s;
    if (!nodes || !n_nodes || !cwbvh_indices) return TT_ERR_INVALID_ARG;
    TT_BH(tt_ctx_bind_device(ctx));  // allocations and launches on the context's GPU
    hipStream_t st = tt_ctx_stream_of(ctx);
    Bvh2Dev B;
    if ((s = bvh2_stage(st, aabbs, (int)n, presorted, B)) != TT_OK) return s;
    const size_t n2 = 2 * (size_t)n;
    // BVH2 levels, root first (for the bottom-up cost pass)
    DBuf<int> order, cnt1, err;
    TT_BH(order.alloc(n2));
    TT_BH(cnt1.alloc(1));
    TT_BH(err.alloc(1));
    TT_BH(hipMemsetAsync(err.p, 0, sizeof(int), st));
    const int zero = 0;
    TT_BH(hipMemcpyAsync(order.p, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    std::vector<int> lvl{0, 1};
    while (lvl.back() > lvl[lvl.size() - 2]) {
        const int lo = lvl[lvl.size() - 2], hi = lvl.back();
        TT_BH(hipMemcpyAsync(cnt1.p, &zero, sizeof(int), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_bvh2_level, dim3(grid_of(hi - lo)), dim3(kBlock), 0, st, hi - lo, order.p + lo, B.left.p,
                           B.count.p, order.p + hi, cnt1.p, (int)(n2 - (size_t)hi));
        int m = 0;
        TT_BH(hipMemcpyAsync(&m, cnt1.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipStreamSynchronize(st));
        if ((size_t)hi + (size_t)m > n2) TT_BFAIL(TT_ERR_INVALID_ARG, "BVH2 levels: not a binary tree");
        lvl.push_back(hi + m);
    }
    // cost pass, deepest level first
    DBuf<float> cost;
    DBuf<Dec> dec;
    DBuf<int> nprim, firstpos;
    TT_BH(cost.alloc(n2 * 7));
    TT_BH(dec.alloc(n2 * 7));
    TT_BH(nprim.alloc(n2));
    TT_BH(firstpos.alloc(n2));
    for (size_t L = lvl.size() - 1; L-- > 0;) {
        const int lo = lvl[L], hi = lvl[L + 1];
        if (hi > lo)
            hipLaunchKernelGGL(k_cost8, dim3(grid_of(hi - lo)), dim3(kBlock), 0, st, hi - lo, order.p + lo, B.box.p,
                               B.left.p, B.count.p, cost.p, dec.p, nprim.p, firstpos.p, err.p);
    }
    // collapse: CWBVH8 levels top down (records appended per level)
    const size_t cap = std::max<size_t>(1, (size_t)n);
    DBuf<Rec8> rec;
    DBuf<int> nrec;
    TT_BH(rec.alloc(cap));
    TT_BH(nrec.alloc(1));
    Rec8 root{};
    root.bvh2 = 0;
    root.idx = 0;
    root.C = 1;
    root.Ct = 0;
    const int one = 1;
    TT_BH(hipMemcpyAsync(rec.p, &root, sizeof(Rec8), hipMemcpyHostToDevice, st));
    TT_BH(hipMemcpyAsync(nrec.p, &one, sizeof(int), hipMemcpyHostToDevice, st));
    std::vector<int> r8{0, 1};
    while (r8.back() > r8[r8.size() - 2]) {
        const int lo = r8[r8.size() - 2], hi = r8.back();
        hipLaunchKernelGGL(k_expand8, dim3(grid_of(hi - lo)), dim3(kBlock), 0, st, lo, hi, (int)cap, rec.p, nrec.p, B.box.p,
                           B.left.p, B.count.p, dec.p, nprim.p, err.p);
        int h[2] = {0, 0};
        TT_BH(hipMemcpyAsync(&h[0], nrec.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipMemcpyAsync(&h[1], err.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipStreamSynchronize(st));
        if (h[1]) TT_BFAIL(TT_ERR_UNSUPPORTED, "BVH8 stage: BVH8Builder.build fails on this tree");
        if ((size_t)h[0] > cap) TT_BFAIL(TT_ERR_UNSUPPORTED, "BVH8 stage: more CWBVH8 nodes than BVH2 nodes");
        r8.push_back(h[0]);
    }
    const int total = r8.back();
    if ((uint32_t)total > max_nodes) TT_BFAIL(TT_ERR_INVALID_ARG, "tt_blas_build_device: max_nodes too small");
    for (size_t L = r8.size() - 1; L-- > 0;) {
        const int lo = r8[L], hi = r8[L + 1];
        if (hi > lo) hipLaunchKernelGGL(k_up8, dim3(grid_of(hi - lo)), dim3(kBlock), 0, st, lo, hi, rec.p);
    }
    for (size_t L = 0; L + 1 < r8.size(); L++) {
        const int lo = r8[L], hi = r8[L + 1];
        if (hi > lo) hipLaunchKernelGGL(k_down8, dim3(grid_of(hi - lo)), dim3(kBlock), 0, st, lo, hi, rec.p);
    }
    DBuf<tt_cwbvh_node> out;
    DBuf<int> idxo;
    TT_BH(out.alloc((size_t)total));
    TT_BH(idxo.alloc(n));
    TT_BH(hipMemsetAsync(out.p, 0, (size_t)total * sizeof(tt_cwbvh_node), st));
    TT_BH(hipMemsetAsync(idxo.p, 0, (size_t)n * sizeof(int), st));
    hipLaunchKernelGGL(k_fill8, dim3(grid_of(total)), dim3(kBlock), 0, st, total, rec.p, B.box.p, dec.p, nprim.p,
                       firstpos.p, B.final_idx.p, out.p, idxo.p, err.p);
    TT_BH(hipGetLastError());
    int e = 0;
    TT_BH(hipMemcpyAsync(&e, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    TT_BH(hipMemcpyAsync(nodes, out.p, (size_t)total * sizeof(tt_cwbvh_node), hipMemcpyDeviceToHost, st));
    TT_BH(hipMemcpyAsync(cwbvh_indices, idxo.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st));
    TT_BH(hipStreamSynchronize(st));
    if (e) TT_BFAIL(TT_ERR_UNSUPPORTED, "BVH8 stage: a node's quantization exponent is not a power of two");
    *n_nodes = (uint32_t)total;
    if (bvh2_depth) *bvh2_depth = B.depth;
    return TT_OK;
}

// The three presorts of BVH2Builder on the GPU. TT_ERR_UNSUPPORTED (the caller sorts on the host,
// tt_bvh2_presort) when a key is not finite or a depth-exhausted partition is too large for the
// one-thread heapsort.
static tt_status presort_device(hipStream_t st, const float* aabbs, int n, int32_t* presorted) {
    const int n3 = 3 * n;
    DBuf<Box> prims;
    DBuf<float> cent;
    DBuf<int> it, part, gerank, lerank, alist, blist, pk, cnt, err;
    DBuf<SortPart> parts, next;
    DBuf<int2> res, child;
    const size_t pmax = (size_t)n3 / 17 + 4;  // live partitions per level (> 16 elements each)
    TT_BH(prims.alloc(n));
    TT_BH(cent.alloc(n3));
    TT_BH(it.alloc(n3));
    TT_BH(part.alloc(n3));
    TT_BH(gerank.alloc(n3));
    TT_BH(lerank.alloc(n3));
    TT_BH(alist.alloc(n3));
    TT_BH(blist.alloc(n3));
    TT_BH(pk.alloc(pmax));
    TT_BH(parts.alloc(pmax));
    TT_BH(next.alloc(pmax));
    TT_BH(res.alloc(pmax));
    TT_BH(child.alloc(pmax));
    TT_BH(cnt.alloc(1));
    TT_BH(err.alloc(1));
    TT_BH(hipMemcpyAsync(prims.p, aabbs, (size_t)n * sizeof(Box), hipMemcpyHostToDevice, st));
    TT_BH(hipMemsetAsync(err.p, 0, sizeof(int), st));
    hipLaunchKernelGGL(k_centroids, dim3(grid_of(n)), dim3(kBlock), 0, st, n, prims.p, cent.p, it.p, err.p);
    int bad = 0;
    TT_BH(hipMemcpyAsync(&bad, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    TT_BH(hipStreamSynchronize(st));
    if (bad) TT_BFAIL(TT_ERR_UNSUPPORTED, "presort: non-finite centroid keys (host sort)");
    if (n <= 16) TT_BFAIL(TT_ERR_UNSUPPORTED, "presort: tiny inputs are sorted on the host");
    // Sort(length): IntroSort(0, length - 1, 2 * FloorLog2(length)), FloorLog2 = bit length
    int fl = 0;
    for (int m = n; m >= 1; m /= 2) fl++;
    std::vector<SortPart> roots;
    std::vector<int> part_h(n3, -1);
    for (int d = 0; d < 3; d++) roots.push_back(SortPart{d * n, d * n + n - 1, 2 * fl});
    int P = (int)roots.size();
    for (int s = 0; s < P; s++)
        for (int p = roots[s].lo; p <= roots[s].hi; p++) part_h[p] = s;
    TT_BH(hipMemcpyAsync(parts.p, roots.data(), (size_t)P * sizeof(SortPart), hipMemcpyHostToDevice, st));
    TT_BH(hipMemcpyAsync(part.p, part_h.data(), (size_t)n3 * sizeof(int), hipMemcpyHostToDevice, st));
    auto cnt_it = rocprim::make_counting_iterator<int>(0);
    size_t tb = 0, t1 = 0;
    {
        auto ge = rocprim::make_transform_iterator(cnt_it, GeFlag{it.p, part.p, parts.p, pk.p, cent.p, n});
        TT_BH(rocprim::exclusive_scan_by_key(nullptr, t1, part.p, ge, gerank.p, 0, (size_t)n3, rocprim::plus<int>(),
                                             rocprim::equal_to<int>(), st));
        tb = std::max(tb, t1);
        auto le = rocprim::make_transform_iterator(cnt_it, LeFlagRev{it.p, part.p, parts.p, pk.p, cent.p, n, n3});
        auto rk = rocprim::make_transform_iterator(cnt_it, PartKeyRev{part.p, n3});
        TT_BH(rocprim::exclusive_scan_by_key(nullptr, t1, rk, le, lerank.p, 0, (size_t)n3, rocprim::plus<int>(),
                                             rocprim::equal_to<int>(), st));
        tb = std::max(tb, t1);
    }
    DBuf<unsigned char> tstore;
    TT_BH(tstore.alloc(tb));
    while (P > 0) {
        hipLaunchKernelGGL(k_pivot, dim3(grid_of(P)), dim3(kBlock), 0, st, P, parts.p, it.p, cent.p, n, pk.p);
        size_t t = tb;
        auto ge = rocprim::make_transform_iterator(cnt_it, GeFlag{it.p, part.p, parts.p, pk.p, cent.p, n});
        TT_BH(rocprim::exclusive_scan_by_key(tstore.p, t, part.p, ge, gerank.p, 0, (size_t)n3, rocprim::plus<int>(),
                                             rocprim::equal_to<int>(), st));
        t = tb;
        auto le = rocprim::make_transform_iterator(cnt_it, LeFlagRev{it.p, part.p, parts.p, pk.p, cent.p, n, n3});
        auto rk = rocprim::make_transform_iterator(cnt_it, PartKeyRev{part.p, n3});
        TT_BH(rocprim::exclusive_scan_by_key(tstore.p, t, rk, le, lerank.p, 0, (size_t)n3, rocprim::plus<int>(),
                                             rocprim::equal_to<int>(), st));
        hipLaunchKernelGGL(k_stops, dim3(grid_of(n3)), dim3(kBlock), 0, st, n3, part.p, parts.p, it.p, pk.p, cent.p, n,
                           gerank.p, lerank.p, alist.p, blist.p);
        hipLaunchKernelGGL(k_crossing, dim3(grid_of(P)), dim3(kBlock), 0, st, P, parts.p, gerank.p, lerank.p, alist.p,
                           blist.p, n3, res.p);
        hipLaunchKernelGGL(k_pswap, dim3(grid_of(n3)), dim3(kBlock), 0, st, n3, part.p, parts.p, res.p, alist.p, blist.p,
                           it.p);
        TT_BH(hipMemsetAsync(cnt.p, 0, sizeof(int), st));
        hipLaunchKernelGGL(k_children_sort, dim3(grid_of(P)), dim3(kBlock), 0, st, P, parts.p, res.p, it.p, cent.p, n,
                           next.p, cnt.p, child.p, err.p);
        hipLaunchKernelGGL(k_repart, dim3(grid_of(n3)), dim3(kBlock), 0, st, n3, part.p, res.p, child.p);
        TT_BH(hipGetLastError());
        int h[2] = {0, 0};
        TT_BH(hipMemcpyAsync(&h[0], cnt.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipMemcpyAsync(&h[1], err.p, sizeof(int), hipMemcpyDeviceToHost, st));
        TT_BH(hipStreamSynchronize(st));
        if (h[1]) TT_BFAIL(TT_ERR_UNSUPPORTED, "presort: a depth-exhausted partition is too large (host sort)");
        if ((size_t)h[0] > pmax) TT_BFAIL(TT_ERR_UNSUPPORTED, "presort: too many partitions");
        std::swap(parts.p, next.p);
        P = h[0];
    }
    TT_BH(hipMemcpyAsync(presorted, it.p, (size_t)n3 * sizeof(int), hipMemcpyDeviceToHost, st));
    TT_BH(hipStreamSynchronize(st));
    return TT_OK;
}

extern "C" tt_status tt_bvh2_presort_device(tt_ctx* ctx, const float* aabbs, uint32_t n, int32_t* presorted) {
    if (!ctx || !aabbs || !n || !presorted || n >= (1u << 29)) return TT_ERR_INVALID_ARG;
    g_err[0] = 0;
    if (tt_ctx_bind_device(ctx) != hipSuccess) {  // allocations and launches on the context's GPU
        tt_ctx_set_error(ctx, "tt_bvh2_presort_device: hipSetDevice failed");
        return TT_ERR_HIP;
    }
    const tt_status s = presort_device(tt_ctx_stream_of(ctx), aabbs, (int)n, presorted);
    if (s != TT_OK) tt_ctx_set_error(ctx, g_err[0] ? g_err : "tt_bvh2_presort_device failed");
    return s;
}
