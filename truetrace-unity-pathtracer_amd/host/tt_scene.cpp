// tt_scene.cpp — C++ restatement of TrueTrace's CPU acceleration-structure pipeline
// (the producer side of the trace boundary). See include/truetrace_scene.h for the map
// from functions here to the reference C# files. Compiled with -ffp-contract=off so every
// float expression rounds like the C# source (IEEE single, no fusion).
#include "../../include/truetrace_scene.h"

#include <pthread.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <new>
#include <thread>
#include <vector>

namespace {

struct V3 {
    float x, y, z;
};
static inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator/(V3 a, float d) { return v3(a.x / d, a.y / d, a.z / d); }
static inline V3 operator*(float d, V3 a) { return v3(a.x * d, a.y * d, a.z * d); }
static inline float& at(V3& v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline float dotv(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // Vector3.Dot

// CommonVars.AABB (CommonVars.cs:304-402); C# field order BBMax then BBMin.
struct AABB {
    V3 BBMax, BBMin;
    void init() {
        const float mx = std::numeric_limits<float>::max();
        BBMax = v3(-mx, -mx, -mx);  // float.MinValue
        BBMin = v3(mx, mx, mx);
    }
    void Extend(const AABB& b) {
        if (b.BBMin.x < BBMin.x) BBMin.x = b.BBMin.x;
        if (b.BBMin.y < BBMin.y) BBMin.y = b.BBMin.y;
        if (b.BBMin.z < BBMin.z) BBMin.z = b.BBMin.z;
        if (b.BBMax.x > BBMax.x) BBMax.x = b.BBMax.x;
        if (b.BBMax.y > BBMax.y) BBMax.y = b.BBMax.y;
        if (b.BBMax.z > BBMax.z) BBMax.z = b.BBMax.z;
    }
    void Extend(V3 P) {
        if (P.x < BBMin.x) BBMin.x = P.x;
        if (P.x > BBMax.x) BBMax.x = P.x;
        if (P.y < BBMin.y) BBMin.y = P.y;
        if (P.y > BBMax.y) BBMax.y = P.y;
        if (P.z < BBMin.z) BBMin.z = P.z;
        if (P.z > BBMax.z) BBMax.z = P.z;
    }
    void Create(V3 A, V3 B) {
        BBMax = A;
        BBMin = A;
        Extend(B);
    }
    void Validate(V3 Scale) {
        for (int i = 0; i < 3; i++) {
            if (at(BBMax, i) - at(BBMin, i) < at(Scale, i)) {
                at(BBMin, i) -= at(Scale, i);
                at(BBMax, i) += at(Scale, i);
            }
        }
    }
};

static inline float surface_area(const AABB& a) {
    const V3 s = a.BBMax - a.BBMin;
    return 2.0f * ((s.x * s.y) + (s.x * s.z) + (s.y * s.z));
}

// ---------------------------------------------------------------- .NET introsort
// Restatement of the .NET Framework reference-source ArraySortHelper<T> IntrospectiveSort
// used by System.Array.Sort(T[], Comparison<T>) (BVH2Builder.cs:137-147).
struct KeyCmp {
    const float* k;
    int operator()(int a, int b) const {
        const float sign = k[a] - k[b];
        return sign < 0 ? -1 : (sign == 0 ? 0 : 1);
    }
};

struct DotNetSort {
    int* keys;
    KeyCmp cmp;
    void SwapIfGreater(int a, int b) {
        if (a != b && cmp(keys[a], keys[b]) > 0) {
            const int t = keys[a];
            keys[a] = keys[b];
            keys[b] = t;
        }
    }
    void Swap(int i, int j) {
        if (i != j) {
            const int t = keys[i];
            keys[i] = keys[j];
            keys[j] = t;
        }
    }
    void InsertionSort(int lo, int hi) {
        for (int i = lo; i < hi; i++) {
            int j = i;
            const int t = keys[i + 1];
            while (j >= lo && cmp(t, keys[j]) < 0) {
                keys[j + 1] = keys[j];
                j--;
            }
            keys[j + 1] = t;
        }
    }
    void DownHeap(int i, int n, int lo) {
        const int d = keys[lo + i - 1];
        while (i <= n / 2) {
            int child = 2 * i;
            if (child < n && cmp(keys[lo + child - 1], keys[lo + child]) < 0) child++;
            if (!(cmp(d, keys[lo + child - 1]) < 0)) break;
            keys[lo + i - 1] = keys[lo + child - 1];
            i = child;
        }
        keys[lo + i - 1] = d;
    }
    void Heapsort(int lo, int hi) {
        const int n = hi - lo + 1;
        for (int i = n / 2; i >= 1; i = i - 1) DownHeap(i, n, lo);
        for (int i = n; i > 1; i = i - 1) {
            Swap(lo, lo + i - 1);
            DownHeap(1, i - 1, lo);
        }
    }
    int PickPivotAndPartition(int lo, int hi) {
        const int middle = lo + ((hi - lo) >> 1);
        SwapIfGreater(lo, middle);
        SwapIfGreater(lo, hi);
        SwapIfGreater(middle, hi);
        const int pivot = keys[middle];
        Swap(middle, hi - 1);
        int left = lo, right = hi - 1;
        while (left < right) {
            while (cmp(keys[++left], pivot) < 0) {
            }
            while (cmp(pivot, keys[--right]) < 0) {
            }
            if (left >= right) break;
            Swap(left, right);
        }
        Swap(left, hi - 1);
        return left;
    }
    void IntroSort(int lo, int hi, int depthLimit) {
        while (hi > lo) {
            const int partitionSize = hi - lo + 1;
            if (partitionSize <= 16) {
                if (partitionSize == 1) return;
                if (partitionSize == 2) {
                    SwapIfGreater(lo, hi);
                    return;
                }
                if (partitionSize == 3) {
                    SwapIfGreater(lo, hi - 1);
                    SwapIfGreater(lo, hi);
                    SwapIfGreater(hi - 1, hi);
                    return;
                }
                InsertionSort(lo, hi);
                return;
            }
            if (depthLimit == 0) {
                Heapsort(lo, hi);
                return;
            }
            depthLimit--;
            const int p = PickPivotAndPartition(lo, hi);
            IntroSort(p + 1, hi, depthLimit);
            hi = p - 1;
        }
    }
    static int FloorLog2(int n) {
        int result = 0;
        while (n >= 1) {
            result++;
            n = n / 2;
        }
        return result;
    }
    void Sort(int length) {
        if (length < 2) return;
        IntroSort(0, length - 1, 2 * FloorLog2(length));
    }
};

// A thread with a large stack (the builders recurse to BVH2 depth); runs inline if it cannot start.
struct BigThread {
    pthread_t th{};
    bool started = false;
    std::function<void()> fn;
    template <class F>
    void start(F&& f) {
        fn = std::forward<F>(f);
        pthread_attr_t attr;
        pthread_attr_init(&attr);
        pthread_attr_setstacksize(&attr, (size_t)1 << 28);
        auto tramp = [](void* p) -> void* {
            (*static_cast<std::function<void()>*>(p))();
            return nullptr;
        };
        started = pthread_create(&th, &attr, tramp, &fn) == 0;
        pthread_attr_destroy(&attr);
    }
    void join() {
        if (started) pthread_join(th, nullptr);
        else fn();
    }
};

// ---------------------------------------------------------------- BVH2Builder
struct BVHNode2Data {
    AABB aabb;
    int left;
    uint32_t count;
};

// BVH2Builder.cs:9-217. Both constructors (BLAS over triangle AABBs, TLAS over mesh AABBs)
// run the same full-sweep SAH over per-axis presorted centroids.
struct BVH2Builder {
    std::vector<BVHNode2Data> BVH2Nodes;
    std::vector<int> DimensionedIndices, temp, FinalIndices;
    std::vector<char> indices_going_left;
    std::vector<float> SAH;
    const AABB* Primitives = nullptr;
    int PrimCount = 0;
    std::atomic<uint32_t> max_depth{0};

    struct ObjectSplit {
        int index;
        float cost;
        int dimension;
        AABB aabb_left, aabb_right;
    };

    // The full SAH sweep of one axis (BVH2Builder.cs:62-96): the split with the lowest cost, ties to
    // the lowest index (the sweep runs downwards with `cost <= best`). Scratch (SAH, temp) is used at
    // [first_index, first_index + index_count) of its axis, so disjoint subtrees and the three axes
    // can run concurrently.
    struct AxisBest {
        float cost;
        int index;
        AABB right;
    };
    AxisBest sweep_axis(int dimension, int first_index, int index_count) {
        AxisBest b;
        b.cost = std::numeric_limits<float>::max();
        b.index = -1;
        b.right.init();
        AABB aabb_left, aabb_right;
        aabb_left.init();
        aabb_right.init();
        const int Offset = PrimCount * dimension + first_index;
        float* sah = &SAH[(size_t)PrimCount * dimension + first_index];
        for (int i = 1; i < index_count; i++) {
            aabb_left.Extend(Primitives[DimensionedIndices[Offset + i - 1]]);
            sah[i] = surface_area(aabb_left) * (float)i;
        }
        for (int i = index_count - 1; i > 0; i--) {
            aabb_right.Extend(Primitives[DimensionedIndices[Offset + i]]);
            const float cost = sah[i] + surface_area(aabb_right) * (float)(index_count - i);
            if (cost <= b.cost) {
                b.cost = cost;
                b.index = first_index + i;
                b.right = aabb_right;
            }
        }
        return b;
    }
    // partition_sah: the reference sweeps x, y, z in turn with one running `cost <= split.cost`, so
    // an axis takes over exactly when its own best cost is <= the best so far.
    static constexpr int kAxisParMin = 1 << 20;
    ObjectSplit partition_sah(int first_index, int index_count) {
        ObjectSplit split;
        split.cost = std::numeric_limits<float>::max();
        split.index = -1;
        split.dimension = -1;
        split.aabb_left.init();
        split.aabb_right.init();
        AxisBest best[3];
        if (parallel && index_count >= kAxisParMin) {
            std::thread t1([&] { best[1] = sweep_axis(1, first_index, index_count); });
            std::thread t2([&] { best[2] = sweep_axis(2, first_index, index_count); });
            best[0] = sweep_axis(0, first_index, index_count);
            t1.join();
            t2.join();
        } else {
            for (int d = 0; d < 3; d++) best[d] = sweep_axis(d, first_index, index_count);
        }
        for (int d = 0; d < 3; d++) {
            if (best[d].index != -1 && best[d].cost <= split.cost) {
                split.cost = best[d].cost;
                split.index = best[d].index;
                split.dimension = d;
                split.aabb_right = best[d].right;
            }
        }
        const int Offset = split.dimension * PrimCount;
        for (int i = first_index; i < split.index; i++)
            split.aabb_left.Extend(Primitives[DimensionedIndices[Offset + i]]);
        return split;
    }

    // BuildRecursive (BVH2Builder.cs:166-217). A subtree of k primitives takes 2(k-1) node slots of
    // the sequential depth-first numbering, so the right subtree's first slot is known before the
    // left one is built: large subtrees near the root are built on their own threads and the nodes
    // are exactly the sequential ones.
    static constexpr int kParMin = 1 << 16;
    static constexpr uint32_t kParDepth = 4;
    bool parallel = true;  // TT_BUILD_SERIAL set: one thread (the tests compare both)
    void BuildRecursive(int nodesi, int node_index, int first_index, int index_count, uint32_t depth) {
        for (uint32_t m = max_depth.load(std::memory_order_relaxed); depth > m &&
             !max_depth.compare_exchange_weak(m, depth, std::memory_order_relaxed);) {
        }
        if (index_count == 1) {
            BVH2Nodes[nodesi].left = first_index;
            BVH2Nodes[nodesi].count = (uint32_t)index_count;
            return;
        }
        ObjectSplit sp = partition_sah(first_index, index_count);
        int Offset = sp.dimension * PrimCount;
        const int IndexEnd = first_index + index_count;
        for (int i = first_index; i < IndexEnd; i++)
            indices_going_left[DimensionedIndices[Offset + i]] = i < sp.index;
        for (int dim = 0; dim < 3; dim++) {
            if (dim == sp.dimension) continue;
            int left = first_index;
            int right = sp.index;
            Offset = dim * PrimCount;
            for (int i = first_index; i < IndexEnd; i++) {
                const int index = DimensionedIndices[Offset + i];
                temp[indices_going_left[index] ? (left++) : (right++)] = index;
            }
            std::memcpy(&DimensionedIndices[Offset + first_index], temp.data() + first_index,
                        sizeof(int) * (size_t)index_count);
        }
        BVH2Nodes[nodesi].left = node_index;
        BVH2Nodes[BVH2Nodes[nodesi].left].aabb = sp.aabb_left;
        BVH2Nodes[BVH2Nodes[nodesi].left + 1].aabb = sp.aabb_right;
        const int l = BVH2Nodes[nodesi].left;
        const int n_left = sp.index - first_index, n_right = first_index + index_count - sp.index;
        const int next_left = node_index + 2, next_right = next_left + 2 * (n_left - 1);
        if (parallel && index_count >= kParMin && depth < kParDepth) {
            BigThread t;
            t.start([=] { BuildRecursive(l, next_left, first_index, n_left, depth + 1); });
            BuildRecursive(l + 1, next_right, sp.index, n_right, depth + 1);
            t.join();
        } else {
            BuildRecursive(l, next_left, first_index, n_left, depth + 1);
            BuildRecursive(l + 1, next_right, sp.index, n_right, depth + 1);
        }
    }

    void build(const AABB* prims, int n) {
        PrimCount = n;
        Primitives = prims;
        FinalIndices.resize(n);
        temp.assign(n, 0);
        SAH.assign((size_t)n * 3, 0.0f);
        indices_going_left.assign(n, 0);
        DimensionedIndices.resize((size_t)n * 3);
        std::vector<float> cx(n), cy(n), cz(n);
        BVHNode2Data zero{};
        zero.aabb.BBMax = v3(0, 0, 0);
        zero.aabb.BBMin = v3(0, 0, 0);
        zero.left = 0;
        zero.count = 0;
        BVH2Nodes.assign((size_t)n * 2, zero);  // NativeArrayOptions.ClearMemory
        BVH2Nodes[0].aabb.init();
        for (int i = 0; i < n; i++) {
            FinalIndices[i] = i;
            cx[i] = (prims[i].BBMax.x - prims[i].BBMin.x) / 2.0f + prims[i].BBMin.x;
            cy[i] = (prims[i].BBMax.y - prims[i].BBMin.y) / 2.0f + prims[i].BBMin.y;
            cz[i] = (prims[i].BBMax.z - prims[i].BBMin.z) / 2.0f + prims[i].BBMin.z;
            BVH2Nodes[0].aabb.Extend(prims[i]);
        }
        const float* centers[3] = {cx.data(), cy.data(), cz.data()};
        auto sort_axis = [&](int d) {  // the three per-axis sorts are independent
            int* seg = &DimensionedIndices[(size_t)n * d];
            for (int i = 0; i < n; i++) seg[i] = i;
            DotNetSort s{seg, KeyCmp{centers[d]}};
            s.Sort(n);
        };
        parallel = std::getenv("TT_BUILD_SERIAL") == nullptr;
        const auto ts = std::chrono::steady_clock::now();
        if (parallel && n >= kParMin) {
            std::thread t1(sort_axis, 1), t2(sort_axis, 2);
            sort_axis(0);
            t1.join();
            t2.join();
        } else {
            for (int d = 0; d < 3; d++) sort_axis(d);
        }
        const auto tr = std::chrono::steady_clock::now();
        BuildRecursive(0, 2, 0, n, 0);
        std::memcpy(FinalIndices.data(), DimensionedIndices.data(), sizeof(int) * (size_t)n);
        if (std::getenv("TT_BUILD_TIMES"))
            std::fprintf(stderr, "[build] bvh2 n=%d presort %.3f s, recursive SAH %.3f s\n", n,
                         std::chrono::duration<double>(tr - ts).count(),
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - tr).count());
    }
};

// ---------------------------------------------------------------- BVH8Builder
// CommonVars.BVHNode8Data (CommonVars.cs:159-175), unpacked form.
struct BVHNode8Data {
    uint32_t e[3];
    uint32_t imask;
    uint32_t base_index_child;
    uint32_t base_index_triangle;
    uint8_t meta[8];
    uint8_t quantized_min_x[8], quantized_max_x[8];
    uint8_t quantized_min_y[8], quantized_max_y[8];
    uint8_t quantized_min_z[8], quantized_max_z[8];
    V3 p;
};

// Mathf.* are float wrappers over System.Math (double).
static inline float MathfLog2(float f) { return (float)(std::log((double)f) / std::log(2.0)); }
static inline float MathfCeil(float f) { return (float)std::ceil((double)f); }
static inline float MathfFloor(float f) { return (float)std::floor((double)f); }
static inline float MathfPow(float f, float p) { return (float)std::pow((double)f, (double)p); }
// (byte)(uint)x of a C# float (unchecked): truncate toward zero, wrap to 8 bits.
static inline uint8_t to_byte(float x) {
    if (!(x == x)) return 0;  // NaN: x64 conversion yields 0 after the byte wrap
    if (x <= -1.0f || x >= 4294967296.0f) return 0;
    return (uint8_t)(uint32_t)x;
}
static inline uint32_t asuint(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

struct BVH8Builder {
    struct Decision {
        int Type;  // 0 LEAF, 1 INTERNAL, 2 DISTRIBUTE
        int dist_left;
        int dist_right;
    };
    std::vector<float> cost;
    std::vector<Decision> decisions;
    std::vector<int> cwbvh_indices;
    std::vector<BVHNode8Data> BVH8Nodes;
    int cwbvhindex_count = 0;
    int cwbvhnode_count = 0;
    const BVHNode2Data* nodes = nullptr;
    float cost2[8][8];

    bool parallel = false;  // the cost pass of large trees runs its top subtrees on their own threads
    int calculate_cost(int node_index, uint32_t depth = 0) {
        const BVHNode2Data& node = nodes[node_index];
        int num_primitives;
        if (node.count > 0) {
            num_primitives = (int)node.count;
            if (num_primitives != 1) return -1;
            const float cost_leaf = surface_area(node.aabb) * (float)num_primitives;
            for (int i = 0; i < 7; i++) {
                cost[node_index * 7 + i] = cost_leaf;
                decisions[node_index * 7 + i].Type = 0;
            }
        } else {
            const int l = node.left;
            if (parallel && depth < 4) {  // disjoint subtrees write disjoint cost / decision entries
                int a = 0;
                BigThread t;
                t.start([&] { a = calculate_cost(l, depth + 1); });
                const int b = calculate_cost(l + 1, depth + 1);
                t.join();
                num_primitives = a + b;
            } else {
                num_primitives = calculate_cost(l, depth + 1) + calculate_cost(l + 1, depth + 1);
            }
            {
                const float cost_leaf = num_primitives <= 3 ? (float)num_primitives * surface_area(node.aabb)
                                                            : std::numeric_limits<float>::max();
                float cost_distribute = std::numeric_limits<float>::max();
                int dist_left = -1, dist_right = -1;
                for (int k = 0; k < 7; k++) {
                    const float c = cost[node.left * 7 + k] + cost[(node.left + 1) * 7 + 6 - k];
                    if (c < cost_distribute) {
                        cost_distribute = c;
                        dist_left = k;
                        dist_right = 6 - k;
                    }
                }
                const float cost_internal = cost_distribute + surface_area(node.aabb);
                if (cost_leaf < cost_internal) {
                    cost[node_index * 7] = cost_leaf;
                    decisions[node_index * 7].Type = 0;
                } else {
                    cost[node_index * 7] = cost_internal;
                    decisions[node_index * 7].Type = 1;
                }
                decisions[node_index * 7].dist_left = dist_left;
                decisions[node_index * 7].dist_right = dist_right;
            }
            for (int i = 1; i < 7; i++) {
                float cost_distribute = cost[node_index * 7 + i - 1];
                int dist_left = -1, dist_right = -1;
                for (int k = 0; k < i; k++) {
                    const float c = cost[node.left * 7 + k] + cost[(node.left + 1) * 7 + i - k - 1];
                    if (c < cost_distribute) {
                        cost_distribute = c;
                        dist_left = k;
                        dist_right = i - k - 1;
                    }
                }
                cost[node_index * 7 + i] = cost_distribute;
                if (dist_left != -1) {
                    decisions[node_index * 7 + i].Type = 2;
                    decisions[node_index * 7 + i].dist_left = dist_left;
                    decisions[node_index * 7 + i].dist_right = dist_right;
                } else {
                    decisions[node_index * 7 + i] = decisions[node_index * 7 + i - 1];
                }
            }
        }
        return num_primitives;
    }

    bool get_children(int node_index, int i, int& child_count, int* children) {
        if (nodes[node_index].count > 0) {
            if (child_count >= 8) return false;
            children[child_count++] = node_index;
            return true;
        }
        const int dist_left = decisions[node_index * 7 + i].dist_left;
        const int dist_right = decisions[node_index * 7 + i].dist_right;
        if (!(dist_left >= 0 && dist_left < 7) || !(dist_right >= 0 && dist_right < 7)) return false;
        if (child_count >= 8) return false;
        const int l = nodes[node_index].left;
        if (decisions[l * 7 + dist_left].Type == 2) {
            if (!get_children(l, dist_left, child_count, children)) return false;
        } else {
            if (child_count >= 8) return false;
            children[child_count++] = l;
        }
        if (decisions[(l + 1) * 7 + dist_right].Type == 2) {
            if (!get_children(l + 1, dist_right, child_count, children)) return false;
        } else {
            if (child_count >= 8) return false;
            children[child_count++] = l + 1;
        }
        return true;
    }

    void order_children(int node_index, int* children, int child_count) {
        const V3 p = (nodes[node_index].aabb.BBMax + nodes[node_index].aabb.BBMin) / 2.0f;
        for (int c = 0; c < child_count; c++) {
            for (int s = 0; s < 8; s++) {
                const V3 direction = v3((((s >> 2) & 1) == 1) ? -1.0f : 1.0f, (((s >> 1) & 1) == 1) ? -1.0f : 1.0f,
                                        (((s >> 0) & 1) == 1) ? -1.0f : 1.0f);
                const AABB& ca = nodes[children[c]].aabb;
                cost2[c][s] = dotv((ca.BBMax + ca.BBMin) / 2.0f - p, direction);
            }
        }
        int assignment[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
        bool slot_filled[8] = {false, false, false, false, false, false, false, false};
        while (true) {
            float min_cost = std::numeric_limits<float>::max();
            int min_slot = -1, min_index = -1;
            for (int c = 0; c < child_count; c++) {
                if (assignment[c] == -1) {
                    for (int s = 0; s < 8; s++) {
                        if (!slot_filled[s] && cost2[c][s] < min_cost) {
                            min_cost = cost2[c][s];
                            min_slot = s;
                            min_index = c;
                        }
                    }
                }
            }
            if (min_slot == -1) break;
            slot_filled[min_slot] = true;
            assignment[min_index] = min_slot;
        }
        int children_copy[8];
        std::memcpy(children_copy, children, sizeof(children_copy));
        for (int i = 0; i < 8; i++) children[i] = -1;
        for (int i = 0; i < child_count; i++) children[assignment[i]] = children_copy[i];
    }

    int count_primitives(int node_index, const int* indices) {
        if (nodes[node_index].count > 0) {
            for (uint32_t i = 0; i < nodes[node_index].count; i++)
                cwbvh_indices[cwbvhindex_count++] = indices[nodes[node_index].left + (int)i];
            return (int)nodes[node_index].count;
        }
        return count_primitives(nodes[node_index].left, indices) +
               count_primitives(nodes[node_index].left + 1, indices);
    }

    bool collapse(const int* indices_bvh, int node_index_cwbvh, int node_index_bvh) {
        BVHNode8Data node = BVH8Nodes[node_index_cwbvh];
        const AABB aabb = nodes[node_index_bvh].aabb;
        node.p = aabb.BBMin;
        const int Nq = 8;
        const float denom = 1.0f / (float)((1 << Nq) - 1);
        V3 e = v3(MathfPow(2, MathfCeil(MathfLog2((aabb.BBMax.x - aabb.BBMin.x) * denom))),
                  MathfPow(2, MathfCeil(MathfLog2((aabb.BBMax.y - aabb.BBMin.y) * denom))),
                  MathfPow(2, MathfCeil(MathfLog2((aabb.BBMax.z - aabb.BBMin.z) * denom))));
        const V3 one_over_e = v3(1.0f / e.x, 1.0f / e.y, 1.0f / e.z);
        const uint32_t u_ex = asuint(e.x), u_ey = asuint(e.y), u_ez = asuint(e.z);
        if ((u_ex & 0x807FFFFFu) || (u_ey & 0x807FFFFFu) || (u_ez & 0x807FFFFFu)) return false;
        node.e[0] = u_ex >> 23;
        node.e[1] = u_ey >> 23;
        node.e[2] = u_ez >> 23;
        int child_count = 0;
        int children[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
        if (!get_children(node_index_bvh, 0, child_count, children)) return false;
        order_children(node_index_bvh, children, child_count);
        node.imask = 0;
        node.base_index_child = (uint32_t)cwbvhnode_count;
        node.base_index_triangle = (uint32_t)cwbvhindex_count;
        int node_internal_count = 0, node_triangle_count = 0;
        for (int i = 0; i < 8; i++) {
            const int child_index = children[i];
            if (child_index == -1) continue;
            const AABB& ca = nodes[child_index].aabb;
            node.quantized_min_x[i] = to_byte(MathfFloor((ca.BBMin.x - node.p.x) * one_over_e.x));
            node.quantized_min_y[i] = to_byte(MathfFloor((ca.BBMin.y - node.p.y) * one_over_e.y));
            node.quantized_min_z[i] = to_byte(MathfFloor((ca.BBMin.z - node.p.z) * one_over_e.z));
            node.quantized_max_x[i] = to_byte(MathfCeil((ca.BBMax.x - node.p.x) * one_over_e.x));
            node.quantized_max_y[i] = to_byte(MathfCeil((ca.BBMax.y - node.p.y) * one_over_e.y));
            node.quantized_max_z[i] = to_byte(MathfCeil((ca.BBMax.z - node.p.z) * one_over_e.z));
            switch (decisions[child_index * 7].Type) {
                case 0: {
                    const int triangle_count = count_primitives(child_index, indices_bvh);
                    if (!(triangle_count > 0 && triangle_count <= 3)) return false;
                    for (int j = 0; j < triangle_count; j++) node.meta[i] |= (uint8_t)(1 << (j + 5));
                    node.meta[i] |= (uint8_t)node_triangle_count;
                    node_triangle_count += triangle_count;
                    if (node_triangle_count > 24) return false;
                    break;
                }
                case 1: {
                    node.meta[i] = (uint8_t)((node_internal_count + 24) | 0x20);
                    node.imask |= (uint32_t)(uint8_t)(1 << node_internal_count);
                    cwbvhnode_count++;
                    node_internal_count++;
                    break;
                }
                default:
                    return false;
            }
        }
        BVH8Nodes[node_index_cwbvh] = node;
        for (int i = 0; i < 8; i++) {
            const int child_index = children[i];
            if (child_index == -1) continue;
            if (decisions[child_index * 7].Type == 1) {
                if (!collapse(indices_bvh, (int)node.base_index_child + (node.meta[i] & 31) - 24, child_index))
                    return false;
            }
        }
        return true;
    }

    bool build(const BVH2Builder& bvh2) {
        const size_t n2 = bvh2.BVH2Nodes.size();
        cost.assign(n2 * 7, 0.0f);
        decisions.assign(n2 * 7, Decision{0, 0, 0});
        BVHNode8Data zero;
        std::memset(&zero, 0, sizeof(zero));
        BVH8Nodes.assign(n2, zero);
        cwbvh_indices.assign(bvh2.FinalIndices.size(), 0);
        std::memset(cost2, 0, sizeof(cost2));
        nodes = bvh2.BVH2Nodes.data();
        cwbvhindex_count = 0;
        cwbvhnode_count = 1;
        parallel = bvh2.parallel && bvh2.PrimCount >= (1 << 16);
        if (calculate_cost(0) < 0) return false;
        if (!collapse(bvh2.FinalIndices.data(), 0, 0)) return false;
        BVH8Nodes.resize((size_t)cwbvhnode_count);
        return true;
    }
};

// CommonFunctions.Aggregate — CommonVars.cs:662-688
static void Aggregate(const std::vector<BVHNode8Data>& in, tt_cwbvh_node* out) {
    auto pack4 = [](const uint8_t* b) -> uint32_t {
        return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    };
    for (size_t i = 0; i < in.size(); i++) {
        const BVHNode8Data& n = in[i];
        tt_cwbvh_node& o = out[i];
        o.p[0] = n.p.x;
        o.p[1] = n.p.y;
        o.p[2] = n.p.z;
        o.e_imask = n.e[0] | (n.e[1] << 8) | (n.e[2] << 16) | (n.imask << 24);
        o.base_child = n.base_index_child;
        o.base_tri = n.base_index_triangle;
        o.meta[0] = pack4(n.meta);
        o.meta[1] = pack4(n.meta + 4);
        o.qlo_x[0] = pack4(n.quantized_min_x);
        o.qlo_x[1] = pack4(n.quantized_min_x + 4);
        o.qhi_x[0] = pack4(n.quantized_max_x);
        o.qhi_x[1] = pack4(n.quantized_max_x + 4);
        o.qlo_y[0] = pack4(n.quantized_min_y);
        o.qlo_y[1] = pack4(n.quantized_min_y + 4);
        o.qhi_y[0] = pack4(n.quantized_max_y);
        o.qhi_y[1] = pack4(n.quantized_max_y + 4);
        o.qlo_z[0] = pack4(n.quantized_min_z);
        o.qlo_z[1] = pack4(n.quantized_min_z + 4);
        o.qhi_z[0] = pack4(n.quantized_max_z);
        o.qhi_z[1] = pack4(n.quantized_max_z + 4);
    }
}

// Vector3.normalized (UnityEngine): mag = (float)Math.Sqrt(x*x+y*y+z*z); > 1e-5 ? v/mag : 0
static inline V3 normalized(V3 v) {
    const float mag = (float)std::sqrt((double)(v.x * v.x + v.y * v.y + v.z * v.z));
    if (mag > 1e-5f) return v / mag;
    return v3(0, 0, 0);
}

// Run fn on a thread with a large stack (the C# builders recurse to BVH2 depth).
template <class F>
static bool run_big_stack(F&& fn) {
    struct Box {
        F* f;
    } box{&fn};
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, (size_t)1 << 30);
    pthread_t th;
    auto tramp = [](void* p) -> void* {
        (*static_cast<Box*>(p)->f)();
        return nullptr;
    };
    if (pthread_create(&th, &attr, tramp, &box) != 0) {
        pthread_attr_destroy(&attr);
        fn();
        return true;
    }
    pthread_join(th, nullptr);
    pthread_attr_destroy(&attr);
    return true;
}

}  // namespace

struct tt_blas {
    std::vector<tt_cwbvh_node> nodes;
    std::vector<tt_cuda_triangle> tris;
    std::vector<int32_t> leaf_of;  // CWBVHIndicesBufferInverted
    AABB aabb_untransformed;
    uint32_t bvh2_depth = 0;
    double seconds = 0;
};

struct tt_scene_build {
    std::vector<tt_cwbvh_node> nodes;
    std::vector<tt_cuda_triangle> tris;
    std::vector<int32_t> tlas_indices;
    std::vector<tt_mesh_data> meshdata;
    std::vector<float> mesh_aabbs;  // MeshAABBs, n_mesh x {BBMax, BBMin}
    uint32_t tlas_nodes = 0;
};

extern "C" {

uint32_t tt_pack_octahedral(float x, float y, float z) {
    // CommonFunctions.PackOctahedral — CommonVars.cs:816-833
    const float halfMaxUInt16 = 32767.5f;
    const float sx = (x >= 0.0f) ? 1.0f : -1.0f, sy = (y >= 0.0f) ? 1.0f : -1.0f;
    const float absX = x * sx, absY = y * sy;
    const float Tot = absX + absY + std::fabs(z);
    float tx = absX / Tot, ty = absY / Tot;
    if (z < 0.0f) {
        const float ox = tx;
        tx = 1.0f - ty;
        ty = 1.0f - ox;
    }
    const float fx = halfMaxUInt16 + tx * halfMaxUInt16 * sx;
    const float fy = halfMaxUInt16 + ty * halfMaxUInt16 * sy;
    const uint32_t ux = (fx == fx && fx > 0.0f) ? (uint32_t)fx : 0u;
    const uint32_t uy = (fy == fy && fy > 0.0f) ? (uint32_t)fy : 0u;
    return ux | (uy << 16);
}

void tt_dotnet_sort_by_key(int32_t* items, uint32_t n, const float* keys) {
    DotNetSort s{items, KeyCmp{keys}};
    s.Sort((int)n);
}

tt_status tt_bvh2_build(const float* aabbs, uint32_t n, int32_t* final_indices, float* node_aabbs,
                        int32_t* node_left, uint32_t* node_count) {
    if (!aabbs || !n || !final_indices) return TT_ERR_INVALID_ARG;
    std::vector<AABB> prims(n);
    for (uint32_t i = 0; i < n; i++) {
        prims[i].BBMax = v3(aabbs[6 * i + 0], aabbs[6 * i + 1], aabbs[6 * i + 2]);
        prims[i].BBMin = v3(aabbs[6 * i + 3], aabbs[6 * i + 4], aabbs[6 * i + 5]);
    }
    BVH2Builder b;
    run_big_stack([&] { b.build(prims.data(), (int)n); });
    std::memcpy(final_indices, b.FinalIndices.data(), sizeof(int) * n);
    for (size_t i = 0; i < b.BVH2Nodes.size(); i++) {
        const BVHNode2Data& nd = b.BVH2Nodes[i];
        if (node_aabbs) {
            float* o = node_aabbs + 6 * i;
            o[0] = nd.aabb.BBMax.x; o[1] = nd.aabb.BBMax.y; o[2] = nd.aabb.BBMax.z;
            o[3] = nd.aabb.BBMin.x; o[4] = nd.aabb.BBMin.y; o[5] = nd.aabb.BBMin.z;
        }
        if (node_left) node_left[i] = nd.left;
        if (node_count) node_count[i] = nd.count;
    }
    return TT_OK;
}

// ParentObject.BuildTotal (ParentObject.cs:973-1111) for one merged child with identity
// child->parent transform (TransMat = I, Ofst = Ofst2 = 0): the AggTriangles and the triangle AABBs
// the builders consume. Triangles are independent: large meshes are prepared on several threads.
namespace {
struct BlasPrep {
    std::vector<tt_cuda_triangle> agg;
    std::vector<AABB> Triangles;
    AABB aabb_untransformed;
};
tt_status blas_prepare(const tt_mesh_input* m, BlasPrep& P) {
    if (!m || !m->positions || !m->indices || m->n_indices < 3 || m->n_indices % 3) return TT_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < m->n_indices; i++)
        if (m->indices[i] < 0 || (uint32_t)m->indices[i] >= m->n_vertices) return TT_ERR_INVALID_ARG;
    const uint32_t ntri = m->n_indices / 3;
    const V3 ParentScale = v3(0.001f / m->lossy_scale[0], 0.001f / m->lossy_scale[1], 0.001f / m->lossy_scale[2]);
    P.agg.assign(ntri, tt_cuda_triangle{});
    P.Triangles.resize(ntri);
    auto P3 = [&](int i) { return v3(m->positions[3 * i], m->positions[3 * i + 1], m->positions[3 * i + 2]); };
    auto N = [&](int i) { return m->normals ? v3(m->normals[3 * i], m->normals[3 * i + 1], m->normals[3 * i + 2]) : v3(0, 1, 0); };
    auto T = [&](int i) { return m->tangents ? v3(m->tangents[4 * i], m->tangents[4 * i + 1], m->tangents[4 * i + 2]) : v3(1, 0, 0); };
    auto range = [&](uint32_t t0, uint32_t t1) {
        for (uint32_t t = t0; t < t1; t++) {
            const int Index1 = m->indices[3 * t], Index2 = m->indices[3 * t + 2], Index3 = m->indices[3 * t + 1];
            const V3 V1 = P3(Index1), V2 = P3(Index2), V3_ = P3(Index3);
            tt_cuda_triangle& tri = P.agg[t];
            std::memset(&tri, 0, sizeof(tri));
            for (int k = 0; k < 2; k++) {
                tri.tex0[k] = m->uvs ? m->uvs[2 * Index1 + k] : 0.0f;
                tri.texedge1[k] = m->uvs ? m->uvs[2 * Index2 + k] : 0.0f;
                tri.texedge2[k] = m->uvs ? m->uvs[2 * Index3 + k] : 0.0f;
            }
            const V3 e1 = V2 - V1, e2 = V3_ - V1;
            tri.pos0[0] = V1.x; tri.pos0[1] = V1.y; tri.pos0[2] = V1.z;
            tri.posedge1[0] = e1.x; tri.posedge1[1] = e1.y; tri.posedge1[2] = e1.z;
            tri.posedge2[0] = e2.x; tri.posedge2[1] = e2.y; tri.posedge2[2] = e2.z;
            const int idx[3] = {Index1, Index2, Index3};
            for (int k = 0; k < 3; k++) {
                const V3 n = normalized(N(idx[k]));
                tri.norms[k] = tt_pack_octahedral(n.x, n.y, n.z);
                const V3 tg = normalized(T(idx[k]));
                tri.tans[k] = tt_pack_octahedral(tg.x, tg.y, tg.z);
            }
            tri.MatDat = m->matdat ? (uint32_t)m->matdat[t] : 0u;
            P.Triangles[t].Create(V1, V2);
            P.Triangles[t].Extend(V3_);
            P.Triangles[t].Validate(ParentScale);
        }
    };
    const uint32_t nth = (ntri >= (1u << 16) && std::getenv("TT_BUILD_SERIAL") == nullptr)
                             ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
    if (nth > 1) {
        std::vector<std::thread> th;
        for (uint32_t k = 1; k < nth; k++)
            th.emplace_back(range, (uint32_t)((uint64_t)ntri * k / nth), (uint32_t)((uint64_t)ntri * (k + 1) / nth));
        range(0, (uint32_t)((uint64_t)ntri / nth));
        for (auto& t : th) t.join();
    } else {
        range(0, ntri);
    }
    // ConstructAABB (:1143-1149)
    P.aabb_untransformed.init();
    for (uint32_t t = 0; t < ntri; t++) P.aabb_untransformed.Extend(P.Triangles[t]);
    return TT_OK;
}

// Construct's BVH8 stage (:679-742), the cwbvh_indices permutation (:1084-1090) and Aggregate
// (:1091-1092) over a finished BVH2.
tt_status blas_finish(BlasPrep& P, BVH2Builder& bvh2, tt_blas* b) {
    const uint32_t ntri = (uint32_t)P.agg.size();
    bool ok = false;
    BVH8Builder bvh8;
    double t_bvh8 = 0.0;
    run_big_stack([&] {
        const auto t8 = std::chrono::steady_clock::now();
        ok = bvh8.build(bvh2);
        t_bvh8 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t8).count();
    });
    if (std::getenv("TT_BUILD_TIMES")) std::fprintf(stderr, "[build] blas n=%u bvh8 %.3f s\n", ntri, t_bvh8);
    if (!ok) return TT_ERR_UNSUPPORTED;
    b->aabb_untransformed = P.aabb_untransformed;
    b->bvh2_depth = bvh2.max_depth;
    b->tris.resize(ntri);
    b->leaf_of.assign(ntri, 0);
    for (uint32_t i = 0; i < ntri; i++) {
        b->tris[i] = P.agg[bvh8.cwbvh_indices[i]];
        b->leaf_of[bvh8.cwbvh_indices[i]] = (int32_t)i;
    }
    b->nodes.resize(bvh8.BVH8Nodes.size());
    Aggregate(bvh8.BVH8Nodes, b->nodes.data());
    return TT_OK;
}
}  // namespace

tt_status tt_blas_build(const tt_mesh_input* m, tt_blas** out) {
    if (!out) return TT_ERR_INVALID_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    BlasPrep P;
    tt_status st = blas_prepare(m, P);
    if (st != TT_OK) return st;
    if (std::getenv("TT_BUILD_TIMES"))
        std::fprintf(stderr, "[build] blas n=%zu triangles+boxes %.3f s\n", P.agg.size(),
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    tt_blas* b = new (std::nothrow) tt_blas();
    if (!b) return TT_ERR_OOM;
    BVH2Builder bvh2;
    run_big_stack([&] { bvh2.build(P.Triangles.data(), (int)P.Triangles.size()); });
    st = blas_finish(P, bvh2, b);
    if (st != TT_OK) {
        delete b;
        return st;
    }
    b->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = b;
    return TT_OK;
}

extern "C++" {
namespace {
// splits [0, n) over up to 16 threads for large n (independent iterations)
template <class F>
void parallel_range(uint32_t n, F&& f) {
    const uint32_t nth = (n >= (1u << 16) && std::getenv("TT_BUILD_SERIAL") == nullptr)
                             ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
    if (nth == 1) {
        f(0u, n);
        return;
    }
    std::vector<std::thread> th;
    for (uint32_t k = 1; k < nth; k++)
        th.emplace_back(f, (uint32_t)((uint64_t)n * k / nth), (uint32_t)((uint64_t)n * (k + 1) / nth));
    f(0u, (uint32_t)((uint64_t)n / nth));
    for (auto& t : th) t.join();
}
void write_aabbs(const BlasPrep& P, float* aabbs) {
    parallel_range((uint32_t)P.Triangles.size(), [&](uint32_t t0, uint32_t t1) {
        for (uint32_t t = t0; t < t1; t++) {
            const AABB& a = P.Triangles[t];
            float* o = aabbs + 6 * (size_t)t;
            o[0] = a.BBMax.x; o[1] = a.BBMax.y; o[2] = a.BBMax.z;
            o[3] = a.BBMin.x; o[4] = a.BBMin.y; o[5] = a.BBMin.z;
        }
    });
}
}  // namespace
}  // extern "C++"

struct tt_blas_prep {
    BlasPrep P;
};

tt_status tt_blas_prepare_aabbs(const tt_mesh_input* m, float* aabbs) {
    if (!aabbs) return TT_ERR_INVALID_ARG;
    BlasPrep P;
    const tt_status st = blas_prepare(m, P);
    if (st != TT_OK) return st;
    write_aabbs(P, aabbs);
    return TT_OK;
}

tt_status tt_blas_prepare(const tt_mesh_input* m, float* aabbs, tt_blas_prep** out) {
    if (!aabbs || !out) return TT_ERR_INVALID_ARG;
    tt_blas_prep* p = new (std::nothrow) tt_blas_prep();
    if (!p) return TT_ERR_OOM;
    const tt_status st = blas_prepare(m, p->P);
    if (st != TT_OK) {
        delete p;
        return st;
    }
    write_aabbs(p->P, aabbs);
    *out = p;
    return TT_OK;
}

void tt_blas_prep_free(tt_blas_prep* p) { delete p; }

tt_status tt_bvh2_presort(const float* aabbs, uint32_t n, int32_t* presorted) {
    if (!aabbs || !n || !presorted) return TT_ERR_INVALID_ARG;
    std::vector<float> c[3];
    for (int d = 0; d < 3; d++) c[d].resize(n);
    for (uint32_t i = 0; i < n; i++) {  // BVH2Builder's centroid: (max - min) / 2 + min
        const float* a = aabbs + 6 * (size_t)i;
        for (int d = 0; d < 3; d++) c[d][i] = (a[d] - a[3 + d]) / 2.0f + a[3 + d];
    }
    auto sort_axis = [&](int d) {
        int32_t* seg = presorted + (size_t)n * d;
        for (uint32_t i = 0; i < n; i++) seg[i] = (int32_t)i;
        DotNetSort s{seg, KeyCmp{c[d].data()}};
        s.Sort((int)n);
    };
    if (n >= (1u << 16) && std::getenv("TT_BUILD_SERIAL") == nullptr) {
        std::thread t1(sort_axis, 1), t2(sort_axis, 2);
        sort_axis(0);
        t1.join();
        t2.join();
    } else {
        for (int d = 0; d < 3; d++) sort_axis(d);
    }
    return TT_OK;
}

tt_status tt_blas_build_from_bvh2(const tt_mesh_input* m, const int32_t* final_indices, const float* node_aabbs,
                                  const int32_t* node_left, const uint32_t* node_count, uint32_t max_depth,
                                  tt_blas** out) {
    if (!out || !final_indices || !node_aabbs || !node_left || !node_count) return TT_ERR_INVALID_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    BlasPrep P;
    tt_status st = blas_prepare(m, P);
    if (st != TT_OK) return st;
    const uint32_t n = (uint32_t)P.Triangles.size();
    BVH2Builder bvh2;
    bvh2.PrimCount = (int)n;
    bvh2.parallel = std::getenv("TT_BUILD_SERIAL") == nullptr;
    bvh2.max_depth = max_depth;
    bvh2.FinalIndices.assign(final_indices, final_indices + n);
    bvh2.BVH2Nodes.resize(2 * (size_t)n);
    for (size_t i = 0; i < 2 * (size_t)n; i++) {
        const float* a = node_aabbs + 6 * i;
        BVHNode2Data& nd = bvh2.BVH2Nodes[i];
        nd.aabb.BBMax = v3(a[0], a[1], a[2]);
        nd.aabb.BBMin = v3(a[3], a[4], a[5]);
        nd.left = node_left[i];
        nd.count = node_count[i];
    }
    {  // structure check: a binary tree over the n positions (children after their parent), a permutation
        std::vector<char> seen(n, 0);
        std::vector<int> stack{0};
        uint32_t leaves = 0;
        while (!stack.empty()) {
            const int i = stack.back();
            stack.pop_back();
            const BVHNode2Data& nd = bvh2.BVH2Nodes[(size_t)i];
            if (nd.count == 1) {
                if (nd.left < 0 || (uint32_t)nd.left >= n || seen[(size_t)nd.left]) return TT_ERR_INVALID_ARG;
                seen[(size_t)nd.left] = 1;
                leaves++;
            } else if (nd.count == 0) {
                if (nd.left <= i || (size_t)nd.left + 1 >= 2 * (size_t)n) return TT_ERR_INVALID_ARG;
                stack.push_back(nd.left);
                stack.push_back(nd.left + 1);
            } else {
                return TT_ERR_INVALID_ARG;
            }
        }
        if (leaves != n) return TT_ERR_INVALID_ARG;
        std::fill(seen.begin(), seen.end(), 0);
        for (uint32_t k = 0; k < n; k++) {
            if (final_indices[k] < 0 || (uint32_t)final_indices[k] >= n || seen[(size_t)final_indices[k]])
                return TT_ERR_INVALID_ARG;
            seen[(size_t)final_indices[k]] = 1;
        }
    }
    tt_blas* b = new (std::nothrow) tt_blas();
    if (!b) return TT_ERR_OOM;
    st = blas_finish(P, bvh2, b);
    if (st != TT_OK) {
        delete b;
        return st;
    }
    b->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = b;
    return TT_OK;
}

namespace {
tt_status blas_from_cwbvh(const BlasPrep& P, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                          const int32_t* cwbvh_indices, uint32_t bvh2_depth, tt_blas** out,
                          std::chrono::steady_clock::time_point t0) {
    const uint32_t ntri = (uint32_t)P.agg.size();
    std::vector<char> seen(ntri, 0);
    for (uint32_t i = 0; i < ntri; i++) {  // a permutation of the triangles (sequential: duplicate check)
        const int32_t k = cwbvh_indices[i];
        if (k < 0 || (uint32_t)k >= ntri || seen[(size_t)k]) return TT_ERR_INVALID_ARG;
        seen[(size_t)k] = 1;
    }
    tt_blas* b = new (std::nothrow) tt_blas();
    if (!b) return TT_ERR_OOM;
    b->aabb_untransformed = P.aabb_untransformed;
    b->bvh2_depth = bvh2_depth;
    b->tris.resize(ntri);
    b->leaf_of.assign(ntri, 0);
    parallel_range(ntri, [&](uint32_t i0, uint32_t i1) {  // disjoint writes: cwbvh_indices is a permutation
        for (uint32_t i = i0; i < i1; i++) {
            b->tris[i] = P.agg[(size_t)cwbvh_indices[i]];
            b->leaf_of[(size_t)cwbvh_indices[i]] = (int32_t)i;
        }
    });
    b->nodes.assign(nodes, nodes + n_nodes);
    b->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = b;
    return TT_OK;
}
}  // namespace

tt_status tt_blas_build_from_cwbvh(const tt_mesh_input* m, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                                   const int32_t* cwbvh_indices, uint32_t bvh2_depth, tt_blas** out) {
    if (!out || !nodes || !n_nodes || !cwbvh_indices) return TT_ERR_INVALID_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    BlasPrep P;
    tt_status st = blas_prepare(m, P);
    if (st != TT_OK) return st;
    return blas_from_cwbvh(P, nodes, n_nodes, cwbvh_indices, bvh2_depth, out, t0);
}

tt_status tt_blas_build_from_cwbvh_prepared(tt_blas_prep* prep, const tt_cwbvh_node* nodes, uint32_t n_nodes,
                                            const int32_t* cwbvh_indices, uint32_t bvh2_depth, tt_blas** out) {
    if (!prep) return TT_ERR_INVALID_ARG;
    tt_status st = TT_ERR_INVALID_ARG;
    if (out && nodes && n_nodes && cwbvh_indices)
        st = blas_from_cwbvh(prep->P, nodes, n_nodes, cwbvh_indices, bvh2_depth, out, std::chrono::steady_clock::now());
    delete prep;
    return st;
}

tt_status tt_blas_copy_leaf_order(const tt_blas* b, int32_t* out) {
    if (!b || !out) return TT_ERR_INVALID_ARG;
    std::copy(b->leaf_of.begin(), b->leaf_of.end(), out);
    return TT_OK;
}

tt_status tt_blas_get_info(const tt_blas* b, tt_blas_info* info) {
    if (!b || !info) return TT_ERR_INVALID_ARG;
    info->n_nodes = (uint32_t)b->nodes.size();
    info->n_tris = (uint32_t)b->tris.size();
    info->bvh2_depth = b->bvh2_depth;
    info->aabb_min[0] = b->aabb_untransformed.BBMin.x;
    info->aabb_min[1] = b->aabb_untransformed.BBMin.y;
    info->aabb_min[2] = b->aabb_untransformed.BBMin.z;
    info->aabb_max[0] = b->aabb_untransformed.BBMax.x;
    info->aabb_max[1] = b->aabb_untransformed.BBMax.y;
    info->aabb_max[2] = b->aabb_untransformed.BBMax.z;
    info->build_seconds = b->seconds;
    return TT_OK;
}

tt_status tt_blas_copy(const tt_blas* b, tt_cwbvh_node* nodes, tt_cuda_triangle* tris) {
    if (!b) return TT_ERR_INVALID_ARG;
    if (nodes) std::memcpy(nodes, b->nodes.data(), b->nodes.size() * sizeof(tt_cwbvh_node));
    if (tris) std::memcpy(tris, b->tris.data(), b->tris.size() * sizeof(tt_cuda_triangle));
    return TT_OK;
}

void tt_blas_free(tt_blas* b) { delete b; }

// ParentObject.UpdateAABB / AssetManager.CreateAABB with CommonFunctions.transform_position /
// transform_direction (CommonVars.cs:775-790): world AABB from center/extent.
static AABB transformed_aabb(const AABB& a, const float* l2w) {
    auto Mx = [&](int r, int c) { return l2w[c * 4 + r]; };
    const V3 center = 0.5f * (a.BBMin + a.BBMax);
    const V3 extent = 0.5f * (a.BBMax - a.BBMin);
    V3 nc, ne;
    nc.x = Mx(0, 0) * center.x + Mx(0, 1) * center.y + Mx(0, 2) * center.z + Mx(0, 3);
    nc.y = Mx(1, 0) * center.x + Mx(1, 1) * center.y + Mx(1, 2) * center.z + Mx(1, 3);
    nc.z = Mx(2, 0) * center.x + Mx(2, 1) * center.y + Mx(2, 2) * center.z + Mx(2, 3);
    ne.x = std::fabs(Mx(0, 0)) * extent.x + std::fabs(Mx(0, 1)) * extent.y + std::fabs(Mx(0, 2)) * extent.z;
    ne.y = std::fabs(Mx(1, 0)) * extent.x + std::fabs(Mx(1, 1)) * extent.y + std::fabs(Mx(1, 2)) * extent.z;
    ne.z = std::fabs(Mx(2, 0)) * extent.x + std::fabs(Mx(2, 1)) * extent.y + std::fabs(Mx(2, 2)) * extent.z;
    AABB o;
    o.BBMin = nc - ne;
    o.BBMax = nc + ne;
    return o;
}

tt_status tt_scene_assemble(const tt_parent_desc* parents, uint32_t n_parents,
                            const tt_parent_desc* iparents, uint32_t n_iparents,
                            const tt_instance_desc* instances, uint32_t n_instances,
                            tt_scene_build** out) {
    if (!out || (n_parents && !parents) || (n_iparents && !iparents) || (n_instances && !instances))
        return TT_ERR_INVALID_ARG;
    const uint32_t n_mesh = n_parents + n_instances;
    if (n_mesh == 0) return TT_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < n_parents; i++) if (!parents[i].blas) return TT_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < n_iparents; i++) if (!iparents[i].blas) return TT_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < n_instances; i++) if (instances[i].instance_parent >= n_iparents) return TT_ERR_INVALID_ARG;
    tt_scene_build* s = new (std::nothrow) tt_scene_build();
    if (!s) return TT_ERR_OOM;

    // AccumulateData (AssetManager.cs:994-1185): TLAS slots 2*(P+I), then parents, then
    // instance parents, node and triangle buffers concatenated in that order.
    uint64_t node_total = 2ull * n_mesh, tri_total = 0;
    for (uint32_t i = 0; i < n_parents; i++) { node_total += parents[i].blas->nodes.size(); tri_total += parents[i].blas->tris.size(); }
    for (uint32_t i = 0; i < n_iparents; i++) { node_total += iparents[i].blas->nodes.size(); tri_total += iparents[i].blas->tris.size(); }
    if (node_total > 0x7fffffffull || tri_total > 0x7fffffffull) { delete s; return TT_ERR_UNSUPPORTED; }
    tt_cwbvh_node zero_node;
    std::memset(&zero_node, 0, sizeof(zero_node));
    s->nodes.assign((size_t)node_total, zero_node);
    s->tris.resize((size_t)tri_total);

    // UpdateTLAS (:1655-1750): MyMeshDataCompacted per parent, per instance.
    std::vector<AABB> MeshAABBs(n_mesh);
    int32_t aggregated_bvh_node_count = (int32_t)(2 * n_mesh);
    int32_t AggTriCount = 0, MatOffset = 0;
    s->meshdata.resize(n_mesh);
    auto place = [&](const tt_blas* b) {
        std::memcpy(&s->nodes[(size_t)aggregated_bvh_node_count], b->nodes.data(), b->nodes.size() * sizeof(tt_cwbvh_node));
        std::memcpy(&s->tris[(size_t)AggTriCount], b->tris.data(), b->tris.size() * sizeof(tt_cuda_triangle));
    };
    for (uint32_t i = 0; i < n_parents; i++) {
        const tt_blas* b = parents[i].blas;
        place(b);
        tt_mesh_data& md = s->meshdata[i];
        std::memset(&md, 0, sizeof(md));
        std::memcpy(md.W2L, parents[i].world_to_local, sizeof(md.W2L));
        md.TriOffset = AggTriCount;
        md.NodeOffset = aggregated_bvh_node_count;
        md.MaterialOffset = MatOffset;
        md.mesh_data_bvh_offsets = aggregated_bvh_node_count;
        MatOffset += (int32_t)parents[i].material_count;
        MeshAABBs[i] = transformed_aabb(b->aabb_untransformed, parents[i].local_to_world);
        aggregated_bvh_node_count += (int32_t)b->nodes.size();
        AggTriCount += (int32_t)b->tris.size();
    }
    struct Agg { int32_t tri, node, mat, root; };
    std::vector<Agg> aggs(n_iparents);
    for (uint32_t i = 0; i < n_iparents; i++) {
        const tt_blas* b = iparents[i].blas;
        place(b);
        aggs[i] = Agg{AggTriCount, aggregated_bvh_node_count, MatOffset, aggregated_bvh_node_count};
        MatOffset += (int32_t)iparents[i].material_count;
        aggregated_bvh_node_count += (int32_t)b->nodes.size();
        AggTriCount += (int32_t)b->tris.size();
    }
    for (uint32_t i = 0; i < n_instances; i++) {
        const Agg& a = aggs[instances[i].instance_parent];
        tt_mesh_data& md = s->meshdata[n_parents + i];
        std::memset(&md, 0, sizeof(md));
        std::memcpy(md.W2L, instances[i].world_to_local, sizeof(md.W2L));
        md.TriOffset = a.tri;
        md.NodeOffset = a.node;
        md.MaterialOffset = a.mat;
        md.mesh_data_bvh_offsets = a.root;
        MeshAABBs[n_parents + i] = transformed_aabb(iparents[instances[i].instance_parent].blas->aabb_untransformed,
                                                    instances[i].local_to_world);
    }

    // ConstructNewTLAS (:1350-1356, :1411-1412): BVH2 over mesh AABBs, BVH8, Aggregate.
    bool ok = false;
    BVH2Builder bvh2;
    BVH8Builder bvh8;
    run_big_stack([&] {
        bvh2.build(MeshAABBs.data(), (int)n_mesh);
        ok = bvh8.build(bvh2);
    });
    if (!ok || bvh8.BVH8Nodes.size() > 2ull * n_mesh) {
        delete s;
        return TT_ERR_UNSUPPORTED;
    }
    Aggregate(bvh8.BVH8Nodes, s->nodes.data());
    s->tlas_nodes = (uint32_t)bvh8.BVH8Nodes.size();
    s->mesh_aabbs.resize(6 * (size_t)n_mesh);
    for (uint32_t i = 0; i < n_mesh; i++) {
        const AABB& b = MeshAABBs[i];
        const float v[6] = {b.BBMax.x, b.BBMax.y, b.BBMax.z, b.BBMin.x, b.BBMin.y, b.BBMin.z};
        std::memcpy(&s->mesh_aabbs[6 * (size_t)i], v, sizeof(v));
    }
    s->tlas_indices.assign(bvh8.cwbvh_indices.begin(), bvh8.cwbvh_indices.end());
    *out = s;
    return TT_OK;
}

tt_status tt_scene_build_get_info(const tt_scene_build* s, tt_scene_build_info* info) {
    if (!s || !info) return TT_ERR_INVALID_ARG;
    info->n_nodes = (uint32_t)s->nodes.size();
    info->n_tris = (uint32_t)s->tris.size();
    info->n_tlas_indices = (uint32_t)s->tlas_indices.size();
    info->n_mesh = (uint32_t)s->meshdata.size();
    info->tlas_nodes = s->tlas_nodes;
    info->pad = 0;
    return TT_OK;
}

tt_status tt_scene_build_copy(const tt_scene_build* s, tt_cwbvh_node* nodes, tt_cuda_triangle* tris,
                              int32_t* tlas_indices, tt_mesh_data* meshdata) {
    if (!s) return TT_ERR_INVALID_ARG;
    if (nodes) std::memcpy(nodes, s->nodes.data(), s->nodes.size() * sizeof(tt_cwbvh_node));
    if (tris) std::memcpy(tris, s->tris.data(), s->tris.size() * sizeof(tt_cuda_triangle));
    if (tlas_indices) std::memcpy(tlas_indices, s->tlas_indices.data(), s->tlas_indices.size() * sizeof(int32_t));
    if (meshdata) std::memcpy(meshdata, s->meshdata.data(), s->meshdata.size() * sizeof(tt_mesh_data));
    return TT_OK;
}

tt_status tt_scene_build_copy_mesh_aabbs(const tt_scene_build* s, float* out6) {
    if (!s || !out6) return TT_ERR_INVALID_ARG;
    std::memcpy(out6, s->mesh_aabbs.data(), s->mesh_aabbs.size() * sizeof(float));
    return TT_OK;
}

void tt_scene_build_free(tt_scene_build* s) { delete s; }

}  // extern "C"
