// tt_refit.h — refit plans (host) and device state shared by tt_refit.hip and tt_api.hip: the TLAS
// refit (AssetManager.RefitTLAS) and the BLAS refit of deforming / skinned meshes
// (ParentObject.RefitMesh), which share NodeInitializer / layer refit / NodeUpdate / NodeCompress.
#ifndef TT_REFIT_H
#define TT_REFIT_H
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "tt_device.h"

// DocumentNodes (AssetManager.cs:1257-1297, ParentObject.cs:638-677 — the same walk) and the
// ForwardStack / LayerStack construction (AssetManager.cs:1364-1390, ParentObject.cs:706-730),
// from a node array whose root is node 0 and whose child indices are local to it (the TLAS
// region, or one BLAS). Returned as flat arrays.
struct RefitPlan {
    bool ok = true;          // false: a child index points outside [0, n_nodes) or the tree is too deep
    uint32_t n_tlas = 0;     // node count bound (TLAS nodes, or the BLAS's nodes)
    int32_t leaf_end = 0;    // largest leaf range end (primitive boxes the refit reads)
    std::vector<int32_t> pair_bvh, pair_slot, leaf, depth, parent, to_bvh, fwd;
    std::vector<std::vector<int32_t>> layers;  // NodePair indices per depth
};

// Device state of a prepared refit (one launch per refit: tt_refit.hip refit_tree).
struct RefitDev {
    int32_t *starts = nullptr, *fwd = nullptr, *parent = nullptr, *node_of = nullptr;
    uint32_t* arrive = nullptr;
    float* bb = nullptr;
    uint32_t n_pairs = 0, n_nodes = 0, n_starts = 0;
};

bool tt_refit_build_plan(const tt_cwbvh_node* nodes, uint32_t n_tlas_nodes, RefitPlan& R);
hipError_t tt_refit_prepare(const RefitPlan& R, const tt_cwbvh_node* host_nodes, uint32_t n_tlas_nodes, RefitDev& d);
// box_index: TLASCWBVHIndices for the TLAS (RefitBVHLayer), nullptr for a BLAS (RefitLayer reads
// the triangle boxes in leaf order directly)
hipError_t tt_refit_run(RefitDev& d, const float* boxes, const int32_t* box_index, tt_cwbvh_node* nodes, hipStream_t st);

// Construct (BVHRefitter.compute:72-120): one thread per triangle of the deformed mesh; writes the
// triangle's AABB (leaf order) and its positions / edges / packed normals into AggTris and the
// derived 48-B traversal layout.
struct BlasConstructArgs {
    const float* vertices;        // vertex_stride floats per vertex: position at +0, normal at +3
    const int32_t* indices;       // 3 per triangle (Unity order; the triangle is (i0, i2, i1))
    const int32_t* leaf_of;       // CWBVHIndicesBufferInverted: source triangle -> leaf-order index
    uint32_t n_tris, n_vertices, vertex_stride;
    float m[16];                  // Transform, column-major
    float* boxes;                 // n_tris x {BBMax, BBMin}
    tt_cuda_triangle* tris88;     // AggTris + TriOffset
    TriPos* tripos;               // traversal layout + TriOffset
};
hipError_t tt_blas_construct(const BlasConstructArgs& a, hipStream_t st);
void tt_refit_free(RefitDev& d);

#endif  // TT_REFIT_H
