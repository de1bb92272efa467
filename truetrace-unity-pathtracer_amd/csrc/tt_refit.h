// tt_refit.h — TLAS refit plan (host) and device state shared by tt_refit.hip and tt_api.hip.
#ifndef TT_REFIT_H
#define TT_REFIT_H
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "tt_device.h"

// DocumentNodes (AssetManager.cs:1257-1297) and the ForwardStack / LayerStack construction
// (:1364-1390), from the TLAS region of the uploaded nodes. Returned as flat arrays.
struct RefitPlan {
    bool ok = true;          // false: a TLAS child index points outside [0, n_tlas_nodes)
    uint32_t n_tlas = 0;
    std::vector<int32_t> pair_bvh, pair_slot, leaf, depth, parent, to_bvh, fwd;
    std::vector<std::vector<int32_t>> layers;  // NodePair indices per depth
};

// Device state of a prepared refit.
struct RefitDev {
    int32_t *pair_bvh = nullptr, *pair_slot = nullptr, *to_bvh = nullptr, *fwd = nullptr, *layers = nullptr;
    float *bb = nullptr, *P = nullptr, *boxes = nullptr;
    uint32_t *E = nullptr, *Q = nullptr;
    uint32_t n_pairs = 0, n_nodes = 0, n_boxes = 0;
    std::vector<uint32_t> layer_off, layer_n;  // into `layers`
};

bool tt_refit_build_plan(const tt_cwbvh_node* nodes, uint32_t n_tlas_nodes, RefitPlan& R);
hipError_t tt_refit_prepare(const RefitPlan& R, const tt_cwbvh_node* host_nodes, uint32_t n_tlas_nodes, RefitDev& d);
hipError_t tt_refit_run(RefitDev& d, const float* boxes, const int32_t* tlas_idx, tt_cwbvh_node* nodes, hipStream_t st);
void tt_refit_free(RefitDev& d);

#endif  // TT_REFIT_H
