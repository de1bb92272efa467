// tt_synth.h — seeded synthetic meshes for the BASELINE.json configs (host side, C ABI).
#ifndef TT_SYNTH_H
#define TT_SYNTH_H
#include "../../include/truetrace_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tt_synth_mesh tt_synth_mesh;

tt_status tt_synth_cornell(tt_synth_mesh** out);
tt_status tt_synth_soup(uint64_t seed, uint32_t n_tris, float extent, float tri_size, tt_synth_mesh** out);
tt_status tt_synth_sponza(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out);
tt_status tt_synth_prop(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out);
tt_status tt_synth_ground(double x0, double x1, double z0, double z1, uint32_t nu, uint32_t nv,
                          tt_synth_mesh** out);
tt_status tt_synth_san_miguel(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out);
tt_synth_mesh* tt_synth_mesh_from_arrays(const float* pos, uint32_t n_vertices, const int32_t* idx,
                                         uint32_t n_indices, const int32_t* matdat);
/* Pointers stay valid until tt_synth_mesh_free. lossy_scale defaults to (1,1,1). */
tt_status tt_synth_mesh_view(const tt_synth_mesh* m, tt_mesh_input* view);
void tt_synth_mesh_free(tt_synth_mesh* m);

#ifdef __cplusplus
}
#endif
#endif
