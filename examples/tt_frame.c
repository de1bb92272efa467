/* tt_frame.c — a plain C host driving one frame of the trace path through the C ABI, the way
 * RayTracingMaster drives it per bounce (RayTracingMaster.cs:954-1007): build the scene buffers
 * with the AssetManager restatement (include/truetrace_scene.h: ParentObject BLAS build +
 * AssetManager aggregation), upload them (AssetManager.SetMeshTraceBuffers, AssetManager.cs:75-88),
 * generate the primary rays (Generate, RayGenKernels.compute:40-57), trace bounce 0 with
 * _PrimaryTriangleInfo, enqueue the diffuse bounce and trace bounce 1 (kernel_trace,
 * IntersectionKernels.compute:60-260). All buffers are host arrays: the library stages them, as
 * the C# P/Invoke shim does. Only the two shared libraries are linked; no HIP header is needed.
 *
 * The scene is the BASELINE C1 Cornell box: room [-1,1]^3 with five walls (the
 * +z side open) plus a ceiling light quad |x|,|z| <= 0.25 at y = 0.999; camera (0,0,3.4) looking
 * -z, vertical FOV 40 degrees.
 *
 *   tt_frame [W H [dump_path]]   prints a one-line summary; with dump_path writes the uploaded
 *                                buffers, the traced rays and the info image (tests re-trace them
 *                                with the CPU oracle: tests/test_gpu_parity.py). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "truetrace_hip.h"
#include "truetrace_scene.h"

#define CHECK(call)                                                                        \
    do {                                                                                   \
        tt_status st_ = (call);                                                            \
        if (st_ != TT_OK) {                                                                \
            fprintf(stderr, "%s failed: %d %s\n", #call, (int)st_, ctx ? tt_last_error(ctx) : ""); \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

static const float kQuads[6][4][3] = {
    {{-1, -1, -1}, {1, -1, -1}, {1, -1, 1}, {-1, -1, 1}},              /* floor   */
    {{-1, 1, -1}, {-1, 1, 1}, {1, 1, 1}, {1, 1, -1}},                  /* ceiling */
    {{-1, -1, -1}, {-1, 1, -1}, {1, 1, -1}, {1, -1, -1}},              /* back    */
    {{-1, -1, -1}, {-1, -1, 1}, {-1, 1, 1}, {-1, 1, -1}},              /* left    */
    {{1, -1, -1}, {1, 1, -1}, {1, 1, 1}, {1, -1, 1}},                  /* right   */
    {{-0.25f, 0.999f, -0.25f}, {0.25f, 0.999f, -0.25f}, {0.25f, 0.999f, 0.25f}, {-0.25f, 0.999f, 0.25f}}, /* light */
};

static void identity(float* m) {
    memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
}

/* Unity cameraToWorldMatrix (camera looks down -z) and projectionMatrix.inverse, column-major. */
static void unity_camera(const double pos[3], const double fwd[3], double vfov_deg, unsigned w, unsigned h,
                         double near_plane, double far_plane, float* c2w, float* inv_proj) {
    const double fl = sqrt(fwd[0] * fwd[0] + fwd[1] * fwd[1] + fwd[2] * fwd[2]);
    const double f[3] = {fwd[0] / fl, fwd[1] / fl, fwd[2] / fl};
    double r[3] = {f[2], 0.0, -f[0]}; /* up (0,1,0) x forward: Unity is left-handed */
    const double rl = sqrt(r[0] * r[0] + r[2] * r[2]);
    r[0] /= rl;
    r[2] /= rl;
    const double u[3] = {f[1] * r[2] - f[2] * r[1], f[2] * r[0] - f[0] * r[2], f[0] * r[1] - f[1] * r[0]};
    memset(c2w, 0, 16 * sizeof(float));
    for (int i = 0; i < 3; i++) {
        c2w[0 * 4 + i] = (float)r[i];
        c2w[1 * 4 + i] = (float)u[i];
        c2w[2 * 4 + i] = (float)-f[i];
        c2w[3 * 4 + i] = (float)pos[i];
    }
    c2w[15] = 1.0f;
    /* inverse of the OpenGL-style perspective matrix Unity builds */
    const double ft = 1.0 / tan(vfov_deg * 3.14159265358979323846 / 360.0), aspect = (double)w / (double)h;
    const double a = (far_plane + near_plane) / (near_plane - far_plane), b = 2.0 * far_plane * near_plane / (near_plane - far_plane);
    memset(inv_proj, 0, 16 * sizeof(float));
    inv_proj[0 * 4 + 0] = (float)(aspect / ft);
    inv_proj[1 * 4 + 1] = (float)(1.0 / ft);
    inv_proj[2 * 4 + 3] = (float)(1.0 / b);
    inv_proj[3 * 4 + 2] = -1.0f;
    inv_proj[3 * 4 + 3] = (float)(a / b);
}

static int write_block(FILE* f, const void* p, size_t n) { return n == 0 || fwrite(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    tt_ctx* ctx = NULL;
    const unsigned W = argc > 2 ? (unsigned)atoi(argv[1]) : 256u, H = argc > 2 ? (unsigned)atoi(argv[2]) : 256u;
    const char* dump = argc > 3 ? argv[3] : NULL;
    const float far_plane = 1000.0f;
    if (W == 0 || H == 0 || W > 8192 || H > 8192) {
        fprintf(stderr, "usage: tt_frame [W H [dump_path]]\n");
        return 2;
    }
    if (tt_abi_version() != TT_ABI_VERSION) {
        fprintf(stderr, "ABI version mismatch: library %d, header %d\n", (int)tt_abi_version(), TT_ABI_VERSION);
        return 1;
    }
    if (tt_device_count() < 1) {
        fprintf(stderr, "no HIP device\n");
        return 3;
    }

    /* ParentObject mesh: 6 quads, 12 triangles, 4 vertices per quad */
    float pos[6 * 4 * 3];
    int32_t idx[6 * 6];
    for (int q = 0; q < 6; q++) {
        memcpy(pos + q * 12, kQuads[q], sizeof(kQuads[q]));
        const int32_t v = q * 4, t[6] = {v, v + 1, v + 2, v, v + 2, v + 3};
        memcpy(idx + q * 6, t, sizeof(t));
    }
    tt_mesh_input mesh;
    memset(&mesh, 0, sizeof(mesh));
    mesh.positions = pos;
    mesh.n_vertices = 24;
    mesh.indices = idx;
    mesh.n_indices = 36;
    mesh.lossy_scale[0] = mesh.lossy_scale[1] = mesh.lossy_scale[2] = 1.0f;
    tt_blas* blas = NULL;
    CHECK(tt_blas_build(&mesh, &blas));
    tt_parent_desc parent;
    memset(&parent, 0, sizeof(parent));
    parent.blas = blas;
    identity(parent.local_to_world);
    identity(parent.world_to_local);
    parent.material_count = 1;
    tt_scene_build* sb = NULL;
    CHECK(tt_scene_assemble(&parent, 1, NULL, 0, NULL, 0, &sb));
    tt_scene_build_info si;
    CHECK(tt_scene_build_get_info(sb, &si));
    tt_cwbvh_node* nodes = calloc(si.n_nodes, sizeof(*nodes));
    tt_cuda_triangle* tris = calloc(si.n_tris, sizeof(*tris));
    int32_t* tlas = calloc(si.n_tlas_indices, sizeof(*tlas));
    tt_mesh_data* md = calloc(si.n_mesh, sizeof(*md));
    tt_material* mats = calloc(1, sizeof(*mats)); /* opaque, no flags */
    tt_ray_data* rays = calloc(2 * (size_t)W * H, sizeof(*rays));
    uint32_t* info = calloc((size_t)W * H * 4, sizeof(uint32_t));
    if (!nodes || !tris || !tlas || !md || !mats || !rays || !info) return 1;
    CHECK(tt_scene_build_copy(sb, nodes, tris, tlas, md));

    tt_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.device = 0;
    cfg.max_rays = 2 * (uint64_t)W * H;
    CHECK(tt_ctx_create(&cfg, &ctx));
    CHECK(tt_scene_upload(ctx, nodes, si.n_nodes, tris, si.n_tris, tlas, si.n_tlas_indices, md, si.n_mesh, mats, 1));

    tt_camera cam;
    memset(&cam, 0, sizeof(cam));
    const double cpos[3] = {0.0, 0.0, 3.4}, cfwd[3] = {0.0, 0.0, -1.0};
    unity_camera(cpos, cfwd, 40.0, W, H, 0.3, far_plane, cam.cam_to_world, cam.cam_inv_proj);
    cam.near_plane = 0.3f;
    cam.far_plane = far_plane;
    cam.width = W;
    cam.height = H;
    cam.jitter = 1;
    cam.max_bounce = 1;
    CHECK(tt_generate_primary(ctx, &cam, rays));

    tt_trace_params p;
    memset(&p, 0, sizeof(p));
    p.n_rays = W * H;
    p.bounce = 0;
    p.far_plane = far_plane;
    p.screen_width = W;
    p.screen_height = H;
    p.flags = TT_TRACE_STATS;
    tt_stats s0, s1;
    CHECK(tt_trace_closest(ctx, &p, rays, info, NULL, &s0));
    uint32_t n_next = 0;
    CHECK(tt_enqueue_diffuse_bounce(ctx, &p, rays, 0, 1, &n_next));
    p.n_rays = n_next;
    p.bounce = 1;
    CHECK(tt_trace_closest(ctx, &p, rays, NULL, NULL, &s1));
    printf("tt_frame %ux%u: %u tris, %u nodes; bounce 0: %llu rays, %llu hits, %.2f nodes/ray; "
           "bounce 1: %u rays, %llu hits\n",
           W, H, si.n_tris, si.n_nodes, (unsigned long long)s0.rays, (unsigned long long)s0.hits,
           s0.rays ? (double)s0.node_visits / (double)s0.rays : 0.0, n_next, (unsigned long long)s1.hits);

    /* the same frame through the multi-GPU group of the ABI (tt_group_*): 2 members sharing device 0 (copy
     * gather; on a node, devices {0, .., 7} and RCCL), the screen-order primary records into a host array */
    uint32_t* ghits = (uint32_t*)malloc(sizeof(uint32_t) * 4 * (size_t)W * H);
    if (!ghits) return 2;
    tt_group_config gc;
    memset(&gc, 0, sizeof(gc));
    gc.width = W;
    gc.height = H;
    gc.flags = TT_GROUP_COPY_GATHER;
    const int32_t gdev[2] = {0, 0};
    tt_group* grp = NULL;
    if (tt_group_create(gdev, 2, &gc, &grp) != TT_OK) {
        fprintf(stderr, "tt_group_create failed\n");
        return 1;
    }
    if (tt_group_scene_upload(grp, nodes, si.n_nodes, tris, si.n_tris, tlas, si.n_tlas_indices, md, si.n_mesh, mats, 1) !=
            TT_OK ||
        tt_group_trace_frame(grp, &cam, ghits, NULL, 0) != TT_OK) {
        fprintf(stderr, "group frame failed: %s\n", tt_group_last_error(grp));
        return 1;
    }
    size_t gdiff = 0;
    for (size_t i = 0; i < (size_t)W * H; i++)
        gdiff += memcmp(ghits + 4 * i, rays[i].hits, 16) != 0;
    tt_group_destroy(grp);
    free(ghits);
    printf("tt_frame group: 2 members, %zu of %u primary records differ from the single-context frame\n", gdiff, W * H);

    int rc = gdiff ? 4 : 0;
    if (dump) {
        FILE* f = fopen(dump, "wb");
        const uint32_t hdr[10] = {0x54544652u, W, H, si.n_nodes, si.n_tris, si.n_tlas_indices, si.n_mesh, 1u,
                                  si.tlas_nodes, n_next};
        const int ok = f && write_block(f, hdr, sizeof(hdr)) && write_block(f, nodes, sizeof(*nodes) * si.n_nodes) &&
                       write_block(f, tris, sizeof(*tris) * si.n_tris) &&
                       write_block(f, tlas, sizeof(*tlas) * si.n_tlas_indices) &&
                       write_block(f, md, sizeof(*md) * si.n_mesh) && write_block(f, mats, sizeof(*mats)) &&
                       write_block(f, rays, sizeof(*rays) * 2 * (size_t)W * H) &&
                       write_block(f, info, sizeof(uint32_t) * 4 * (size_t)W * H);
        if (f) fclose(f);
        if (!ok) {
            fprintf(stderr, "cannot write %s\n", dump);
            rc = 1;
        }
    }
    tt_ctx_destroy(ctx);
    tt_scene_build_free(sb);
    tt_blas_free(blas);
    free(nodes);
    free(tris);
    free(tlas);
    free(md);
    free(mats);
    free(rays);
    free(info);
    return rc;
}
