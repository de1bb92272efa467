/*
 * tt_oracle.c — TEST INFRASTRUCTURE ONLY (see tt_oracle.h for the policy and the
 * parity status). A deliberately literal, one-ray-at-a-time restatement of the reference
 * HLSL; every block cites the reference lines it follows. Build with -ffp-contract=off:
 * the only fused operations are the explicit fmaf() calls of the numerics contract.
 */
#include "tt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef struct { float x, y, z; } v3;
typedef struct { v3 origin, direction, direction_inv; } Ray;        /* CommonData.cginc:80-84 */
typedef struct { float t, u, v; int mesh_id, triangle_id; } RayHit;  /* CommonData.cginc:91-96 */
typedef struct { uint32_t x, y; } uint2;

typedef struct scene {
    const tt_cwbvh_node* nodes; uint32_t n_nodes;
    const tt_cuda_triangle* tris; uint32_t n_tris;
    const int32_t* tlas; uint32_t n_tlas;
    const tt_mesh_data* md; uint32_t n_mesh;
    const tt_material* mats; uint32_t n_mat;
} scene;

/* ---------------------------------------------------------- pinned numerics */
static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vrcp(v3 a) { return mk(1.0f / a.x, 1.0f / a.y, 1.0f / a.z); }
static inline float vdot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 vcross(v3 a, v3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline uint32_t asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t firstbithigh(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
static inline uint32_t countbits(uint32_t x) { return (uint32_t)__builtin_popcount(x); }

/* Unity column-major matrix: element (r,c) at m[c*4+r]. */
static inline float M(const float* m, int r, int c) { return m[c * 4 + r]; }
/* mul((float3x3)W2L, d) */
static inline v3 mul33(const float* m, v3 d) {
    return mk(fmaf(M(m, 0, 2), d.z, fmaf(M(m, 0, 1), d.y, M(m, 0, 0) * d.x)),
              fmaf(M(m, 1, 2), d.z, fmaf(M(m, 1, 1), d.y, M(m, 1, 0) * d.x)),
              fmaf(M(m, 2, 2), d.z, fmaf(M(m, 2, 1), d.y, M(m, 2, 0) * d.x)));
}
/* mul(W2L, float4(o, 1)).xyz */
static inline v3 mul34(const float* m, v3 o) {
    return mk(fmaf(M(m, 0, 2), o.z, fmaf(M(m, 0, 1), o.y, M(m, 0, 0) * o.x)) + M(m, 0, 3),
              fmaf(M(m, 1, 2), o.z, fmaf(M(m, 1, 1), o.y, M(m, 1, 0) * o.x)) + M(m, 1, 3),
              fmaf(M(m, 2, 2), o.z, fmaf(M(m, 2, 1), o.y, M(m, 2, 0) * o.x)) + M(m, 2, 3));
}

/* ray_get_octant_inv4 — CommonData.cginc:635-640 */
static inline uint32_t ray_get_octant_inv4(v3 d) {
    return (d.x < 0.0f ? 0u : 0x04040404u) | (d.y < 0.0f ? 0u : 0x02020202u) |
           (d.z < 0.0f ? 0u : 0x01010101u);
}

/* cwbvh_node_intersect — CommonData.cginc:641-707 */
static uint32_t cwbvh_node_intersect(const Ray* ray, uint32_t oct_inv4, float max_distance,
                                     const tt_cwbvh_node* n) {
    const uint32_t node_0w = n->e_imask;
    const uint32_t e_x = node_0w & 0xff, e_y = (node_0w >> 8) & 0xff, e_z = (node_0w >> 16) & 0xff;
    const v3 adjusted_ray_direction_inv = mk(asfloat(e_x << 23) * ray->direction_inv.x,
                                             asfloat(e_y << 23) * ray->direction_inv.y,
                                             asfloat(e_z << 23) * ray->direction_inv.z);
    const v3 adjusted_ray_origin = vmul(ray->direction_inv, vsub(ld3(n->p), ray->origin));
    uint32_t hit_mask = 0;
    for (int i = 0; i < 2; i++) {
        const uint32_t meta4 = n->meta[i];
        const uint32_t is_inner4 = (meta4 & (meta4 << 1)) & 0x10101010u;
        const uint32_t inner_mask4 = (((is_inner4 << 3) >> 7) & 0x01010101u) * 0xffu;
        const uint32_t bit_index4 = (meta4 ^ (oct_inv4 & inner_mask4)) & 0x1f1f1f1fu;
        const uint32_t child_bits4 = (meta4 >> 5) & 0x07070707u;
        const uint32_t q_lo_x = n->qlo_x[i], q_hi_x = n->qhi_x[i];
        const uint32_t q_lo_y = n->qlo_y[i], q_hi_y = n->qhi_y[i];
        const uint32_t q_lo_z = n->qlo_z[i], q_hi_z = n->qhi_z[i];
        const uint32_t x_min = ray->direction.x < 0.0f ? q_hi_x : q_lo_x;
        const uint32_t x_max = ray->direction.x < 0.0f ? q_lo_x : q_hi_x;
        const uint32_t y_min = ray->direction.y < 0.0f ? q_hi_y : q_lo_y;
        const uint32_t y_max = ray->direction.y < 0.0f ? q_lo_y : q_hi_y;
        const uint32_t z_min = ray->direction.z < 0.0f ? q_hi_z : q_lo_z;
        const uint32_t z_max = ray->direction.z < 0.0f ? q_lo_z : q_hi_z;
        for (int j = 0; j < 4; j++) {
            v3 tmin3 = mk((float)((x_min >> (j * 8)) & 0xff), (float)((y_min >> (j * 8)) & 0xff),
                          (float)((z_min >> (j * 8)) & 0xff));
            v3 tmax3 = mk((float)((x_max >> (j * 8)) & 0xff), (float)((y_max >> (j * 8)) & 0xff),
                          (float)((z_max >> (j * 8)) & 0xff));
            tmin3 = mk(fmaf(tmin3.x, adjusted_ray_direction_inv.x, adjusted_ray_origin.x),
                       fmaf(tmin3.y, adjusted_ray_direction_inv.y, adjusted_ray_origin.y),
                       fmaf(tmin3.z, adjusted_ray_direction_inv.z, adjusted_ray_origin.z));
            tmax3 = mk(fmaf(tmax3.x, adjusted_ray_direction_inv.x, adjusted_ray_origin.x),
                       fmaf(tmax3.y, adjusted_ray_direction_inv.y, adjusted_ray_origin.y),
                       fmaf(tmax3.z, adjusted_ray_direction_inv.z, adjusted_ray_origin.z));
            const float tmin = fmaxf(fmaxf(tmin3.x, tmin3.y), fmaxf(tmin3.z, 1e-8f)); /* EPSILON :3 */
            const float tmax = fminf(fminf(tmax3.x, tmax3.y), fminf(tmax3.z, max_distance));
            if (tmin < tmax) {
                const uint32_t child_bits = (child_bits4 >> (j * 8)) & 0xff;
                const uint32_t bit_index = (bit_index4 >> (j * 8)) & 0xff;
                hit_mask |= child_bits << bit_index;
            }
        }
    }
    return hit_mask;
}

/* ------------------------------------------------------------ alpha atlas (f3) */
static const uint8_t* g_atlas = NULL;
static uint32_t g_atlas_w = 0, g_atlas_h = 0;

void tt_oracle_set_alpha_atlas(const uint8_t* texels, uint32_t width, uint32_t height) {
    g_atlas = texels;
    g_atlas_w = texels ? width : 0;
    g_atlas_h = texels ? height : 0;
}

/* AlignUV — CommonData.cginc:569-591 (Rotation 0, IsAlbedo false); AlphaTex packs the atlas
 * rectangle as 15-bit fixed point /16384 (max corner in .x, min corner in .y). */
static void align_uv(float bu, float bv, const float scale[4], const int32_t tex[2], float* ou, float* ov) {
    if (tex[0] <= 0) {
        *ou = -1.0f;
        *ov = -1.0f;
        return;
    }
    const float dx = (float)(((uint32_t)tex[0]) & 0x7FFFu) / 16384.0f;
    const float dy = (float)(((uint32_t)tex[0]) >> 15) / 16384.0f;
    const float dz = (float)(((uint32_t)tex[1]) & 0x7FFFu) / 16384.0f;
    const float dw = (float)(((uint32_t)tex[1]) >> 15) / 16384.0f;
    float x = bu * scale[0] + scale[2];
    float y = bv * scale[1] + scale[3];
    x = x < 0.0f ? 1.0f - fmodf(fabsf(x), 1.0f) : fmodf(fabsf(x), 1.0f);
    y = y < 0.0f ? 1.0f - fmodf(fabsf(y), 1.0f) : fmodf(fabsf(y), 1.0f);
    *ou = x * (dx - dz) + dz;
    *ov = y * (dy - dw) + dw;
}

static int atlas_clamp(float c, uint32_t n) { return (int)fminf(fmaxf(c, 0.0f), (float)(n - 1)); }
static float atlas_texel(int x, int y) { return (float)g_atlas[(size_t)y * g_atlas_w + (size_t)x] / 255.0f; }

/* SampleLevel(my_point_clamp_sampler, uv, 0) on the R8 atlas (pinned point filter) */
static float sample_point(float u, float v) {
    return atlas_texel(atlas_clamp(floorf(u * (float)g_atlas_w), g_atlas_w),
                       atlas_clamp(floorf(v * (float)g_atlas_h), g_atlas_h));
}

/* SampleLevel(my_linear_clamp_sampler, uv, 0) on the R8 atlas (pinned bilinear filter) */
static float sample_linear(float u, float v) {
    const float x = u * (float)g_atlas_w - 0.5f, y = v * (float)g_atlas_h - 0.5f;
    const float x0 = floorf(x), y0 = floorf(y);
    const float fx = x - x0, fy = y - y0;
    const int ix0 = atlas_clamp(x0, g_atlas_w), ix1 = atlas_clamp(x0 + 1.0f, g_atlas_w);
    const int iy0 = atlas_clamp(y0, g_atlas_h), iy1 = atlas_clamp(y0 + 1.0f, g_atlas_h);
    const float a = atlas_texel(ix0, iy0) * (1.0f - fx) + atlas_texel(ix1, iy0) * fx;
    const float b = atlas_texel(ix0, iy1) * (1.0f - fx) + atlas_texel(ix1, iy1) * fx;
    return a * (1.0f - fy) + b * fy;
}

/* BaseUv = tex0 * (1 - u - v) + texedge1 * u + texedge2 * v (raw vertex UVs, ParentObject.cs:1039-1041) */
/* ------------------------------------------------ texture atlas (f1 stained glass) */
/* _TextureAtlas decoded to RGBA half texels (Texture2D<half4>, CommonData.cginc:272). */
static const uint16_t* g_tex = NULL;
static uint32_t g_tex_w = 0, g_tex_h = 0;

void tt_oracle_set_texture_atlas(const uint16_t* rgba_half, uint32_t width, uint32_t height) {
    g_tex = rgba_half;
    g_tex_w = rgba_half ? width : 0;
    g_tex_h = rgba_half ? height : 0;
}

/* IEEE binary16 -> binary32, exact (NaNs keep their payload, quieted) */
static float half_to_float(uint16_t h) {
    const uint32_t sign = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t bits;
    if (e == 0x1fu) {
        bits = sign | 0x7f800000u | (m << 13) | (m ? 0x00400000u : 0u);
    } else if (e != 0) {
        bits = sign | ((e + 112u) << 23) | (m << 13);
    } else if (m == 0) {
        bits = sign;
    } else { /* subnormal half: normalise */
        uint32_t mm = m, ee = 113u;
        while (!(mm & 0x400u)) {
            mm <<= 1;
            ee--;
        }
        bits = sign | (ee << 23) | ((mm & 0x3ffu) << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

/* StainedGlassShadows tint (CommonData.cginc:621-622): throughput *= surfaceColor *
 * (_TextureAtlas.SampleLevel(my_point_clamp_sampler, AlignUV(BaseUv, AlbedoTexScale, AlbedoTex), 0).xyz
 * + 2) / 3, per component in that association, IEEE division (pinned). */
static void glass_tint(const tt_material* m, float bu, float bv, float throughput[3]) {
    float tu, tv;
    align_uv(bu, bv, m->AlbedoTexScale, m->AlbedoTex, &tu, &tv);
    const int x = atlas_clamp(floorf(tu * (float)g_tex_w), g_tex_w);
    const int y = atlas_clamp(floorf(tv * (float)g_tex_h), g_tex_h);
    const uint16_t* t = &g_tex[4 * ((size_t)y * g_tex_w + (size_t)x)];
    for (int k = 0; k < 3; k++) throughput[k] = throughput[k] * ((m->surfaceColor[k] * (half_to_float(t[k]) + 2.0f)) / 3.0f);
}

static void base_uv(const tt_cuda_triangle* T, float u, float v, float* bu, float* bv) {
    const float w = 1.0f - u - v;
    *bu = T->tex0[0] * w + T->texedge1[0] * u + T->texedge2[0] * v;
    *bv = T->tex0[1] * w + T->texedge1[1] * u + T->texedge2[1] * v;
}

static v3 vnormalize(v3 v);

/* IgnoreBackfacing (IntersectionKernels.compute:46): dot(normalize(cross(normalize(posedge1),
 * normalize(posedge2))), ray.direction) <= 0 rejects, ray.direction being the ray in the space the
 * triangle is tested in (object space inside a BLAS). normalize pinned as v * (1 / sqrt(dot(v, v))). */
static int backfacing(const v3 e1, const v3 e2, const v3 d) {
    return vdot(vnormalize(vcross(vnormalize(e1), vnormalize(e2))), d) <= 0.0f;
}

/* IntersectTriangle — IntersectionKernels.compute:14-57 (AdvancedAlphaMapped on; GlobalDefines.cginc
 * :1-11). IgnoreGlassMain (:42-44) and IgnoreBackfacing (:45-47) are compile-time defines there, off
 * by default; here they are the TT_TRACE_IGNORE_GLASS / TT_TRACE_IGNORE_BACKFACING launch flags.
 * Returns 0, or 3 when a Cutout material is reached without an alpha atlas (unsupported). */
static int intersect_triangle(const scene* s, int mesh_id, int tri_id, const Ray* ray,
                              RayHit* ray_hit, int MatOffset, int CurBounce, uint32_t flags, uint32_t* accepts) {
    const tt_cuda_triangle* T = &s->tris[tri_id];
    const v3 pos0 = ld3(T->pos0), posedge1 = ld3(T->posedge1), posedge2 = ld3(T->posedge2);
    const v3 h = vcross(ray->direction, posedge2);
    const float a = vdot(posedge1, h);
    const float f = 1.0f / a;
    const v3 sv = vsub(ray->origin, pos0);
    const float u = f * vdot(sv, h);
    if (u >= 0.0f && u <= 1.0f) {
        const v3 q = vcross(sv, posedge1);
        const float v = f * vdot(ray->direction, q);
        if (v >= 0.0f && u + v <= 1.0f) {
            const float t = f * vdot(posedge2, q);
            if (t > 0 && t < ray_hit->t) {
                ++*accepts;
                /* _Materials[MatOffset + MatDat]; an out-of-range StructuredBuffer read returns zeros
                 * in D3D, i.e. a material with no flags (MatType 0, Tag 0) */
                const int MaterialIndex = MatOffset + (int)T->MatDat;
                float specTrans = 0.0f;
                if (MaterialIndex >= 0 && (uint32_t)MaterialIndex < s->n_mat) {
                    const tt_material* m = &s->mats[MaterialIndex];
                    specTrans = m->specTrans;
                    if (m->MatType == TT_MAT_CUTOUT_INDEX) { /* :35-40 */
                        if (!g_atlas) return 3;
                        float bu, bv, au, av;
                        base_uv(T, u, v, &bu, &bv);
                        align_uv(bu, bv, m->AlbedoTexScale, m->AlphaTex, &au, &av);
                        if (sample_linear(au, av) < m->AlphaCutoff) return 0;
                    }
                }
                if ((flags & TT_TRACE_IGNORE_GLASS) && specTrans == 1.0f) return 0; /* :42-44 */
                if ((flags & TT_TRACE_IGNORE_BACKFACING) && CurBounce == 0 && specTrans != 1.0f && /* :45-47 */
                    backfacing(posedge1, posedge2, ray->direction))
                    return 0;
                if (MaterialIndex >= 0 && (uint32_t)MaterialIndex < s->n_mat &&
                    CurBounce == 0 && ((((int)s->mats[MaterialIndex].Tag) >> TT_FLAG_INVISIBLE) & 1) == 1)
                    return 0;
                ray_hit->t = t;
                ray_hit->u = u;
                ray_hit->v = v;
                ray_hit->mesh_id = mesh_id;
                ray_hit->triangle_id = tri_id;
            }
        }
    }
    return 0;
}

/* set() — CommonData.cginc:430-434 */
static void set_hit(tt_ray_data* r, const RayHit* h) {
    const uint32_t uv = (uint32_t)(h->u * 65535.0f) | ((uint32_t)(h->v * 65535.0f) << 16);
    r->hits[0] = (uint32_t)h->mesh_id;
    r->hits[1] = (uint32_t)h->triangle_id;
    r->hits[2] = asuint(h->t);
    r->hits[3] = uv;
}

typedef struct trace_job {
    const scene* s;
    const tt_trace_params* p;
    tt_ray_data* rays;
    uint32_t* info;
    const tt_col_data* colors;
    tt_oracle_ray_counts* counts;
} trace_job;

/* IntersectBVH — IntersectionKernels.compute:60-254 (HardwareRT off). */
static int intersect_bvh(const trace_job* J, uint32_t i) {
    const scene* s = J->s;
    const tt_trace_params* P = J->p;
    const int CurBounce = P->bounce;
    const float FarPlane = P->far_plane;
    tt_oracle_ray_counts cnt = {0, 0, 0, 0, 0, 0};

    uint2 stack[TT_STACK_SIZE];
    int stack_size = 0;
    uint2 current_group, triangle_group;
    uint32_t oct_inv4;
    int tlas_stack_size;
    Ray ray, ray2;
    int NodeOffset, TriOffset, MatOffset;
    int mesh_id = -1;
    int Reps;

    /* :79-83 ray pop; odd bounces read the second half of the ping-pong buffer */
    uint32_t ray_index = i;
    if (CurBounce % 2 == 1) ray_index += P->screen_width * P->screen_height;
    tt_ray_data* GlobalRay = &J->rays[ray_index];
    /* CreateRayHit — CommonData.cginc:364-372 */
    RayHit bestHit = {FarPlane, 0.0f, 0.0f, 0, -1};

    /* :139-153 */
    TriOffset = 0;
    MatOffset = 0;
    Reps = 0;
    ray.origin = ld3(GlobalRay->origin);
    ray.direction = ld3(GlobalRay->direction);
    ray.direction_inv = vrcp(ray.direction);
    NodeOffset = 0;
    tlas_stack_size = -1;
    ray2 = ray;
    oct_inv4 = ray_get_octant_inv4(ray.direction);
    current_group.x = 0u;
    current_group.y = 0x80000000u;
    int status = 1; /* Reps exhausted unless the loop returns */

    while (Reps < TT_MAX_REPS) {
        if (current_group.y & 0xff000000u) { /* :157-187 internal node step */
            const uint32_t child_index_offset = firstbithigh(current_group.y);
            const uint32_t slot_index = (child_index_offset - 24) ^ (oct_inv4 & 0xff);
            const uint32_t relative_index = countbits(current_group.y & ~(0xffffffffu << slot_index));
            const uint32_t child_node_index = current_group.x + relative_index;
            current_group.y &= ~(1u << child_index_offset);
            if (current_group.y & 0xff000000u) {
                if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                stack[stack_size++] = current_group;
                if ((uint32_t)stack_size > cnt.max_stack) cnt.max_stack = (uint32_t)stack_size;
            }
            const tt_cwbvh_node* TempNode = &s->nodes[child_node_index];
            const uint32_t hitmask = cwbvh_node_intersect(&ray, oct_inv4, bestHit.t, TempNode);
            current_group.y = (hitmask & 0xff000000u) | ((TempNode->e_imask >> 24) & 0xff);
            triangle_group.y = (hitmask & 0x00ffffffu);
            current_group.x = TempNode->base_child + (uint32_t)NodeOffset;
            triangle_group.x = TempNode->base_tri + (uint32_t)TriOffset;
            Reps++;
            cnt.node_visits++;
        } else { /* :188-191 */
            triangle_group = current_group;
            current_group.x = 0u;
            current_group.y = 0u;
        }

        if (triangle_group.y != 0) {
            if (tlas_stack_size == -1) { /* :194-219 TLAS leaf -> enter BLAS */
                const uint32_t mesh_offset = firstbithigh(triangle_group.y);
                triangle_group.y &= ~(1u << mesh_offset);
                mesh_id = s->tlas[triangle_group.x + mesh_offset];
                const tt_mesh_data* MD = &s->md[mesh_id];
                NodeOffset = MD->NodeOffset;
                TriOffset = MD->TriOffset;
                if (triangle_group.y != 0) {
                    if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                    stack[stack_size++] = triangle_group;
                }
                if (current_group.y & 0xff000000u) {
                    if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                    stack[stack_size++] = current_group;
                }
                if ((uint32_t)stack_size > cnt.max_stack) cnt.max_stack = (uint32_t)stack_size;
                tlas_stack_size = stack_size;
                const int root_index = (MD->mesh_data_bvh_offsets & 0x7fffffff);
                MatOffset = MD->MaterialOffset;
                ray.direction = mul33(MD->W2L, ray.direction);
                ray.origin = mul34(MD->W2L, ray.origin);
                ray.direction_inv = vrcp(ray.direction);
                oct_inv4 = ray_get_octant_inv4(ray.direction);
                current_group.x = (uint32_t)root_index;
                current_group.y = 0x80000000u;
                cnt.blas_entries++;
            } else { /* :220-226 leaf triangles, highest bit first */
                while (triangle_group.y != 0) {
                    const uint32_t triangle_index = firstbithigh(triangle_group.y);
                    triangle_group.y &= ~(1u << triangle_index);
                    cnt.tri_tests++;
                    if (intersect_triangle(s, mesh_id, (int)(triangle_group.x + triangle_index), &ray,
                                           &bestHit, MatOffset, CurBounce, P->flags, &cnt.accepts)) {
                        status = 3;
                        goto done;
                    }
                }
            }
        }

        if ((current_group.y & 0xff000000u) == 0) {
            if (stack_size == 0) { /* :229-241 finished: write _PrimaryTriangleInfo + hit */
                const uint32_t PixIndex = GlobalRay->PixelIndex;
                const uint32_t W = P->screen_width, H = P->screen_height;
                const uint32_t tx = PixIndex % W, ty = PixIndex / W;
                if (J->info && ty < H) {
                    uint32_t* o = &J->info[(size_t)4 * ((size_t)ty * W + tx)];
                    if (CurBounce == 0) {
                        o[0] = (uint32_t)bestHit.mesh_id;
                        o[1] = (uint32_t)(bestHit.triangle_id - s->md[bestHit.mesh_id].TriOffset);
                        o[2] = asuint(bestHit.u);
                        o[3] = asuint(bestHit.v);
                    } else {
                        const float w = J->colors[PixIndex].Data[3];
                        if (w == -1.0f || (float)CurBounce == w) {
                            const int restir = (P->flags & TT_TRACE_USE_RESTIRGI) != 0;
                            const int asvgf = (P->flags & TT_TRACE_USE_ASVGF) != 0;
                            if (restir && bestHit.t != FarPlane) {
                                o[0] = (uint32_t)bestHit.mesh_id;
                                o[1] = (uint32_t)(bestHit.triangle_id - s->md[bestHit.mesh_id].TriOffset);
                                o[2] = (uint32_t)(bestHit.u * 65535.0f) | ((uint32_t)(bestHit.v * 65535.0f) << 16);
                            } else if (asvgf || bestHit.t != FarPlane) {
                                o[0] = asuint(ray2.direction.x);
                                o[1] = asuint(ray2.direction.y);
                                o[2] = asuint(ray2.direction.z);
                            } else {
                                o[0] = asuint(ray2.direction.x * bestHit.t + ray2.origin.x);
                                o[1] = asuint(ray2.direction.y * bestHit.t + ray2.origin.y);
                                o[2] = asuint(ray2.direction.z * bestHit.t + ray2.origin.z);
                            }
                            o[3] = bestHit.t == FarPlane ? 1u : 0u;
                        }
                    }
                }
                set_hit(GlobalRay, &bestHit);
                status = 0;
                goto done;
            }
            if (stack_size == tlas_stack_size) { /* :243-249 BLAS -> TLAS */
                NodeOffset = 0;
                TriOffset = 0;
                tlas_stack_size = -1;
                ray = ray2;
                oct_inv4 = ray_get_octant_inv4(ray.direction);
            }
            current_group = stack[--stack_size];
        }
    }
done:
    cnt.status = (uint32_t)status;
    if (J->counts) J->counts[i] = cnt;
    return status;
}

typedef struct worker {
    const trace_job* J;
    uint32_t tid, nthreads;
    int worst;
} worker;

#define TT_ORACLE_CHUNK 4096u

static void* worker_main(void* arg) {
    worker* w = (worker*)arg;
    const uint32_t n = w->J->p->n_rays;
    for (uint32_t base = w->tid * TT_ORACLE_CHUNK; base < n; base += w->nthreads * TT_ORACLE_CHUNK) {
        const uint32_t end = base + TT_ORACLE_CHUNK < n ? base + TT_ORACLE_CHUNK : n;
        for (uint32_t i = base; i < end; i++) {
            const int st = intersect_bvh(w->J, i);
            if (st > w->worst) w->worst = st;
        }
    }
    return NULL;
}

static tt_status check_scene(const scene* s) {
    for (uint32_t m = 0; m < s->n_mat; m++)
        if (s->mats[m].MatType == TT_MAT_CUTOUT_INDEX && !g_atlas) return TT_ERR_UNSUPPORTED;
    return TT_OK;
}

tt_status tt_oracle_trace(const tt_cwbvh_node* nodes, uint32_t n_nodes,
                          const tt_cuda_triangle* tris, uint32_t n_tris,
                          const int32_t* tlas_indices, uint32_t n_tlas,
                          const tt_mesh_data* meshdata, uint32_t n_mesh,
                          const tt_material* materials, uint32_t n_mat,
                          const tt_trace_params* p, tt_ray_data* global_rays,
                          uint32_t* primary_info, const tt_col_data* global_colors,
                          tt_oracle_ray_counts* counts, int32_t nthreads) {
    if (!nodes || !tris || !tlas_indices || !meshdata || !p || !global_rays) return TT_ERR_INVALID_ARG;
    if (n_mat && !materials) return TT_ERR_INVALID_ARG;
    if (primary_info && p->bounce > 0 && !global_colors) return TT_ERR_INVALID_ARG;
    if (p->screen_width == 0 || p->screen_height == 0) return TT_ERR_INVALID_ARG;
    scene s = {nodes, n_nodes, tris, n_tris, tlas_indices, n_tlas, meshdata, n_mesh, materials, n_mat};
    tt_status st = check_scene(&s);
    if (st != TT_OK) return st;
    trace_job J = {&s, p, global_rays, primary_info, global_colors, counts};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    worker ws[1024];
    pthread_t th[1024];
    for (int t = 0; t < nthreads; t++) {
        ws[t].J = &J;
        ws[t].tid = (uint32_t)t;
        ws[t].nthreads = (uint32_t)nthreads;
        ws[t].worst = 0;
    }
    if (nthreads == 1) {
        worker_main(&ws[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker_main, &ws[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    int worst = 0;
    for (int t = 0; t < nthreads; t++) if (ws[t].worst > worst) worst = ws[t].worst;
    if (worst == 2) return TT_ERR_STACK_OVERFLOW;
    if (worst == 3) return TT_ERR_UNSUPPORTED;
    return TT_OK;
}

/* ------------------------------------------------------ any-hit (kernel_shadow) */
/* triangle_intersect_shadow — CommonData.cginc:593-634 with AdvancedAlphaMapped,
 * IgnoreGlassShadow and StainedGlassShadows on (GlobalDefines.cginc:1-8). The material checks run
 * BEFORE the t-range test (:611-629): a glass surface (specTrans == 1) that passes the alpha test
 * tints `throughput` even outside (0, max_distance) and never occludes. Returns 1 = occluder,
 * 0 = not, 3 = a material whose atlas was not set (Cutout: alpha atlas, glass: texture atlas). */
static int intersect_triangle_shadow(const scene* s, int tri_id, const Ray* ray, float max_distance,
                                     int MatOffset, uint32_t* accepts, float throughput[3]) {
    const tt_cuda_triangle* T = &s->tris[tri_id];
    const int MaterialIndex = MatOffset + (int)T->MatDat;
    const v3 pos0 = ld3(T->pos0), posedge1 = ld3(T->posedge1), posedge2 = ld3(T->posedge2);
    const v3 h = vcross(ray->direction, posedge2);
    const float a = vdot(posedge1, h);
    const float f = 1.0f / a;
    const v3 sv = vsub(ray->origin, pos0);
    const float u = f * vdot(sv, h);
    if (u >= 0.0f && u <= 1.0f) {
        const v3 q = vcross(sv, posedge1);
        const float v = f * vdot(ray->direction, q);
        if (v >= 0.0f && u + v <= 1.0f) {
            const float t = f * vdot(posedge2, q);
            /* out-of-range _Materials reads return zeros (no flags, MatType 0, specTrans 0) */
            if (MaterialIndex >= 0 && (uint32_t)MaterialIndex < s->n_mat) {
                const tt_material* m = &s->mats[MaterialIndex];
                const int tag = (int)m->Tag;
                if (((tag >> TT_FLAG_IS_BACKGROUND) & 1) || ((tag >> TT_FLAG_SHADOW_CASTER) & 1)) return 0;
                if (m->MatType == TT_MAT_CUTOUT_INDEX || m->specTrans == 1.0f) { /* :613-627 */
                    float bu, bv;
                    base_uv(T, u, v, &bu, &bv);
                    if (m->MatType == TT_MAT_CUTOUT_INDEX) { /* :616, point sampler */
                        if (!g_atlas) return 3;
                        float au, av;
                        align_uv(bu, bv, m->AlbedoTexScale, m->AlphaTex, &au, &av);
                        if (sample_point(au, av) < m->AlphaCutoff) return 0;
                    }
                    if (m->specTrans == 1.0f) { /* IgnoreGlassShadow + StainedGlassShadows: tint, never occlude */
                        if (!g_tex) return 3;
                        glass_tint(m, bu, bv, throughput);
                        return 0;
                    }
                }
            }
            if (t > 0.0f && t < max_distance) {
                ++*accepts;
                return 1;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------ row f1 colour encodings (RadianceCache path)
 * packRGBE / unpackRGBE (CommonData.cginc:479-509), EncodeRGB / DecodeRGB (:1576-1619) and HLSL pow
 * as D3D lowers it, exp2(y * log2(x)) with float intermediates. The reference leaves log2 / exp2 to
 * the driver; the pinned semantics (include/truetrace_hip.h, tt_trace_shadow_ex): log2 / exp2
 * evaluated in double with the fixed series below and rounded once to float, floor(log2) and
 * pow(2, n) exact via frexp / ldexp, round() half-to-even, D3D float -> uint, minNum / maxNum,
 * mul rows as fmaf chains, HLSL's unsuffixed literals as doubles rounded to float. */
static float p_log2f(float xf) {
    if (xf != xf || xf < 0.0f) return NAN;
    if (xf == 0.0f) return -INFINITY;
    if (xf == INFINITY) return xf;
    int e;
    double m = frexp((double)xf, &e);
    if (m < 0.70710678118654752) { m = m * 2.0; e = e - 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    static const double inv_odd[10] = {1.0 / 19.0, 1.0 / 17.0, 1.0 / 15.0, 1.0 / 13.0, 1.0 / 11.0,
                                       1.0 / 9.0,  1.0 / 7.0,  1.0 / 5.0,  1.0 / 3.0,  1.0};
    double q = 1.0 / 21.0;
    for (int k = 0; k < 10; k++) q = q * s2 + inv_odd[k];
    return (float)((double)e + (2.0 * s * q) * 1.4426950408889634);
}
static float p_exp2f(float yf) {
    if (yf != yf) return yf;
    if (yf >= 128.0f) return INFINITY;
    if (yf < -160.0f) return 0.0f;
    const double y = (double)yf, k = floor(y), f = y - k;
    const double r = f * 0.69314718055994531;
    double term = 1.0, sum = 1.0;
    for (int n = 1; n <= 22; n++) { term = term * r / (double)n; sum = sum + term; }
    return (float)ldexp(sum, (int)k);
}
static float p_pow(float x, float y) { return p_exp2f(y * p_log2f(x)); }
static uint32_t d3d_ftou(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}
static float clampf3(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
static float mrow(float m0, float m1, float m2, float x, float y, float z) { return fmaf(m2, z, fmaf(m1, y, m0 * x)); }

static uint32_t packRGBE(const float v[3]) { /* :479-496 */
    float va[3];
    for (int k = 0; k < 3; k++) va[k] = fmaxf(0.0f, v[k]);
    const float max_abs = fmaxf(va[0], fmaxf(va[1], va[2]));
    if (max_abs == 0.0f) return 0u;
    int e;
    (void)frexpf(max_abs, &e);
    const float exponent = (float)(e - 1); /* floor(log2(max_abs)) */
    uint32_t result = d3d_ftou(clampf3(exponent + 20.0f, 0.0f, 31.0f)) << 27;
    const float scale = p_exp2f(-exponent) * 256.0f; /* pow(2, -exponent) * 256 */
    uint32_t vu[3];
    for (int k = 0; k < 3; k++) vu[k] = d3d_ftou(fminf(511.0f, rintf(va[k] * scale)));
    return result | vu[0] | (vu[1] << 9) | (vu[2] << 18);
}
static void unpackRGBE(uint32_t x, float v[3]) { /* :498-509 */
    const int exponent = (int)(x >> 27) - 20;
    const float scale = p_exp2f((float)exponent) / 256.0f;
    v[0] = (float)(x & 0x1ffu) * scale;
    v[1] = (float)((x >> 9) & 0x1ffu) * scale;
    v[2] = (float)((x >> 18) & 0x1ffu) * scale;
}
static uint32_t EncodeRGB(const float c[3]) { /* :1576-1590 */
    const float X = mrow((float)0.4123907992659595, (float)0.3575843393838780, (float)0.1804807884018343, c[0], c[1], c[2]);
    const float Y = mrow((float)0.2126390058715104, (float)0.7151686787677559, (float)0.0721923153607337, c[0], c[1], c[2]);
    const float Z = mrow((float)0.0193308187155918, (float)0.1191947797946259, (float)0.9505321522496608, c[0], c[1], c[2]);
    const float logY = (float)409.6 * (p_log2f(Y) + 20.0f);
    const uint32_t Le = d3d_ftou(clampf3(logY, 0.0f, 16383.0f));
    if (Le == 0u) return 0u;
    const float invDenom = 1.0f / ((-2.0f * X + 12.0f * Y) + 3.0f * ((X + Y) + Z));
    const float u = (4.0f * X) * invDenom, v = (9.0f * Y) * invDenom;
    return (Le << 18) | (d3d_ftou(clampf3(820.0f * u, 0.0f, 511.0f)) << 9) | d3d_ftou(clampf3(820.0f * v, 0.0f, 511.0f));
}
static void DecodeRGB(uint32_t packed, float o[3]) { /* :1592-1619 */
    const uint32_t Le = packed >> 18;
    if (Le == 0u) { o[0] = o[1] = o[2] = 0.0f; return; }
    const float logY = ((float)Le + 0.5f) / (float)409.6 - 20.0f;
    const float Y = p_pow(2.0f, logY);
    const float u = ((float)((packed >> 9) & 0x1ffu) + 0.5f) / 820.0f, v = ((float)(packed & 0x1ffu) + 0.5f) / 820.0f;
    const float invDenom = 1.0f / ((6.0f * u - 16.0f * v) + 12.0f);
    const float x = (9.0f * u) * invDenom, y = (4.0f * v) * invDenom;
    const float s = Y / y;
    const float X = s * x, Z = s * ((1.0f - x) - y);
    o[0] = fmaxf(mrow((float)3.240969941904522, (float)-1.537383177570094, (float)-0.4986107602930032, X, Y, Z), 0.0f);
    o[1] = fmaxf(mrow((float)-0.9692436362808803, (float)1.875967501507721, (float)0.04155505740717569, X, Y, Z), 0.0f);
    o[2] = fmaxf(mrow((float)0.05563007969699373, (float)-0.2039769588889765, (float)1.056971514242878, X, Y, Z), 0.0f);
}

/* exported for the encoder known-answer tests */
uint32_t tt_oracle_pack_rgbe(const float v[3]) { return packRGBE(v); }
void tt_oracle_unpack_rgbe(uint32_t x, float v[3]) { unpackRGBE(x, v); }
uint32_t tt_oracle_encode_rgb(const float c[3]) { return EncodeRGB(c); }
void tt_oracle_decode_rgb(uint32_t x, float v[3]) { DecodeRGB(x, v); }
float tt_oracle_pow(float x, float y) { return p_pow(x, y); }

typedef struct shadow_job {
    const scene* s;
    const tt_shadow_params* p;
    tt_shadow_ray* rays;
    float* visibility;
    tt_col_data* colors;
    float* nee_pos;
    tt_cache_data* cache;
    tt_oracle_ray_counts* counts;
} shadow_job;

/* IntersectBVHShadow — IntersectionKernels.compute:264-500 (HardwareRT off, TerrainExists false).
 * status: 0 = reached |t| (outputs written), 4 = occluded (t = 0 written), 1 = Reps exhausted,
 * 2 = stack overflow, 3 = unsupported material. */
static int intersect_bvh_shadow(const shadow_job* J, uint32_t i) {
    const scene* s = J->s;
    const tt_shadow_params* P = J->p;
    const int CurBounce = P->bounce;
    tt_oracle_ray_counts cnt = {0, 0, 0, 0, 0, 0};
    uint2 stack[TT_STACK_SIZE];
    int stack_size = 0;
    uint2 current_group, triangle_group = {0u, 0u};
    uint32_t oct_inv4;
    int tlas_stack_size;
    Ray ray, ray2;
    int NodeOffset, TriOffset, MatOffset;
    int mesh_id = -1;
    int Reps;
    tt_shadow_ray* SR = &J->rays[i];
    const float max_distance = fabsf(SR->t);
    ray.origin = ld3(SR->origin);
    ray.direction = ld3(SR->direction);
    ray.direction_inv = vrcp(ray.direction);
    ray2 = ray;
    float throughput[3] = {1.0f, 1.0f, 1.0f}; /* :361, scaled by stained-glass tints */
    TriOffset = 0;
    MatOffset = 0;
    Reps = 0;
    NodeOffset = 0;
    oct_inv4 = ray_get_octant_inv4(ray.direction);
    current_group.x = 0u;
    current_group.y = 0x80000000u;
    tlas_stack_size = -1;
    int status = 1;
    (void)mesh_id;

    while (Reps < TT_MAX_REPS) {
        if (current_group.y & 0xff000000u) { /* :374-403 */
            const uint32_t child_index_offset = firstbithigh(current_group.y);
            const uint32_t slot_index = (child_index_offset - 24) ^ (oct_inv4 & 0xff);
            const uint32_t relative_index = countbits(current_group.y & ~(0xffffffffu << slot_index));
            const uint32_t child_node_index = current_group.x + relative_index;
            current_group.y &= ~(1u << child_index_offset);
            if (current_group.y & 0xff000000u) {
                if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                stack[stack_size++] = current_group;
                if ((uint32_t)stack_size > cnt.max_stack) cnt.max_stack = (uint32_t)stack_size;
            }
            const tt_cwbvh_node* TempNode = &s->nodes[child_node_index];
            const uint32_t hitmask = cwbvh_node_intersect(&ray, oct_inv4, max_distance, TempNode);
            current_group.y = (hitmask & 0xff000000u) | ((TempNode->e_imask >> 24) & 0xff);
            triangle_group.y = (hitmask & 0x00ffffffu);
            current_group.x = TempNode->base_child + (uint32_t)NodeOffset;
            triangle_group.x = TempNode->base_tri + (uint32_t)TriOffset;
            Reps++;
            cnt.node_visits++;
        } else { /* :404-407 */
            triangle_group = current_group;
            current_group.x = 0u;
            current_group.y = 0u;
        }
        int hit = 0;
        if (triangle_group.y != 0) {
            if (tlas_stack_size == -1) { /* :411-435 TLAS leaf -> enter BLAS */
                const uint32_t mesh_offset = firstbithigh(triangle_group.y);
                triangle_group.y &= ~(1u << mesh_offset);
                mesh_id = s->tlas[triangle_group.x + mesh_offset];
                const tt_mesh_data* MD = &s->md[mesh_id];
                NodeOffset = MD->NodeOffset;
                TriOffset = MD->TriOffset;
                if (triangle_group.y != 0) {
                    if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                    stack[stack_size++] = triangle_group;
                }
                if (current_group.y & 0xff000000u) {
                    if (stack_size == TT_STACK_SIZE) { status = 2; goto done; }
                    stack[stack_size++] = current_group;
                }
                if ((uint32_t)stack_size > cnt.max_stack) cnt.max_stack = (uint32_t)stack_size;
                tlas_stack_size = stack_size;
                const int root_index = (MD->mesh_data_bvh_offsets & 0x7fffffff);
                MatOffset = MD->MaterialOffset;
                ray.direction = mul33(MD->W2L, ray.direction);
                ray.origin = mul34(MD->W2L, ray.origin);
                ray.direction_inv = vrcp(ray.direction);
                oct_inv4 = ray_get_octant_inv4(ray.direction);
                current_group.x = (uint32_t)root_index;
                current_group.y = 0x80000000u;
                cnt.blas_entries++;
            } else { /* :436-446 leaf triangles until the first occluder */
                while (triangle_group.y != 0) {
                    const uint32_t triangle_index = firstbithigh(triangle_group.y);
                    triangle_group.y &= ~(1u << triangle_index);
                    cnt.tri_tests++;
                    const int r = intersect_triangle_shadow(s, (int)(triangle_group.x + triangle_index), &ray,
                                                            max_distance, MatOffset, &cnt.accepts, throughput);
                    if (r == 3) { status = 3; goto done; }
                    if (r) { hit = 1; break; }
                }
            }
        }
        if (hit) { /* :449-454 */
            SR->t = 0.0f;
            if (J->visibility) for (int k = 0; k < 4; k++) J->visibility[4 * (size_t)i + k] = 0.0f;
            status = 4;
            goto done;
        }
        if ((current_group.y & 0xff000000u) == 0) {
            if (stack_size == 0) { /* :457-485 reached the light: outputs (TerrainExists false) */
                const uint32_t PixelIndex = SR->PixelIndex;
                const uint32_t W = P->screen_width, H = P->screen_height;
                if (J->visibility) {
                    for (int k = 0; k < 3; k++) J->visibility[4 * (size_t)i + k] = throughput[k];
                    J->visibility[4 * (size_t)i + 3] = 1.0f;
                }
                if (CurBounce == 0 && J->nee_pos && PixelIndex / W < H) {
                    float* o = &J->nee_pos[4 * (size_t)PixelIndex];
                    const float d = fabsf(SR->t);
                    o[0] = ray2.origin.x + ray2.direction.x * d;
                    o[1] = ray2.origin.y + ray2.direction.y * d;
                    o[2] = ray2.origin.z + ray2.direction.z * d;
                    o[3] = 0.0f;
                }
                if (PixelIndex / W < H) { /* out-of-range UAV writes are dropped */
                    const int restir = (P->flags & TT_TRACE_USE_RESTIRGI) != 0;
                    const float* il = SR->illumination;
                    if (P->flags & TT_SHADOW_RADIANCE_CACHE) { /* #ifdef RadianceCache */
                        if (J->cache) { /* :464 */
                            float k3[3] = {1.0f, 1.0f, 1.0f}, d[3], o[3];
                            if (!(!restir || SR->t >= 0.0f)) unpackRGBE(asuint(SR->LuminanceIncomming), k3);
                            uint32_t* ci = &J->cache[PixelIndex].CurrentIlluminance;
                            DecodeRGB(*ci, d);
                            for (int k = 0; k < 3; k++) o[k] = d[k] + (il[k] * throughput[k]) * k3[k];
                            *ci = EncodeRGB(o);
                        }
                        if (J->colors) {
                            tt_col_data* C = &J->colors[PixelIndex];
                            if (SR->t >= 0.0f) {
                                if (CurBounce == 0) /* :469 */
                                    for (int k = 0; k < 3; k++) C->Direct[k] = C->Direct[k] + il[k] * throughput[k];
                            } else if (CurBounce != 0 && (restir || C->Data[3] == (float)CurBounce)) { /* :477 */
                                float k3[3] = {1.0f, 1.0f, 1.0f};
                                if (restir) unpackRGBE(asuint(SR->LuminanceIncomming), k3);
                                for (int k = 0; k < 3; k++) C->Indirect[k] = C->Indirect[k] + (il[k] * throughput[k]) * k3[k];
                            } else { /* :481 */
                                float pv[3], o[3];
                                unpackRGBE(C->PrimaryNEERay, pv);
                                for (int k = 0; k < 3; k++) o[k] = p_pow(pv[k], 2.2f) + p_pow(il[k], 1.0f / 2.2f) * throughput[k];
                                C->PrimaryNEERay = packRGBE(o);
                            }
                        }
                    } else if (J->colors) { /* #ifndef RadianceCache */
                        tt_col_data* C = &J->colors[PixelIndex];
                        if (SR->t >= 0.0f) {
                            if (CurBounce == 0)
                                for (int k = 0; k < 3; k++) C->Direct[k] = C->Direct[k] + il[k] * throughput[k];
                            else /* :472 */
                                for (int k = 0; k < 3; k++) C->Indirect[k] = C->Indirect[k] + il[k] * throughput[k];
                        } else if (CurBounce != 0 && (!restir && C->Data[3] == -1.0f)) { /* :479 */
                            for (int k = 0; k < 3; k++) C->Indirect[k] = C->Indirect[k] + il[k] * throughput[k];
                        } else { /* :481 */
                            float pv[3], o[3];
                            unpackRGBE(C->PrimaryNEERay, pv);
                            for (int k = 0; k < 3; k++) o[k] = p_pow(pv[k], 2.2f) + p_pow(il[k], 1.0f / 2.2f) * throughput[k];
                            C->PrimaryNEERay = packRGBE(o);
                        }
                    }
                }
                status = 0;
                goto done;
            }
            if (stack_size == tlas_stack_size) { /* :487-493 */
                NodeOffset = 0;
                TriOffset = 0;
                tlas_stack_size = -1;
                ray = ray2;
                oct_inv4 = ray_get_octant_inv4(ray.direction);
            }
            current_group = stack[--stack_size];
        }
    }
done:
    if (status == 1 && J->visibility) {
        for (int k = 0; k < 3; k++) J->visibility[4 * (size_t)i + k] = 0.0f;
        J->visibility[4 * (size_t)i + 3] = -1.0f;
    }
    cnt.status = (uint32_t)status;
    if (J->counts) J->counts[i] = cnt;
    return status;
}

/* VisabilityCheckCompute — CommonData.cginc:710-819: the same any-hit walk with the distance as
 * given and a zero throughput; returns 1 (visible) when the loop ends, the Reps bound included, 0 at
 * the first occluder, -2 on a stack overflow (the reference has no check), -3 unsupported material. */
static int visibility_check(const scene* s, tt_shadow_ray* SR, tt_oracle_ray_counts* cnt) {
    uint2 stack[TT_STACK_SIZE];
    int stack_size = 0;
    uint2 current_group, triangle_group = {0u, 0u};
    int tlas_stack_size = -1, TriOffset = 0, NodeOffset = 0, MatOffset = 0, Reps = 0;
    const float dist = SR->t;
    Ray ray, ray2;
    ray.origin = ld3(SR->origin);
    ray.direction = ld3(SR->direction);
    ray.direction_inv = vrcp(ray.direction); /* :722 */
    ray2 = ray;
    uint32_t oct_inv4 = ray_get_octant_inv4(ray.direction);
    current_group.x = 0u;
    current_group.y = 0x80000000u;
    float through[3] = {0.0f, 0.0f, 0.0f}; /* :732 */
    while (Reps < TT_MAX_REPS) {
        if (current_group.y & 0xff000000u) { /* :734-761 */
            const uint32_t child_index_offset = firstbithigh(current_group.y);
            const uint32_t slot_index = (child_index_offset - 24) ^ (oct_inv4 & 0xff);
            const uint32_t relative_index = countbits(current_group.y & ~(0xffffffffu << slot_index));
            const uint32_t child_node_index = current_group.x + relative_index;
            current_group.y &= ~(1u << child_index_offset);
            if (current_group.y & 0xff000000u) {
                if (stack_size == TT_STACK_SIZE) return -2;
                stack[stack_size++] = current_group;
            }
            const tt_cwbvh_node* TempNode = &s->nodes[child_node_index];
            const uint32_t hitmask = cwbvh_node_intersect(&ray, oct_inv4, dist, TempNode);
            current_group.y = (hitmask & 0xff000000u) | ((TempNode->e_imask >> 24) & 0xff);
            triangle_group.y = (hitmask & 0x00ffffffu);
            current_group.x = TempNode->base_child + (uint32_t)NodeOffset;
            triangle_group.x = TempNode->base_tri + (uint32_t)TriOffset;
            Reps++;
            cnt->node_visits++;
        } else { /* :762-765 */
            triangle_group = current_group;
            current_group.x = 0u;
            current_group.y = 0u;
        }
        if (triangle_group.y != 0) {
            if (tlas_stack_size == -1) { /* :768-791 */
                const uint32_t mesh_offset = firstbithigh(triangle_group.y);
                triangle_group.y &= ~(1u << mesh_offset);
                const int mesh_id = s->tlas[triangle_group.x + mesh_offset];
                const tt_mesh_data* MD = &s->md[mesh_id];
                NodeOffset = MD->NodeOffset;
                TriOffset = MD->TriOffset;
                if (triangle_group.y != 0) {
                    if (stack_size == TT_STACK_SIZE) return -2;
                    stack[stack_size++] = triangle_group;
                }
                if (current_group.y & 0xff000000u) {
                    if (stack_size == TT_STACK_SIZE) return -2;
                    stack[stack_size++] = current_group;
                }
                tlas_stack_size = stack_size;
                MatOffset = MD->MaterialOffset;
                ray.direction = mul33(MD->W2L, ray.direction);
                ray.origin = mul34(MD->W2L, ray.origin);
                ray.direction_inv = vrcp(ray.direction);
                oct_inv4 = ray_get_octant_inv4(ray.direction);
                current_group.x = (uint32_t)(MD->mesh_data_bvh_offsets & 0x7fffffff);
                current_group.y = 0x80000000u;
                cnt->blas_entries++;
            } else { /* :793-799 */
                while (triangle_group.y != 0) {
                    const uint32_t triangle_index = firstbithigh(triangle_group.y);
                    triangle_group.y &= ~(1u << triangle_index);
                    cnt->tri_tests++;
                    const int r = intersect_triangle_shadow(s, (int)(triangle_group.x + triangle_index), &ray, dist,
                                                            MatOffset, &cnt->accepts, through);
                    if (r == 3) return -3;
                    if (r) return 0;
                }
            }
        }
        if ((current_group.y & 0xff000000u) == 0) { /* :803-816 */
            if (stack_size == 0) break;
            if (stack_size == tlas_stack_size) {
                NodeOffset = 0;
                TriOffset = 0;
                tlas_stack_size = -1;
                ray = ray2;
                oct_inv4 = ray_get_octant_inv4(ray.direction);
            }
            current_group = stack[--stack_size];
        }
    }
    return 1;
}

typedef struct shadow_worker {
    const shadow_job* J;
    uint32_t tid, nthreads;
    int worst;
} shadow_worker;

static void* shadow_worker_main(void* arg) {
    shadow_worker* w = (shadow_worker*)arg;
    const uint32_t n = w->J->p->n_rays;
    for (uint32_t base = w->tid * TT_ORACLE_CHUNK; base < n; base += w->nthreads * TT_ORACLE_CHUNK) {
        const uint32_t end = base + TT_ORACLE_CHUNK < n ? base + TT_ORACLE_CHUNK : n;
        for (uint32_t i = base; i < end; i++) {
            if (w->J->p->flags & TT_SHADOW_VISIBILITY_CHECK) {
                tt_oracle_ray_counts cnt = {0, 0, 0, 0, 0, 0};
                const int v = visibility_check(w->J->s, &w->J->rays[i], &cnt);
                if (v < 0) {
                    if (-v > w->worst) w->worst = -v;
                } else if (w->J->visibility) {
                    for (int k = 0; k < 4; k++) w->J->visibility[4 * (size_t)i + k] = v ? 1.0f : 0.0f;
                }
                cnt.status = v == 1 ? 0u : (v == 0 ? 4u : (uint32_t)-v);
                if (w->J->counts) w->J->counts[i] = cnt;
                continue;
            }
            int st = intersect_bvh_shadow(w->J, i);
            if (st == 4) st = 0;
            if (st > w->worst) w->worst = st;
        }
    }
    return NULL;
}

tt_status tt_oracle_shadow(const tt_cwbvh_node* nodes, uint32_t n_nodes,
                           const tt_cuda_triangle* tris, uint32_t n_tris,
                           const int32_t* tlas_indices, uint32_t n_tlas,
                           const tt_mesh_data* meshdata, uint32_t n_mesh,
                           const tt_material* materials, uint32_t n_mat,
                           const tt_shadow_params* p, tt_shadow_ray* shadow_rays, float* visibility,
                           tt_col_data* global_colors, float* nee_pos, tt_cache_data* cache,
                           tt_oracle_ray_counts* counts, int32_t nthreads) {
    if (!nodes || !tris || !tlas_indices || !meshdata || !p || !shadow_rays) return TT_ERR_INVALID_ARG;
    if (n_mat && !materials) return TT_ERR_INVALID_ARG;
    if (p->screen_width == 0 || p->screen_height == 0) return TT_ERR_INVALID_ARG;
    scene s = {nodes, n_nodes, tris, n_tris, tlas_indices, n_tlas, meshdata, n_mesh, materials, n_mat};
    for (uint32_t m = 0; m < n_mat; m++)
        if ((materials[m].MatType == TT_MAT_CUTOUT_INDEX && !g_atlas) || (materials[m].specTrans == 1.0f && !g_tex))
            return TT_ERR_UNSUPPORTED;
    shadow_job J = {&s, p, shadow_rays, visibility, global_colors, nee_pos, cache, counts};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    shadow_worker ws[1024];
    pthread_t th[1024];
    for (int t = 0; t < nthreads; t++) {
        ws[t].J = &J;
        ws[t].tid = (uint32_t)t;
        ws[t].nthreads = (uint32_t)nthreads;
        ws[t].worst = 0;
    }
    if (nthreads == 1) {
        shadow_worker_main(&ws[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, shadow_worker_main, &ws[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    int worst = 0;
    for (int t = 0; t < nthreads; t++) if (ws[t].worst > worst) worst = ws[t].worst;
    if (worst == 2) return TT_ERR_STACK_OVERFLOW;
    if (worst == 3) return TT_ERR_UNSUPPORTED;
    return TT_OK;
}

/* ------------------------------------------------------------ normal resolve */
/* i_octahedral_32 — CommonData.cginc:849-857 (normalize pinned as v * (1/sqrt(dot))). */
static v3 vnormalize(v3 v) {
    const float inv = 1.0f / sqrtf(vdot(v, v));
    return mk(v.x * inv, v.y * inv, v.z * inv);
}
static v3 i_octahedral_32(uint32_t data) {
    const uint32_t ix = data & 65535u, iy = (data >> 16) & 65535u;
    const float vx = (float)ix / 32767.5f - 1.0f, vy = (float)iy / 32767.5f - 1.0f;
    v3 nor = mk(vx, vy, 1.0f - fabsf(vx) - fabsf(vy));
    const float t = fmaxf(-nor.z, 0.0f);
    nor.x += (nor.x > 0.0f) ? -t : t;
    nor.y += (nor.y > 0.0f) ? -t : t;
    return vnormalize(nor);
}

/* GetTriangleNormal (CommonData.cginc:904-911) and the unsmoothed geometric normal
 * (RayTracingShader.compute:111-118), Inverse = transpose((float3x3)W2L). */
tt_status tt_oracle_resolve_normals(const tt_cuda_triangle* tris, uint32_t n_tris,
                                    const tt_mesh_data* meshdata, uint32_t n_mesh,
                                    const tt_trace_params* p, const tt_ray_data* global_rays,
                                    float* normals6) {
    if (!tris || !meshdata || !p || !global_rays || !normals6) return TT_ERR_INVALID_ARG;
    const uint32_t off = (p->bounce % 2 == 1) ? p->screen_width * p->screen_height : 0;
    for (uint32_t i = 0; i < p->n_rays; i++) {
        const tt_ray_data* r = &global_rays[off + i];
        float* o = &normals6[(size_t)6 * i];
        const float t = asfloat(r->hits[2]);
        const int mesh_id = (int)r->hits[0], tri = (int)r->hits[1];
        if (!(t < p->far_plane) || tri < 0 || (uint32_t)tri >= n_tris || (uint32_t)mesh_id >= n_mesh) {
            for (int k = 0; k < 6; k++) o[k] = 0.0f;
            continue;
        }
        /* get() — CommonData.cginc:441-455 */
        const float u = (float)(r->hits[3] & 0xffff) / 65535.0f;
        const float v = (float)(r->hits[3] >> 16) / 65535.0f;
        const float* W = meshdata[mesh_id].W2L;
        /* Inverse[r][c] = W2L[c][r]; mul(Inverse, x).r = sum_c W2L[c][r] * x_c */
        const tt_cuda_triangle* T = &tris[tri];
        const v3 n0 = i_octahedral_32(T->norms[0]), n1 = i_octahedral_32(T->norms[1]),
                 n2 = i_octahedral_32(T->norms[2]);
        const float w0 = 1.0f - u - v;
        const v3 ni = mk(n0.x * w0 + u * n1.x + v * n2.x, n0.y * w0 + u * n1.y + v * n2.y,
                         n0.z * w0 + u * n1.z + v * n2.z);
        v3 g = mk(fmaf(M(W, 2, 0), ni.z, fmaf(M(W, 1, 0), ni.y, M(W, 0, 0) * ni.x)),
                  fmaf(M(W, 2, 1), ni.z, fmaf(M(W, 1, 1), ni.y, M(W, 0, 1) * ni.x)),
                  fmaf(M(W, 2, 2), ni.z, fmaf(M(W, 1, 2), ni.y, M(W, 0, 2) * ni.x)));
        const float gs = 1.0f / sqrtf(vdot(g, g));
        g = mk(gs * g.x, gs * g.y, gs * g.z);
        const v3 c = vcross(vnormalize(ld3(T->posedge1)), vnormalize(ld3(T->posedge2)));
        v3 us = mk(fmaf(M(W, 2, 0), c.z, fmaf(M(W, 1, 0), c.y, M(W, 0, 0) * c.x)),
                   fmaf(M(W, 2, 1), c.z, fmaf(M(W, 1, 1), c.y, M(W, 0, 1) * c.x)),
                   fmaf(M(W, 2, 2), c.z, fmaf(M(W, 1, 2), c.y, M(W, 0, 2) * c.x)));
        const float us_s = 1.0f / sqrtf(vdot(us, us));
        us = mk(-(us_s * us.x), -(us_s * us.y), -(us_s * us.z));
        if (vdot(us, g) < 0) us = mk(-us.x, -us.y, -us.z);
        o[0] = g.x; o[1] = g.y; o[2] = g.z;
        o[3] = us.x; o[4] = us.y; o[5] = us.z;
    }
    return TT_OK;
}

/* ------------------------------------------------------------ camera rays */
/* pcg_hash / hash_with — CommonData.cginc:374-389; random() non-ASVGF branch :413-426 */
static uint32_t pcg_hash(uint32_t seed) {
    const uint32_t state = seed * 747796405u + 2891336453u;
    const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
static uint32_t hash_with(uint32_t seed, uint32_t hash) {
    seed = (seed ^ 61u) ^ hash;
    seed += seed << 3;
    seed ^= seed >> 4;
    seed *= 0x27d4eb2du;
    return seed;
}
static void random2(uint32_t samdim, uint32_t pixel_index, int32_t frames, int32_t max_bounce,
                    int32_t cur_bounce, float* x, float* y) {
    const uint32_t hash = pcg_hash((pixel_index * 258u + samdim) * (uint32_t)(max_bounce + 1) + (uint32_t)cur_bounce);
    const float k = asfloat(0x2f7fffffu);
    *x = (float)hash_with((uint32_t)frames, hash) * k;
    *y = (float)hash_with((uint32_t)frames + 0xdeadbeefu, hash) * k;
}

tt_status tt_oracle_generate(const float* c2w, const float* ip, uint32_t width, uint32_t height,
                             float near_plane, float far_plane, int32_t jitter,
                             int32_t frames_accumulated, int32_t max_bounce,
                             tt_ray_data* global_rays) {
    if (!c2w || !ip || !global_rays || !width || !height) return TT_ERR_INVALID_ARG;
    for (uint32_t y = 0; y < height; y++) {
        for (uint32_t x = 0; x < width; x++) {
            const uint32_t pixel_index = y * width + x;
            float jx = 0.0f, jy = 0.0f;
            if (jitter) {
                random2(0, pixel_index, frames_accumulated, max_bounce, 0, &jx, &jy);
                jx -= 0.5f;
                jy -= 0.5f;
            }
            const float uvx = ((float)x + jx) / (float)width * 2.0f - 1.0f;
            const float uvy = ((float)y + jy) / (float)height * 2.0f - 1.0f;
            /* origin = mul(CamToWorld, (0,0,0,1)).xyz */
            const v3 origin = mk(M(c2w, 0, 3), M(c2w, 1, 3), M(c2w, 2, 3));
            /* direction = mul(CamInvProj, (uv, 0, 1)).xyz */
            v3 d = mk(fmaf(M(ip, 0, 1), uvy, M(ip, 0, 0) * uvx) + M(ip, 0, 3),
                      fmaf(M(ip, 1, 1), uvy, M(ip, 1, 0) * uvx) + M(ip, 1, 3),
                      fmaf(M(ip, 2, 1), uvy, M(ip, 2, 0) * uvx) + M(ip, 2, 3));
            /* direction = mul(CamToWorld, (d, 0)).xyz; normalize */
            d = mul33(c2w, d);
            d = vnormalize(d);
            tt_ray_data* r = &global_rays[pixel_index];
            r->origin[0] = origin.x + near_plane * d.x;
            r->origin[1] = origin.y + near_plane * d.y;
            r->origin[2] = origin.z + near_plane * d.z;
            r->PixelIndex = pixel_index;
            r->direction[0] = d.x;
            r->direction[1] = d.y;
            r->direction[2] = d.z;
            r->last_pdf = 0.0f;
            r->hits[0] = 0;
            r->hits[1] = 0;
            r->hits[2] = asuint(far_plane);
            r->hits[3] = 0;
        }
    }
    return TT_OK;
}

/* ------------------------------------------------------------ diffuse bounce enqueue (f2) */
/* kernel_shade's diffuse path and next-ray append (RayTracingShader.compute:52-84 sample_disc /
 * sample_cosine_weighted_direction / sample, :99-122 normals, :284 direction, :293 origin offset,
 * :498-506 append). The reference appends with InterlockedAdd, so its order is the atomics'
 * order; the library appends in source order (stable compaction) and so does this restatement.
 * sincos is pinned (HLSL leaves its precision to the driver): cephes minimax polynomials on
 * [-pi/4, pi/4] with explicit fmaf, |phi| > pi/4 reduced by pi/2 (two-constant Cody-Waite). */
void tt_oracle_sincos_pinned(float phi, float* s, float* c) {
    const int big = fabsf(phi) > 0.785398185253143310546875f;
    const float q = phi > 0.0f ? 1.0f : -1.0f;
    const float r = big ? fmaf(-q, -4.37113882867379e-8f, fmaf(-q, 1.57079637050628662109375f, phi)) : phi;
    const float z = r * r;
    const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
    const float cp = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f),
                               z, -0.5f), z, 1.0f);
    *s = big ? q * cp : sp;
    *c = big ? -q * sp : cp;
}
/* octahedral_32 — CommonData.cginc:840-846 (the shading-side encoder; round = round-half-even) */
static uint32_t octahedral_32_cd(v3 nor) {
    const float sx = nor.x >= 0.0f ? 1.0f : -1.0f, sy = nor.y >= 0.0f ? 1.0f : -1.0f;
    const float den = nor.x * sx + nor.y * sy + fabsf(nor.z);
    float x = nor.x / den, y = nor.y / den;
    if (!(nor.z >= 0.0f)) {
        const float ox = x;
        x = (1.0f - (y * sy)) * sx;
        y = (1.0f - (ox * sx)) * sy;
    }
    const uint32_t dx = (uint32_t)rintf(32767.5f + x * 32767.5f), dy = (uint32_t)rintf(32767.5f + y * 32767.5f);
    return dx | (dy << 16u);
}

tt_status tt_oracle_enqueue_diffuse_bounce(const tt_cuda_triangle* tris, uint32_t n_tris, const tt_mesh_data* meshdata,
                                           uint32_t n_mesh, const tt_trace_params* p, tt_ray_data* global_rays,
                                           int32_t frames, int32_t max_bounce, uint32_t* n_next) {
    if (!tris || !meshdata || !p || !global_rays || !n_next) return TT_ERR_INVALID_ARG;
    const uint32_t wh = p->screen_width * p->screen_height;
    if (!wh || p->n_rays > wh) return TT_ERR_INVALID_ARG;
    const uint32_t src = (p->bounce % 2 == 1) ? wh : 0u, dst = (p->bounce % 2 == 1) ? 0u : wh;
    uint32_t out = 0;
    for (uint32_t i = 0; i < p->n_rays; i++) {
        const tt_ray_data* R = &global_rays[src + i];
        const float t = asfloat(R->hits[2]);
        if (!(t < p->far_plane) || (int32_t)R->hits[1] < 0) continue;
        const int32_t mesh_id = (int32_t)R->hits[0], tri = (int32_t)R->hits[1];
        if ((uint32_t)tri >= n_tris || (uint32_t)mesh_id >= n_mesh) return TT_ERR_INVALID_ARG;
        /* sample(pdf, pixel_index): random(1, pixel_index), sample_disc, cosine lobe */
        float rx, ry;
        random2(1, R->PixelIndex, frames, max_bounce, p->bounce, &rx, &ry);
        float a = 2.0f * rx - 1.0f, b = 2.0f * ry - 1.0f;
        if (a == 0.0f) a = 0.00001f;
        if (b == 0.0f) b = 0.00001f;
        float phi, rr;
        if (a * a > b * b) {
            rr = a;
            phi = (0.25f * 3.14159265f) * (b / a);
        } else {
            rr = b;
            phi = (0.25f * 3.14159265f) * (a / b) + (0.5f * 3.14159265f);
        }
        float sp, cp;
        tt_oracle_sincos_pinned(phi, &sp, &cp);
        const float dx = rr * cp, dz = rr * sp;
        const v3 om = mk(dx, sqrtf(fabsf(1.0f - (dx * dx + dz * dz))), dz);
        const float pdf = om.y * 0.318309886548f;
        if (!(pdf > 0.0f)) continue; /* validBSDFSample */
        /* get() and the hit point */
        const float u = (float)(R->hits[3] & 0xffffu) / 65535.0f, v = (float)(R->hits[3] >> 16) / 65535.0f;
        const float* W = meshdata[mesh_id].W2L;
        const tt_cuda_triangle* T = &tris[tri];
        const v3 dir = ld3(R->direction), org = ld3(R->origin);
        const v3 pos = mk(dir.x * t + org.x, dir.y * t + org.y, dir.z * t + org.z);
        /* Geomnorm = GetTriangleNormal(..., Inverse) (CommonData.cginc:904-911), normalize pinned */
        const v3 n0 = i_octahedral_32(T->norms[0]), n1 = i_octahedral_32(T->norms[1]),
                 n2 = i_octahedral_32(T->norms[2]);
        const float w0 = 1.0f - u - v;
        const v3 ni = mk(n0.x * w0 + u * n1.x + v * n2.x, n0.y * w0 + u * n1.y + v * n2.y,
                         n0.z * w0 + u * n1.z + v * n2.z);
        v3 g = vnormalize(mk(fmaf(M(W, 2, 0), ni.z, fmaf(M(W, 1, 0), ni.y, M(W, 0, 0) * ni.x)),
                             fmaf(M(W, 2, 1), ni.z, fmaf(M(W, 1, 1), ni.y, M(W, 0, 1) * ni.x)),
                             fmaf(M(W, 2, 2), ni.z, fmaf(M(W, 1, 2), ni.y, M(W, 0, 2) * ni.x))));
        /* USGNorm = -normalize(mul(Inverse, cross(normalize(e1), normalize(e2)))) (:112-115) */
        const v3 c = vcross(vnormalize(ld3(T->posedge1)), vnormalize(ld3(T->posedge2)));
        v3 us = vnormalize(mk(fmaf(M(W, 2, 0), c.z, fmaf(M(W, 1, 0), c.y, M(W, 0, 0) * c.x)),
                              fmaf(M(W, 2, 1), c.z, fmaf(M(W, 1, 1), c.y, M(W, 0, 1) * c.x)),
                              fmaf(M(W, 2, 2), c.z, fmaf(M(W, 1, 2), c.y, M(W, 0, 2) * c.x))));
        us = mk(-us.x, -us.y, -us.z);
        if (vdot(us, g) < 0) us = mk(-us.x, -us.y, -us.z);
        if (vdot(dir, us) > 0.0f) { /* GotFlipped (:120-121) */
            us = mk(-us.x, -us.y, -us.z);
            g = mk(-g.x, -g.y, -g.z);
        }
        const v3 norm = i_octahedral_32(octahedral_32_cd(g)); /* :123-124 */
        /* ray.direction = normalize(mul(omega_o, GetTangentSpace(norm))) (CommonData.cginc:332-343) */
        const v3 helper = fabsf(norm.x) > 0.99f ? mk(0, 0, 1) : mk(1, 0, 0);
        const v3 tangent = vnormalize(vcross(norm, helper));
        const v3 binormal = vcross(norm, tangent);
        const v3 nd = vnormalize(mk(om.x * tangent.x + om.y * norm.x + om.z * binormal.x,
                                    om.x * tangent.y + om.y * norm.y + om.z * binormal.y,
                                    om.x * tangent.z + om.y * norm.z + om.z * binormal.z));
        /* append (:502-504): origin = USGNorm * NormalOffset + pos, pdf, set2(hit) */
        tt_ray_data* o = &global_rays[dst + out];
        const tt_ray_data src_ray = *R; /* dst never overlaps src (the other half) */
        o->origin[0] = us.x * 0.0001f + pos.x;
        o->origin[1] = us.y * 0.0001f + pos.y;
        o->origin[2] = us.z * 0.0001f + pos.z;
        o->PixelIndex = src_ray.PixelIndex;
        o->direction[0] = nd.x;
        o->direction[1] = nd.y;
        o->direction[2] = nd.z;
        o->last_pdf = pdf;
        for (int k = 0; k < 4; k++) o->hits[k] = src_ray.hits[k];
        out++;
    }
    *n_next = out;
    return TT_OK;
}

int32_t tt_oracle_hardware_threads(void) {
    const long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (int32_t)n : 1;
}

/* ------------------------------------------------------------ TLAS refit (f4) */
/* AssetManager.ConstructNewTLAS / CorrectRefit (AssetManager.cs:1256-1297 DocumentNodes,
 * :1353-1390 ForwardStack / LayerStack, :1420-1456) and the per-frame GPU refit RefitTLAS
 * (:1473-1548): BVHRefitter.compute NodeInitializer (:386-394), RefitBVHLayer (:220-252),
 * NodeUpdate (:277-317), NodeCompress (:344-371). */
typedef struct refit_pairs {
    uint32_t n, cap;
    int32_t* bvh;    /* NodeIndexPairData.BVHNode   */
    int32_t* slot;   /* NodeIndexPairData.InNodeOffset */
    int32_t* leaf;   /* IsLeafList.x */
    int32_t* depth;  /* IsLeafList.y */
    int32_t* parent; /* IsLeafList.z */
    int32_t* to_bvh; /* ToBVHIndex[bvh8 node] */
    int32_t max_depth;
    uint32_t n_nodes; /* bound on BVH8 node indices */
    int bad;          /* a child index left [0, n_nodes) or the recursion got too deep */
    const tt_cwbvh_node* nodes;
} refit_pairs;

static void rp_push(refit_pairs* R, int32_t bvh, int32_t slot) {
    if (R->n == R->cap) {
        R->cap = R->cap ? 2 * R->cap : 64;
        R->bvh = (int32_t*)realloc(R->bvh, sizeof(int32_t) * R->cap);
        R->slot = (int32_t*)realloc(R->slot, sizeof(int32_t) * R->cap);
        R->leaf = (int32_t*)realloc(R->leaf, sizeof(int32_t) * R->cap);
        R->depth = (int32_t*)realloc(R->depth, sizeof(int32_t) * R->cap);
        R->parent = (int32_t*)realloc(R->parent, sizeof(int32_t) * R->cap);
    }
    R->bvh[R->n] = bvh;
    R->slot[R->n] = slot;
    R->leaf[R->n] = 0;
    R->depth[R->n] = 0;
    R->parent[R->n] = 0;
    R->n++;
}

static uint8_t node_meta(const tt_cwbvh_node* n, int k) { return (uint8_t)(n->meta[k >> 2] >> (8 * (k & 3))); }

/* DocumentNodes — AssetManager.cs:1257-1297 / ParentObject.cs:638-677 (the same walk; the NodePair AABBs it computes are reset by
 * NodeInitializer every frame, so they are not kept) */
static void document_nodes(refit_pairs* R, int current, int parent, int next_bvh8, int is_leaf, int recur) {
    if (recur > R->max_depth) R->max_depth = recur;
    R->depth[current] = recur;
    R->parent[current] = parent;
    if (!is_leaf) {
        R->to_bvh[next_bvh8] = current;
        R->leaf[current] = 0;
        const tt_cwbvh_node* node = &R->nodes[next_bvh8];
        for (int i = 0; i < 8; i++) {
            rp_push(R, next_bvh8, i);
            const uint8_t m = node_meta(node, i);
            if ((m & 0x1f) < 24) {
                document_nodes(R, (int)R->n - 1, current, -1, 1, recur + 1);
            } else {
                const int child_index = (int)node->base_child + (m & 31) - 24;
                if (child_index < 0 || (uint32_t)child_index >= R->n_nodes || recur > 256) {
                    R->bad = 1;
                    return;
                }
                document_nodes(R, (int)R->n - 1, current, child_index, 0, recur + 1);
            }
        }
    } else {
        R->leaf[current] = 1;
    }
}

/* pow(2, ceil(log2(x))) pinned exactly (frexp); log2(0) = -inf -> 0, NaN / negative -> NaN */
static float pow2_ceil_log2(float x) {
    if (isnan(x) || x < 0.0f) return NAN;
    if (x == 0.0f) return 0.0f;
    if (isinf(x)) return INFINITY;
    int k;
    const float m = frexpf(x, &k);
    return ldexpf(1.0f, m == 0.5f ? k - 1 : k);
}

/* HLSL float -> uint conversion (D3D: NaN -> 0, saturating) */
static uint32_t ftou_d3d(float f) {
    if (isnan(f) || f <= 0.0f) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

/* The refit shared by the TLAS (RefitBVHLayer: leaf ranges index `boxes` through `box_index`, the
 * TLASCWBVHIndices) and a BLAS (RefitLayer: box_index NULL, leaf ranges are triangle boxes in leaf
 * order). `nodes` is the node array whose root is node 0 (child indices local to it), `n_nodes` a
 * bound on it; NodeCompress rewrites the nodes the plan reaches. */
static tt_status refit_core(tt_cwbvh_node* nodes, uint32_t n_nodes, const int32_t* box_index, uint32_t n_box_index,
                            const float* boxes, uint32_t n_boxes) {
    const uint32_t n_tlas_nodes = n_nodes;
    uint32_t n_tlas_nodes_used = n_nodes;
    const int32_t* tlas_indices = box_index;
    const uint32_t n_tlas_indices = n_box_index;
    const float* mesh_aabbs = boxes;
    const uint32_t n_mesh = n_boxes;
    refit_pairs R;
    memset(&R, 0, sizeof(R));
    R.nodes = nodes;
    R.to_bvh = (int32_t*)calloc(n_tlas_nodes, sizeof(int32_t));
    R.n_nodes = n_nodes;
    rp_push(&R, 0, 0); /* NodePair[0]: the root's dummy entry */
    document_nodes(&R, 0, 0, 0, 0, 0);
    if (R.bad) {
        free(R.bvh); free(R.slot); free(R.leaf); free(R.depth); free(R.parent); free(R.to_bvh);
        return TT_ERR_INVALID_ARG;
    }
    const uint32_t N = R.n;
    /* ForwardStack — :1370-1380 */
    int32_t* fwd = (int32_t*)calloc((size_t)N * 8, sizeof(int32_t));
    for (uint32_t i = 0; i < N; i++) {
        const tt_cwbvh_node* node = &nodes[R.bvh[i]];
        if (R.leaf[i]) {
            const uint8_t m = node_meta(node, R.slot[i]);
            const int first_triangle = m & 0x1f;
            const int num_bits = __builtin_popcount((unsigned)(m >> 5));
            fwd[(size_t)i * 8 + R.slot[i]] = num_bits + ((int)node->base_tri + first_triangle) * 24 + 1;
        } else {
            fwd[(size_t)i * 8 + R.slot[i]] = -(int)i - 1;
        }
        fwd[(size_t)R.parent[i] * 8 + R.slot[i]] = -(int)i - 1;
    }
    /* NodeInitializer + RefitBVHLayer, deepest layer first */
    float* mx = (float*)malloc(sizeof(float) * 3 * N);
    float* mn = (float*)malloc(sizeof(float) * 3 * N);
    for (uint32_t i = 0; i < N; i++)
        for (int a = 0; a < 3; a++) {
            mx[3 * i + a] = -9999999999.0f;
            mn[3 * i + a] = 9999999999.0f;
        }
    tt_status st = TT_OK;
    for (int d = R.max_depth; d >= 0 && st == TT_OK; d--) {
        for (uint32_t i = 0; i < N; i++) {
            if (R.depth[i] != d) continue;
            float rmx[3] = {-99999999.0f, -99999999.0f, -99999999.0f};
            float rmn[3] = {99999999.0f, 99999999.0f, 99999999.0f};
            for (int k = 0; k < 8; k++) {
                const int leaf = fwd[(size_t)i * 8 + k];
                if (leaf == 0) continue;
                if (leaf < 0) {
                    const int c = -leaf - 1;
                    for (int a = 0; a < 3; a++) {
                        rmx[a] = fmaxf(rmx[a], mx[3 * c + a]);
                        rmn[a] = fminf(rmn[a], mn[3 * c + a]);
                    }
                } else {
                    const int v = leaf - 1;
                    const int start = v / 24, end = start + v % 24;
                    for (int i4 = start; i4 < end; i4++) {
                        const int32_t bi = tlas_indices ? ((uint32_t)i4 < n_tlas_indices ? tlas_indices[i4] : -1) : i4;
                        if (bi < 0 || (uint32_t)bi >= n_mesh) {
                            st = TT_ERR_INVALID_ARG;
                            break;
                        }
                        const float* b = &mesh_aabbs[6 * (size_t)bi]; /* AABB {BBMax, BBMin} */
                        for (int a = 0; a < 3; a++) {
                            rmx[a] = fmaxf(rmx[a], b[a]);
                            rmn[a] = fminf(rmn[a], b[3 + a]);
                        }
                    }
                }
            }
            for (int a = 0; a < 3; a++) {
                mx[3 * i + a] = rmx[a];
                mn[3 * i + a] = rmn[a];
            }
        }
    }
    uint32_t n_used = 0;
    for (uint32_t i = 0; i < N; i++)
        if ((uint32_t)R.bvh[i] + 1u > n_used) n_used = (uint32_t)R.bvh[i] + 1u;
    if (n_used < n_tlas_nodes) n_tlas_nodes_used = n_used;
    if (st == TT_OK) {
        /* NodeUpdate into the fixed-layout nodes (p, e, per-slot quantized uints) */
        float* P = (float*)malloc(sizeof(float) * 3 * n_tlas_nodes_used);
        uint32_t* E = (uint32_t*)malloc(sizeof(uint32_t) * 3 * n_tlas_nodes_used);
        uint32_t* Q = (uint32_t*)malloc(sizeof(uint32_t) * 48 * n_tlas_nodes_used); /* [node][axis-min/max][slot] */
        for (uint32_t n = 0; n < n_tlas_nodes_used; n++) {
            const tt_cwbvh_node* s = &nodes[n];
            for (int a = 0; a < 3; a++) {
                P[3 * n + a] = s->p[a];
                E[3 * n + a] = (s->e_imask >> (8 * a)) & 0xff;
            }
            const uint32_t* words[6] = {s->qlo_x, s->qhi_x, s->qlo_y, s->qhi_y, s->qlo_z, s->qhi_z};
            for (int w = 0; w < 6; w++)
                for (int k = 0; k < 8; k++) Q[48 * n + 8 * w + k] = (words[w][k >> 2] >> (8 * (k & 3))) & 0xff;
        }
        for (uint32_t i = 1; i < N; i++) {
            const int node = R.bvh[i];
            const int link = R.to_bvh[node];
            float tmx[3], tmn[3];
            for (int a = 0; a < 3; a++) {
                tmx[a] = mx[3 * i + a];
                tmn[a] = mn[3 * i + a];
            }
            if (tmx[0] < -10000.0f)
                for (int a = 0; a < 3; a++) tmx[a] = tmn[a] = mn[3 * link + a];
            for (int a = 0; a < 3; a++) {
                const float e = pow2_ceil_log2((mx[3 * link + a] - mn[3 * link + a]) * 0.003921569f);
                const float p = mn[3 * link + a];
                uint32_t eu;
                memcpy(&eu, &e, 4);
                P[3 * node + a] = p;
                E[3 * node + a] = eu >> 23;
                Q[48 * node + 8 * (2 * a + 1) + R.slot[i]] = ftou_d3d(ceilf((tmx[a] - p) / e));
                Q[48 * node + 8 * (2 * a) + R.slot[i]] = ftou_d3d(floorf((tmn[a] - p) / e));
            }
        }
        /* NodeCompress — packed exactly as the reference (full uints shifted and OR-ed) */
        for (uint32_t n = 0; n < n_tlas_nodes_used; n++) {
            tt_cwbvh_node* o = &nodes[n];
            const uint32_t imask = o->e_imask >> 24;
            for (int a = 0; a < 3; a++) o->p[a] = P[3 * n + a];
            o->e_imask = E[3 * n + 0] | (E[3 * n + 1] << 8) | (E[3 * n + 2] << 16) | (imask << 24);
            uint32_t* words[6] = {o->qlo_x, o->qhi_x, o->qlo_y, o->qhi_y, o->qlo_z, o->qhi_z};
            for (int w = 0; w < 6; w++)
                for (int h = 0; h < 2; h++) {
                    const uint32_t* q = &Q[48 * n + 8 * w + 4 * h];
                    words[w][h] = q[0] | (q[1] << 8) | (q[2] << 16) | (q[3] << 24);
                }
        }
        free(P);
        free(E);
        free(Q);
    }
    free(mx);
    free(mn);
    free(fwd);
    free(R.bvh);
    free(R.slot);
    free(R.leaf);
    free(R.depth);
    free(R.parent);
    free(R.to_bvh);
    return st;
}

tt_status tt_oracle_tlas_refit(tt_cwbvh_node* nodes, uint32_t n_tlas_nodes, const int32_t* tlas_indices,
                               uint32_t n_tlas_indices, const float* mesh_aabbs, uint32_t n_mesh) {
    if (!nodes || !n_tlas_nodes || !tlas_indices || !mesh_aabbs) return TT_ERR_INVALID_ARG;
    return refit_core(nodes, n_tlas_nodes, tlas_indices, n_tlas_indices, mesh_aabbs, n_mesh);
}

/* ---------------------------------------------------------------- BLAS refit (f4) */
/* Construct — BVHRefitter.compute:72-120, with the numerics the HLSL leaves to DXC pinned as in
 * include/truetrace_hip.h (tt_blas_refit): mul rows fmaf(m2, z, fmaf(m1, y, m0 * x)) (+ m3),
 * normalize(v) = v * (1 / sqrt(dot)), round = round-half-to-even. */
static v3 vtx3(const float* vertices, uint32_t n_vertices, uint32_t stride, int32_t idx, int off) {
    if (idx < 0 || (uint32_t)idx >= n_vertices) return mk(0.0f, 0.0f, 0.0f); /* D3D: OOB reads 0 */
    const float* v = vertices + (size_t)idx * stride + off;
    return mk(v[0], v[1], v[2]);
}
static v3 xform_normal(const float* m, v3 n) {
    const v3 v = mul33(m, n);
    const float inv = 1.0f / sqrtf(fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x)));
    return mk(v.x * inv, v.y * inv, v.z * inv);
}
/* octahedral_32 — BVHRefitter.compute:62-68 */
static uint32_t octahedral_32(v3 n) {
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

tt_status tt_oracle_blas_refit(tt_cwbvh_node* nodes, uint32_t n_nodes, tt_cuda_triangle* tris, uint32_t n_tris,
                               const tt_mesh_data* meshdata, uint32_t n_mesh, uint32_t mesh_index,
                               const float* vertices, uint32_t n_vertices, uint32_t vertex_stride,
                               const int32_t* indices, uint32_t n_mesh_tris, const int32_t* leaf_of_triangle,
                               const float* transform) {
    if (!nodes || !tris || !meshdata || !vertices || !indices || !leaf_of_triangle || !transform || !n_mesh_tris ||
        vertex_stride < 6 || mesh_index >= n_mesh)
        return TT_ERR_INVALID_ARG;
    const tt_mesh_data* md = &meshdata[mesh_index];
    const uint32_t node_base = (uint32_t)md->NodeOffset, tri_base = (uint32_t)md->TriOffset;
    if ((uint32_t)(md->mesh_data_bvh_offsets & 0x7fffffff) != node_base || node_base >= n_nodes) return TT_ERR_UNSUPPORTED;
    if ((uint64_t)tri_base + n_mesh_tris > n_tris) return TT_ERR_INVALID_ARG;
    float* boxes = (float*)malloc(sizeof(float) * 6 * (size_t)n_mesh_tris);
    for (size_t i = 0; i < 6 * (size_t)n_mesh_tris; i++) boxes[i] = 0.0f; /* fresh AABBBuffer */
    for (uint32_t t = 0; t < n_mesh_tris; t++) {
        const int32_t i0 = indices[3 * t], i1 = indices[3 * t + 1], i2 = indices[3 * t + 2];
        /* vidx = Load3(...).xzy: p from i0, p2 from i2, p3 from i1 */
        const v3 p = mul34(transform, vtx3(vertices, n_vertices, vertex_stride, i0, 0));
        const v3 p2 = mul34(transform, vtx3(vertices, n_vertices, vertex_stride, i2, 0));
        const v3 p3 = mul34(transform, vtx3(vertices, n_vertices, vertex_stride, i1, 0));
        const v3 n1 = xform_normal(transform, vtx3(vertices, n_vertices, vertex_stride, i0, 3));
        const v3 n2 = xform_normal(transform, vtx3(vertices, n_vertices, vertex_stride, i2, 3));
        const v3 n3 = xform_normal(transform, vtx3(vertices, n_vertices, vertex_stride, i1, 3));
        const int32_t leaf = leaf_of_triangle[t];
        if (leaf < 0 || (uint32_t)leaf >= n_mesh_tris) continue; /* D3D drops out-of-range writes */
        float mx[3] = {fmaxf(fmaxf(p.x, p2.x), p3.x), fmaxf(fmaxf(p.y, p2.y), p3.y), fmaxf(fmaxf(p.z, p2.z), p3.z)};
        float mn[3] = {fminf(fminf(p.x, p2.x), p3.x), fminf(fminf(p.y, p2.y), p3.y), fminf(fminf(p.z, p2.z), p3.z)};
        for (int k = 0; k < 3; k++)
            if (mx[k] - mn[k] < 0.000001f) {
                mn[k] -= 0.000001f;
                mx[k] += 0.000001f;
            }
        float* b = &boxes[6 * (size_t)leaf];
        for (int k = 0; k < 3; k++) {
            b[k] = mx[k];
            b[3 + k] = mn[k];
        }
        tt_cuda_triangle* T = &tris[tri_base + (uint32_t)leaf];
        T->pos0[0] = p.x; T->pos0[1] = p.y; T->pos0[2] = p.z;
        T->posedge1[0] = p2.x - p.x; T->posedge1[1] = p2.y - p.y; T->posedge1[2] = p2.z - p.z;
        T->posedge2[0] = p3.x - p.x; T->posedge2[1] = p3.y - p.y; T->posedge2[2] = p3.z - p.z;
        T->norms[0] = octahedral_32(n1);
        T->norms[1] = octahedral_32(n2);
        T->norms[2] = octahedral_32(n3);
    }
    /* NodeInitializer, RefitLayer (:177-212, deepest first), NodeUpdate, NodeCompress over the plan
     * of ParentObject.Construct (:679-730) */
    const tt_status st = refit_core(nodes + node_base, n_nodes - node_base, NULL, 0, boxes, n_mesh_tris);
    free(boxes);
    return st;
}
