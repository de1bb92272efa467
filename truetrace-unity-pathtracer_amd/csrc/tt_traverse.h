// tt_traverse.h — device-side building blocks shared by the closest-hit (tt_trace.hip) and the
// any-hit (tt_shadow.hip) CWBVH8 traversal kernels: tuning macros, the node test
// (CommonData.cginc:641-707), the triangle test (IntersectionKernels.compute:14-57), raw-buffer
// fetch helpers and the per-XCD segment ray scheduler.
#ifndef TT_TRAVERSE_H
#define TT_TRAVERSE_H
#include "tt_device.h"

#define TT_WAVE 64
// Threads per persistent block: ONE wave. The scheduler is per wave anyway, and when two grids share
// the chip (the two-part layout) a one-wave block frees its CU slot the moment its wave
// drains instead of waiting for the block's slowest of four: C2 two-part step 0.816-0.824 -> 0.783-0.795
// ms, single-stream launches unchanged (profiles/r03/block/).
#ifndef TT_BLOCK
#define TT_BLOCK 64
#endif
#ifndef TT_SEGS
#define TT_SEGS 8         // ray-range segments, one per XCD group (blockIdx % 8), with stealing
// (Within a dispatch each blockIdx % 8 class runs on one XCD, but the round-robin continues from where the
// previous dispatch left it, so band s meets a different XCD launch after launch -- tools/xcc_map.hip.
// Keying the start segment on the XCC_ID register instead measured neutral (profiles/r06/xcc/): a launch
// finds no previous launch's lines in its XCD's L2 either way.)
#endif
#ifndef TT_CHUNK_BIG
#define TT_CHUNK_BIG 64   // rays per dequeue (the surplus waits in the wave's pool)
#endif
#ifndef TT_REFILL_MIN
#define TT_REFILL_MIN 20  // refill idle lanes once at least this many are idle (16 -> 20: profiles/r04/ab)
#endif
#ifndef TT_PUSH_FAST
#define TT_PUSH_FAST 1  // the stack push tests only "an LDS entry is free" on its common path (0: A/B; profiles/r04/ab)
#endif
#ifndef TT_DRAIN_PRIO
#define TT_DRAIN_PRIO 2  // s_setprio level a wave takes once its launch's queue is dry (0: off; with TT_LONG_PRIO +0.8%, profiles/r04/ab/r04h_*)
#endif
#ifndef TT_LONG_PRIO
#define TT_LONG_PRIO 64  // s_setprio 2 for a wave with a ray past this many node steps, set at refills (0: off)
#endif
#ifndef TT_LONG_PRIO_LEVEL
#define TT_LONG_PRIO_LEVEL 2  // the s_setprio level of TT_LONG_PRIO (A/B: 3 ranks it above draining waves)
#endif
#ifndef TT_UNIFORM_POOL
#define TT_UNIFORM_POOL 1  // readfirstlane the scheduler's pool state after each refill (0: A/B; +1.2% bench, profiles/r04/ab)
#endif
#ifndef TT_LDS_STACK
#define TT_LDS_STACK 12   // stack entries kept in LDS; deeper entries spill to a global area
#endif
#ifndef TT_WAVES_PER_EU
#define TT_WAVES_PER_EU 0 // __launch_bounds__ min waves per SIMD (0: compiler default)
#endif
#if TT_WAVES_PER_EU > 0
#define TT_BOUNDS __launch_bounds__(TT_BLOCK, TT_WAVES_PER_EU)
#else
#define TT_BOUNDS __launch_bounds__(TT_BLOCK)
#endif

// TT_DIAG_BLOCKS builds (tools/diag_blocks.py; never the product): per-block execution counters of
// the closest-hit loop in LDS, flushed to TraceArgs::diag_times at the end of the launch. TT_DB(k): one
// wave execution of block k (counted by the first active lane); TT_DL(k, pred): lanes with pred.
#ifdef TT_DIAG_BLOCKS
#define TT_DB_N 32
__shared__ unsigned long long tt_db[TT_DB_N];
#define TT_DB(k)                                                                               \
    do {                                                                                       \
        const uint64_t m_ = __ballot(1);                                                       \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(m_)) atomicAdd(&tt_db[k], 1ull); \
    } while (0)
#define TT_DL(k, pred)                                                                         \
    do {                                                                                       \
        const uint64_t p_ = __ballot(pred), m_ = __ballot(1);                                  \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(m_))                              \
            atomicAdd(&tt_db[k], (unsigned long long)__popcll(p_));                            \
    } while (0)
#else
#define TT_DB(k) \
    do {         \
    } while (0)
#define TT_DL(k, pred) \
    do {               \
    } while (0)
#endif

namespace {

struct LaneRay {
    float ox, oy, oz, dx, dy, dz, ix, iy, iz;
};

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ uint32_t firstbithigh(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// ray_get_octant_inv4 — CommonData.cginc:635-640
__device__ __forceinline__ uint32_t octant_inv4(const LaneRay& r) {
    return (r.dx < 0.0f ? 0u : 0x04040404u) | (r.dy < 0.0f ? 0u : 0x02020202u) |
           (r.dz < 0.0f ? 0u : 0x01010101u);
}


// Node / triangle fetches are raw buffer loads: a 32-bit byte offset per lane (two full-rate
// shift-adds) instead of a 64-bit address (v_mad_u64_u32), and a bounded descriptor, so an
// out-of-range offset reads zeros instead of faulting. Offsets stay below 2^32 because
// tt_scene_upload rejects node / triangle arrays of 4 GiB or more.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// CPOL: the load's cache-policy bits (gfx950: 2 = nt, non-temporal / streaming). A/B knobs only:
// TT_TRI_CPOL for the triangle loads (does the 12.6 MB of C2's triangles evict its 2.5 MB node set from
// each XCD's L2?), TT_NODE_CPOL for the node loads; both 0 (default policy) in the product.
#ifndef TT_TRI_CPOL
#define TT_TRI_CPOL 0
#endif
#ifndef TT_NODE_CPOL
#define TT_NODE_CPOL 0
#endif
template <int CPOL = 0>
__device__ __forceinline__ uint4 buffer_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, CPOL);
    return make_uint4(v.x, v.y, v.z, v.w);
}
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int CPOL = 0>
__device__ __forceinline__ uint2 buffer_load8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, CPOL);
    return make_uint2(v.x, v.y);
}
template <int CPOL = 0>
__device__ __forceinline__ uint32_t buffer_load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, CPOL);
}
// i * 80 and i * 48 as shift-adds: written plainly, LLVM folds them back into v_mul_lo_u32, a
// quarter-rate instruction on the traversal's critical path. TT_NODE_STRIDE 128: the kernels read a
// derived copy of the node array with every 80-B node at the start of its own 128-B line (tt_api.hip
// keeps it in step with the reference array), so a node visit touches one cache line instead of 1.5.
static_assert(TT_NODE_STRIDE == 80 || TT_NODE_STRIDE == 128, "node stride: 80 (the reference array) or 128");
__device__ __forceinline__ uint32_t node_offset(uint32_t i) {
    if (TT_NODE_STRIDE == 128) return i << 7;
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1\n\tv_lshlrev_b32 %0, 4, %0" : "=&v"(r) : "v"(i));
    return r;
}
__device__ __forceinline__ uint32_t tri_offset(uint32_t i) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 1, %1\n\tv_lshlrev_b32 %0, 4, %0" : "=&v"(r) : "v"(i));
    return r;
}

// cwbvh_node_intersect — CommonData.cginc:641-707
__device__ __forceinline__ uint32_t node_intersect(const uint4 n0, const uint4 n1, const uint4 n2,
                                                   const uint4 n3, const uint4 n4, const LaneRay& r,
                                                   uint32_t oct_inv4, float max_distance) {
    const uint32_t w = n0.w;
    // asfloat(e << 23) per axis: the exponent byte shifted into place by ONE v_lshlrev_b32_sdwa
    // (byte-selected source, so no mask), instead of a shift + an AND each
    uint32_t ex, ey, ez;
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
        : "=v"(ex) : "s"(23u), "v"(w));
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
        : "=v"(ey) : "s"(23u), "v"(w));
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
        : "=v"(ez) : "s"(23u), "v"(w));
    const float adjx = __uint_as_float(ex) * r.ix;
    const float adjy = __uint_as_float(ey) * r.iy;
    const float adjz = __uint_as_float(ez) * r.iz;
    const float orgx = r.ix * (__uint_as_float(n0.x) - r.ox);
    const float orgy = r.iy * (__uint_as_float(n0.y) - r.oy);
    const float orgz = r.iz * (__uint_as_float(n0.z) - r.oz);
    const bool nx = r.dx < 0.0f, ny = r.dy < 0.0f, nz = r.dz < 0.0f;
    uint32_t hit_mask = 0;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const uint32_t meta4 = i == 0 ? n1.z : n1.w;
        const uint32_t is_inner4 = (meta4 & (meta4 << 1)) & 0x10101010u;
        // 0x07 in each inner child's byte (oct_inv4 bytes are <= 7, so 3 bits of the reference's
        // 0xff byte mask suffice); 8 - 1 per byte, no borrow: avoids the quarter-rate v_mul_lo_u32
        const uint32_t inner_mask4 = (is_inner4 >> 1) - (is_inner4 >> 4);
        const uint32_t bit_index4 = (meta4 ^ (oct_inv4 & inner_mask4)) & 0x1f1f1f1fu;
        const uint32_t child_bits4 = (meta4 >> 5) & 0x07070707u;
        const uint32_t qlx = i == 0 ? n2.x : n2.y, qhx = i == 0 ? n2.z : n2.w;
        const uint32_t qly = i == 0 ? n3.x : n3.y, qhy = i == 0 ? n3.z : n3.w;
        const uint32_t qlz = i == 0 ? n4.x : n4.y, qhz = i == 0 ? n4.z : n4.w;
        const uint32_t x_min = nx ? qhx : qlx, x_max = nx ? qlx : qhx;
        const uint32_t y_min = ny ? qhy : qly, y_max = ny ? qly : qhy;
        const uint32_t z_min = nz ? qhz : qlz, z_max = nz ? qlz : qhz;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float tminx = fma_((float)((x_min >> (j * 8)) & 0xffu), adjx, orgx);
            const float tminy = fma_((float)((y_min >> (j * 8)) & 0xffu), adjy, orgy);
            const float tminz = fma_((float)((z_min >> (j * 8)) & 0xffu), adjz, orgz);
            const float tmaxx = fma_((float)((x_max >> (j * 8)) & 0xffu), adjx, orgx);
            const float tmaxy = fma_((float)((y_max >> (j * 8)) & 0xffu), adjy, orgy);
            const float tmaxz = fma_((float)((z_max >> (j * 8)) & 0xffu), adjz, orgz);
            const float tmin = fmaxf(fmaxf(tminx, tminy), fmaxf(tminz, 1e-8f));
            // min(tmaxz, t_max) as a plain v_min_f32 without the per-step canonicalize fminf adds: t_max is
            // never a signalling NaN -- FarPlane (tt_trace_closest rejects a NaN) or an accepted t in the
            // closest-hit kernel, the ray's distance canonicalized at ray start in the any-hit kernel
            float tmaxz_c;
            asm("v_min_f32 %0, %1, %2" : "=v"(tmaxz_c) : "v"(tmaxz), "v"(max_distance));
            const float tmax = fminf(fminf(tmaxx, tmaxy), tmaxz_c);
            // child_bits byte j << bit_index byte j in ONE v_lshlrev_b32_sdwa (both operands byte-selected)
            uint32_t bits;
            if (j == 0)
                asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0"
                    : "=v"(bits) : "v"(bit_index4), "v"(child_bits4));
            else if (j == 1)
                asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1"
                    : "=v"(bits) : "v"(bit_index4), "v"(child_bits4));
            else if (j == 2)
                asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2"
                    : "=v"(bits) : "v"(bit_index4), "v"(child_bits4));
            else
                asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3"
                    : "=v"(bits) : "v"(bit_index4), "v"(child_bits4));
            hit_mask |= (tmin < tmax) ? bits : 0u;
        }
    }
    return hit_mask;
}

struct Best {
    float t, u, v;
    int32_t mesh_id, tri_id;
};

// IntersectTriangle — IntersectionKernels.compute:14-57 (Moller-Trumbore on pos0/edges).
// Evaluated branch-free; the accept predicate is exactly the reference's nested conditions.
// ------------------------------------------------------- alpha atlas (row f3, pinned filtering)
// AlignUV — CommonData.cginc:569-591 (Rotation 0, IsAlbedo false)
__device__ __forceinline__ float2 align_uv(float bu, float bv, const int32_t* tex, const float* scale) {
    if (tex[0] <= 0) return make_float2(-1.0f, -1.0f);
    const float dx = (float)(((uint32_t)tex[0]) & 0x7FFFu) / 16384.0f;
    const float dy = (float)(((uint32_t)tex[0]) >> 15) / 16384.0f;
    const float dz = (float)(((uint32_t)tex[1]) & 0x7FFFu) / 16384.0f;
    const float dw = (float)(((uint32_t)tex[1]) >> 15) / 16384.0f;
    float x = bu * scale[0] + scale[2];
    float y = bv * scale[1] + scale[3];
    x = x < 0.0f ? 1.0f - fmodf(fabsf(x), 1.0f) : fmodf(fabsf(x), 1.0f);
    y = y < 0.0f ? 1.0f - fmodf(fabsf(y), 1.0f) : fmodf(fabsf(y), 1.0f);
    return make_float2(x * (dx - dz) + dz, y * (dy - dw) + dw);
}
__device__ __forceinline__ float2 align_uv(float2 b, const CutoutMat& m) { return align_uv(b.x, b.y, m.alpha_tex, m.scale); }
__device__ __forceinline__ int atlas_clamp(float c, uint32_t n) { return (int)fminf(fmaxf(c, 0.0f), (float)(n - 1u)); }
__device__ __forceinline__ float atlas_texel(const MatView& M, int x, int y) {
    return (float)M.atlas[(size_t)y * M.atlas_w + (size_t)x] / 255.0f;
}
// SampleLevel(my_point_clamp_sampler, uv, 0)
__device__ __forceinline__ float sample_point(const MatView& M, float2 uv) {
    return atlas_texel(M, atlas_clamp(floorf(uv.x * (float)M.atlas_w), M.atlas_w),
                       atlas_clamp(floorf(uv.y * (float)M.atlas_h), M.atlas_h));
}
// SampleLevel(my_linear_clamp_sampler, uv, 0)
__device__ __forceinline__ float sample_linear(const MatView& M, float2 uv) {
    const float x = uv.x * (float)M.atlas_w - 0.5f, y = uv.y * (float)M.atlas_h - 0.5f;
    const float x0 = floorf(x), y0 = floorf(y);
    const float fx = x - x0, fy = y - y0;
    const int ix0 = atlas_clamp(x0, M.atlas_w), ix1 = atlas_clamp(x0 + 1.0f, M.atlas_w);
    const int iy0 = atlas_clamp(y0, M.atlas_h), iy1 = atlas_clamp(y0 + 1.0f, M.atlas_h);
    const float a = atlas_texel(M, ix0, iy0) * (1.0f - fx) + atlas_texel(M, ix1, iy0) * fx;
    const float b = atlas_texel(M, ix0, iy1) * (1.0f - fx) + atlas_texel(M, ix1, iy1) * fx;
    return a * (1.0f - fy) + b * fy;
}
// IEEE binary16 -> binary32 (exact; v_cvt_f32_f16)
__device__ __forceinline__ float half_bits_to_float(uint32_t h) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
}
// _TextureAtlas.SampleLevel(my_point_clamp_sampler, uv, 0).xyz on the decoded RGBA half atlas
__device__ __forceinline__ float3 sample_tex_point(const MatView& M, float2 uv) {
    const int x = atlas_clamp(floorf(uv.x * (float)M.tex_w), M.tex_w);
    const int y = atlas_clamp(floorf(uv.y * (float)M.tex_h), M.tex_h);
    const uint2 t = M.tex[(size_t)y * M.tex_w + (size_t)x];
    return make_float3(half_bits_to_float(t.x & 0xffffu), half_bits_to_float(t.x >> 16),
                       half_bits_to_float(t.y & 0xffffu));
}
// StainedGlassShadows tint factor of a glass surface (CommonData.cginc:621-622):
// surfaceColor * (texel.xyz + 2) / 3 per component, IEEE division (pinned).
__device__ __forceinline__ float3 glass_tint(const MatView& M, const GlassMat& g, float2 buv) {
    const float3 x = sample_tex_point(M, align_uv(buv.x, buv.y, g.albedo_tex, g.scale));
    return make_float3((g.color[0] * (x.x + 2.0f)) / 3.0f, (g.color[1] * (x.y + 2.0f)) / 3.0f,
                       (g.color[2] * (x.z + 2.0f)) / 3.0f);
}

// BaseUv = tex0 * (1 - u - v) + texedge1 * u + texedge2 * v (IntersectionKernels.compute:37)
__device__ __forceinline__ float2 base_uv(const MatView& M, int32_t tri_id, float u, float v) {
    const float2* t = reinterpret_cast<const float2*>(reinterpret_cast<const char*>(M.raw + tri_id) + 60);
    const float2 t0 = t[0], t1 = t[1], t2 = t[2];
    const float w = 1.0f - u - v;
    return make_float2(t0.x * w + t1.x * u + t2.x * v, t0.y * w + t1.y * u + t2.y * v);
}

// One triangle against the ray: `cand` = the reference's geometric accept (u, v range and
// 0 < t < best_t), `accept` = cand and the material checks passed (the record is taken).
struct TriCand {
    float t, u, v;
    bool cand, accept;
};
// The 36 B of positions (+ MatDat when materials are checked) of one triangle: two 16-B loads and
// a 4- or 8-B one.
struct TriData {
    uint4 a, b;
    uint2 c;
};
template <bool MATCHECK>
__device__ __forceinline__ TriData triangle_load(__amdgpu_buffer_rsrc_t tris, int32_t tri_id) {
    const uint32_t to = tri_offset((uint32_t)tri_id);
    TriData d;
    d.a = buffer_load16<TT_TRI_CPOL>(tris, to);
    d.b = buffer_load16<TT_TRI_CPOL>(tris, to + 16u);
    if (MATCHECK) {
        d.c = buffer_load8<TT_TRI_CPOL>(tris, to + 32u);
    } else {
        d.c.x = buffer_load4<TT_TRI_CPOL>(tris, to + 32u);
        d.c.y = 0u;
    }
    return d;
}
// IgnoreBackfacing (IntersectionKernels.compute:46): dot(normalize(cross(normalize(e1), normalize(e2))),
// dir) <= 0, normalize(v) = v * (1 / sqrt(dot(v, v))) with the pinned dot / cross.
__device__ __forceinline__ float3 normalize_pinned(float x, float y, float z) {
    const float inv = 1.0f / sqrtf(fma_(z, z, fma_(y, y, x * x)));
    return make_float3(x * inv, y * inv, z * inv);
}
__device__ __forceinline__ bool backfacing(float e1x, float e1y, float e1z, float e2x, float e2y, float e2z,
                                           const LaneRay& r) {
    const float3 a = normalize_pinned(e1x, e1y, e1z), b = normalize_pinned(e2x, e2y, e2z);
    const float3 n = normalize_pinned(fma_(a.y, b.z, -(a.z * b.y)), fma_(a.z, b.x, -(a.x * b.z)),
                                      fma_(a.x, b.y, -(a.y * b.x)));
    return fma_(n.z, r.dz, fma_(n.y, r.dy, n.x * r.dx)) <= 0.0f;
}

template <bool MATCHECK>
__device__ __forceinline__ TriCand triangle_test(const TriData& d, const MatView& M, bool bounce0, uint32_t tflags,
                                                 int32_t tri_id, int32_t mat_offset, const LaneRay& r, float best_t) {
    const uint4 a = d.a, b = d.b;
    const uint2 c = d.c;
    const float p0x = __uint_as_float(a.x), p0y = __uint_as_float(a.y), p0z = __uint_as_float(a.z);
    const float e1x = __uint_as_float(a.w), e1y = __uint_as_float(b.x), e1z = __uint_as_float(b.y);
    const float e2x = __uint_as_float(b.z), e2y = __uint_as_float(b.w), e2z = __uint_as_float(c.x);
    // h = cross(d, e2); a = dot(e1, h)
    const float hx = fma_(r.dy, e2z, -(r.dz * e2y));
    const float hy = fma_(r.dz, e2x, -(r.dx * e2z));
    const float hz = fma_(r.dx, e2y, -(r.dy * e2x));
    const float aa = fma_(e1z, hz, fma_(e1y, hy, e1x * hx));
    const float f = rcp_rn(aa);
    const float sx = r.ox - p0x, sy = r.oy - p0y, sz = r.oz - p0z;
    const float u = f * fma_(sz, hz, fma_(sy, hy, sx * hx));
    // q = cross(s, e1)
    const float qx = fma_(sy, e1z, -(sz * e1y));
    const float qy = fma_(sz, e1x, -(sx * e1z));
    const float qz = fma_(sx, e1y, -(sy * e1x));
    const float v = f * fma_(r.dz, qz, fma_(r.dy, qy, r.dx * qx));
    const float t = f * fma_(e2z, qz, fma_(e2y, qy, e2x * qx));
    TriCand R;
    R.t = t;
    R.u = u;
    R.v = v;
    // IntersectionKernels.compute:29-31: (u >= 0 && u <= 1) && (v >= 0 && u + v <= 1) && (t > 0 && t < best).
    // u <= 1 is implied by v >= 0 && fl(u + v) <= 1 (v >= 0 gives u + v >= u, rounding is monotonic and u
    // is representable; an infinite or NaN u fails u + v <= 1), so it is not evaluated: same predicate.
    R.cand = (u >= 0.0f) && (v >= 0.0f && u + v <= 1.0f) && (t > 0.0f && t < best_t);
    R.accept = R.cand;
    if (MATCHECK && R.accept) {
        // _Materials[MatOffset + MatDat]; an out-of-range StructuredBuffer read returns zeros in
        // D3D (no flags, MatType 0). Cutout alpha test (:35-40), then Invisible at CurBounce == 0 (:48).
        const uint32_t mi = (uint32_t)(mat_offset + (int32_t)c.y);
        const uint32_t w = mi < M.n_mat ? M.word[mi] : 0u;
        if ((w >> TT_MATWORD_CUTOUT) & 1u) {
            const CutoutMat cm = M.cut[mi];
            if (sample_linear(M, align_uv(base_uv(M, tri_id, u, v), cm)) < cm.cutoff) R.accept = false;
        }
        const bool glass = (w >> TT_MATWORD_GLASS) & 1u;  // specTrans == 1
        if ((tflags & TT_TRACE_IGNORE_GLASS) && glass) R.accept = false;  // :42-44
        if ((tflags & TT_TRACE_IGNORE_BACKFACING) && bounce0 && !glass && R.accept &&  // :45-47
            backfacing(e1x, e1y, e1z, e2x, e2y, e2z, r))
            R.accept = false;
        if (bounce0 && ((w >> TT_FLAG_INVISIBLE) & 1u)) R.accept = false;
    }
    return R;
}
template <bool MATCHECK>
__device__ __forceinline__ TriCand triangle_candidate(__amdgpu_buffer_rsrc_t tris, const MatView& M, bool bounce0,
                                                      uint32_t tflags, int32_t tri_id, int32_t mat_offset,
                                                      const LaneRay& r, float best_t) {
    return triangle_test<MATCHECK>(triangle_load<MATCHECK>(tris, tri_id), M, bounce0, tflags, tri_id, mat_offset, r,
                                   best_t);
}

template <bool MATCHECK>
__device__ __forceinline__ bool intersect_triangle(__amdgpu_buffer_rsrc_t tris, const MatView& M, bool bounce0, uint32_t tflags,
                                                   int32_t tri_id, int32_t mesh_id, int32_t mat_offset,
                                                   const LaneRay& r, Best& best) {
    const TriCand c = triangle_candidate<MATCHECK>(tris, M, bounce0, tflags, tri_id, mat_offset, r, best.t);
    if (c.accept) {
        best.t = c.t;
        best.u = c.u;
        best.v = c.v;
        best.mesh_id = mesh_id;
        best.tri_id = tri_id;
    }
    return c.cand;  // counted as an "accept" (candidate passed the t test) before the material check
}

// ------------------------------------------------------------------ ray scheduler
// The work range is cut into TT_SEGS segments of whole 64-ray tiles; blocks start on segment
// blockIdx % TT_SEGS (one per XCD under round-robin placement, for L2 locality). A dequeue is ONE
// returning atomicAdd on the segment's counter (counted in rays): a wave reserves TT_CHUNK_BIG rays
// (fewer atomics; the surplus waits in the wave's pool). A wave whose segment is exhausted probes the others starting at an offset
// derived from its wave id, so thieves spread over all counters instead of converging on one
// (measured, tools/diag_tl.py: convergent stealing serialised thousands of atomics on one word).
__device__ __forceinline__ uint32_t seg_lo(uint32_t n_tiles, uint32_t seg) {
    return (uint32_t)(((uint64_t)n_tiles * seg / TT_SEGS) << 6);
}
struct SegState {
    uint32_t seg;   // segment this wave dequeues from
    uint32_t dead;  // bit k: segment k seen exhausted by this wave
    uint32_t est;   // this wave's last known counter value of `seg`
};
// Reserves up to max(need, chunk) rays; returns the count (0 once every segment is exhausted).
__device__ __forceinline__ uint32_t sched_reserve(TraceControl* ctl, uint32_t n_rays, uint32_t n_tiles, uint32_t lane,
                                                  uint32_t need, uint32_t wave_id, SegState& S, uint32_t& base) {
    while (S.dead != (1u << TT_SEGS) - 1u) {
        const uint32_t lo = seg_lo(n_tiles, S.seg);
        const uint32_t hi = min(seg_lo(n_tiles, S.seg + 1), n_rays);
        const uint32_t len = hi > lo ? hi - lo : 0u;
        const uint32_t want = max(need, (uint32_t)TT_CHUNK_BIG);
        uint32_t off = 0;
        TT_DB(3);
        if (lane == 0) off = atomicAdd(&ctl->seg_ticket[S.seg * 32u], want);
        off = __builtin_amdgcn_readfirstlane(off);
        if (off < len) {
            S.est = off + want;
            base = lo + off;
            return min(want, len - off);
        }
        S.dead |= 1u << S.seg;
        // next live segment, scanning from a per-wave offset
        const uint32_t start = (S.seg + 1u + wave_id % (TT_SEGS - 1u)) % TT_SEGS;
#pragma unroll
        for (uint32_t k = 0; k < TT_SEGS; k++) {
            const uint32_t c = (start + k) % TT_SEGS;
            if (!((S.dead >> c) & 1u)) {
                S.seg = c;
                break;
            }
        }
        S.est = 0;
    }
    return 0u;
}

// Zeroes the next launch's control block (block 0; plain stores, no fence: the kernel boundary
// orders them before the next launch on the stream).
__device__ __forceinline__ void zero_next_control(TraceControl* next, uint32_t tid) {
    if (blockIdx.x == 0 && next) {
        uint32_t* w = reinterpret_cast<uint32_t*>(next);
        for (uint32_t i = tid; i < (uint32_t)(sizeof(TraceControl) / 4); i += TT_BLOCK) w[i] = 0u;
    }
}

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, TT_WAVE);
    return v;
}

}  // namespace

// Traversal stack: entries [0, TT_LDS_STACK) in LDS s_stack[entry][thread] (64 distinct banks per
// wave access), deeper entries in a global spill area [entry][grid thread]. Expect in scope:
// s_stack, spill, spill_stride, gtid, tid, stack_size.
#if TT_PUSH_FAST  // one compare on the common path (an LDS entry is free); overflow / spill only beyond it
#define TT_PUSH(val, ok)                                                            \
    do {                                                                            \
        if (TT_LDS_STACK >= TT_STACK_SIZE || stack_size < TT_LDS_STACK) {           \
            if (TT_LDS_STACK >= TT_STACK_SIZE && stack_size == TT_STACK_SIZE) {     \
                ok = false;                                                         \
            } else {                                                                \
                s_stack[stack_size][tid] = (val);                                   \
                stack_size++;                                                       \
            }                                                                       \
        } else if (stack_size == TT_STACK_SIZE) {                                   \
            ok = false;                                                             \
        } else {                                                                    \
            spill[(size_t)(stack_size - TT_LDS_STACK) * spill_stride + gtid] = (val); \
            stack_size++;                                                           \
        }                                                                           \
    } while (0)
#else
#define TT_PUSH(val, ok)                                                            \
    do {                                                                            \
        if (stack_size == TT_STACK_SIZE) {                                          \
            ok = false;                                                             \
        } else {                                                                    \
            if (TT_LDS_STACK >= TT_STACK_SIZE || stack_size < TT_LDS_STACK)         \
                s_stack[stack_size][tid] = (val);                                   \
            else                                                                    \
                spill[(size_t)(stack_size - TT_LDS_STACK) * spill_stride + gtid] = (val); \
            stack_size++;                                                           \
        }                                                                           \
    } while (0)
#endif
#define TT_POP(dst)                                                                 \
    do {                                                                            \
        --stack_size;                                                               \
        if (TT_LDS_STACK >= TT_STACK_SIZE || stack_size < TT_LDS_STACK)             \
            dst = s_stack[stack_size][tid];                                         \
        else                                                                        \
            dst = spill[(size_t)(stack_size - TT_LDS_STACK) * spill_stride + gtid]; \
    } while (0)

#endif  // TT_TRAVERSE_H
