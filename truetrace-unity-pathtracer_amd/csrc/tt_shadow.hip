// tt_shadow.hip — gfx950 any-hit CWBVH8 visibility traversal (replaces kernel_shadow,
// TrueTrace/Resources/MainCompute/IntersectionKernels.compute:264-505, HardwareRT off).
//
// Same persistent-wave machinery as the closest-hit kernel (tt_trace.hip): per-XCD segment
// dequeues, in-place lane refill, LDS traversal stack. Differences that follow the reference:
//  * the culling distance is the fixed |t| of the shadow ray (max_distance, :366), not a
//    shrinking best hit;
//  * the first occluder ends the ray (:441-454): t = 0 is written back to ShadowRaysBuffer;
//  * triangle_intersect_shadow (CommonData.cginc:593-634) reads the material BEFORE the t-range
//    test and ignores IsBackground / ShadowCaster surfaces; Cutout runs the point-sampled alpha
//    test; glass (specTrans == 1) never occludes and tints the throughput through the texture
//    atlas (stained-glass shadows), in traversal order;
//  * the same cooperative drain phase as the closest-hit kernel (tt_wide.h): once the queue is dry
//    the live rays regroup into 2/4/8-lane groups; a triangle pass tests up to G of the leaf's
//    triangles and the ray is occluded if any of them occludes (what the sequential loop, which
//    stops at the first occluder, concludes as well).
//  * a ray that reaches |t| writes NEEPosA (bounce 0) and the GlobalColors / CacheBuffer
//    accumulations of :457-485 (Direct, Indirect, PrimaryNEERay, CurrentIlluminance; both the
//    RadianceCache and the plain define set, encoders pinned in tt_encode.h);
//  * TT_SHADOW_VISIBILITY_CHECK: VisabilityCheckCompute (CommonData.cginc:710-819) -- the Reps
//    bound counts as visible and only the visibility is written.
#include "tt_encode.h"
#include "tt_wide.h"

namespace {

// triangle_intersect_shadow — CommonData.cginc:593-634. Returns true for an occluder.
// A glass surface (specTrans == 1) never occludes; it multiplies `thr` by its tint (:617-625).
template <bool MATCHECK>
__device__ __forceinline__ bool shadow_triangle(__amdgpu_buffer_rsrc_t tris, const MatView& M, int32_t tri_id,
                                                int32_t mat_offset, const LaneRay& r, float max_distance,
                                                float3& thr) {
    const uint32_t to = tri_offset((uint32_t)tri_id);
    const uint4 a = buffer_load16(tris, to), b = buffer_load16(tris, to + 16u);
    uint2 c;
    if (MATCHECK) {
        c = buffer_load8(tris, to + 32u);
    } else {
        c.x = buffer_load4(tris, to + 32u);
        c.y = 0u;
    }
    const float p0x = __uint_as_float(a.x), p0y = __uint_as_float(a.y), p0z = __uint_as_float(a.z);
    const float e1x = __uint_as_float(a.w), e1y = __uint_as_float(b.x), e1z = __uint_as_float(b.y);
    const float e2x = __uint_as_float(b.z), e2y = __uint_as_float(b.w), e2z = __uint_as_float(c.x);
    const float hx = fma_(r.dy, e2z, -(r.dz * e2y));
    const float hy = fma_(r.dz, e2x, -(r.dx * e2z));
    const float hz = fma_(r.dx, e2y, -(r.dy * e2x));
    const float aa = fma_(e1z, hz, fma_(e1y, hy, e1x * hx));
    const float f = rcp_rn(aa);
    const float sx = r.ox - p0x, sy = r.oy - p0y, sz = r.oz - p0z;
    const float u = f * fma_(sz, hz, fma_(sy, hy, sx * hx));
    const float qx = fma_(sy, e1z, -(sz * e1y));
    const float qy = fma_(sz, e1x, -(sx * e1z));
    const float qz = fma_(sx, e1y, -(sy * e1x));
    const float v = f * fma_(r.dz, qz, fma_(r.dy, qy, r.dx * qx));
    const float t = f * fma_(e2z, qz, fma_(e2y, qy, e2x * qx));
    const bool in_tri = (u >= 0.0f) && (v >= 0.0f && u + v <= 1.0f);  // u <= 1 implied (tt_traverse.h)
    bool occ = in_tri && (t > 0.0f && t < max_distance);
    if (MATCHECK && in_tri) {
        // IsBackground / ShadowCaster surfaces never occlude (:612); Cutout with the point sampler
        // (:613-616); out-of-range material = zeros
        const uint32_t mi = (uint32_t)(mat_offset + (int32_t)c.y);
        const uint32_t w = mi < M.n_mat ? M.word[mi] : 0u;
        const bool glass = (w >> TT_MATWORD_GLASS) & 1u, cutout = (w >> TT_MATWORD_CUTOUT) & 1u;
        if (((w >> TT_FLAG_IS_BACKGROUND) | (w >> TT_FLAG_SHADOW_CASTER)) & 1u) {
            occ = false;
        } else if (glass || (occ && cutout)) {
            // the alpha test comes first (:616); a glass surface that passes it tints (:621-622)
            const float2 buv = base_uv(M, tri_id, u, v);
            bool rejected = false;
            if (cutout) {
                const CutoutMat cm = M.cut[mi];
                rejected = sample_point(M, align_uv(buv, cm)) < cm.cutoff;
            }
            if (rejected) {
                occ = false;
            } else if (glass) {
                const float3 f = glass_tint(M, M.glass[mi], buv);
                thr.x = thr.x * f.x;
                thr.y = thr.y * f.y;
                thr.z = thr.z * f.z;
                occ = false;
            }
        }
    }
    return occ;
}

struct ShadowWide {
    LaneRay ray, wray;
    float max_distance;
    float3 thr;
    uint2 cg, tg;
    uint32_t oct;
    int32_t stack_size, tlas_ss, NodeOffset, TriOffset, MatOffset, Reps;
    uint32_t ray_index, scol, gcol;
    bool active;
};

struct ShadowCounters {
    uint32_t &nodes, &tris, &blas, &occ, &vis, &reps, &ovf;
};

template <int GN>
__device__ __forceinline__ void regroup_shadow(ShadowWide& s, uint64_t lead, uint32_t lane) {
    const uint32_t grp = lane / GN;
    uint32_t src = 0;
    bool has = false;
    uint64_t m = lead;
    for (uint32_t r = 0; m; r++) {  // wave-uniform: at most 32 leaders
        const uint32_t b = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        if (grp == r) {
            src = b;
            has = true;
        }
    }
    shfl_ray(s.ray, src);
    shfl_ray(s.wray, src);
    s.max_distance = shfl_f(s.max_distance, src);
    s.thr.x = shfl_f(s.thr.x, src);
    s.thr.y = shfl_f(s.thr.y, src);
    s.thr.z = shfl_f(s.thr.z, src);
    s.cg.x = shfl_u(s.cg.x, src);
    s.cg.y = shfl_u(s.cg.y, src);
    s.tg.x = shfl_u(s.tg.x, src);
    s.tg.y = shfl_u(s.tg.y, src);
    s.oct = shfl_u(s.oct, src);
    s.stack_size = shfl_i(s.stack_size, src);
    s.tlas_ss = shfl_i(s.tlas_ss, src);
    s.NodeOffset = shfl_i(s.NodeOffset, src);
    s.TriOffset = shfl_i(s.TriOffset, src);
    s.MatOffset = shfl_i(s.MatOffset, src);
    s.Reps = shfl_i(s.Reps, src);
    s.ray_index = shfl_u(s.ray_index, src);
    s.scol = shfl_u(s.scol, src);
    s.gcol = shfl_u(s.gcol, src);
    s.active = has;
}

// The drain loop of the any-hit kernel for groups of G lanes (tt_wide.h's wide_phase with the
// any-hit step): `occlude(st)` / `reach(st)` / `exhaust(st)` write a finished ray's outputs (group's
// first lane only).
template <bool STATS, bool MATCHECK, int G, class Occ, class Reach, class Exh>
__device__ void shadow_wide_phase(const ShadowArgs& A, ShadowWide& st, uint2 (*s_stack)[TT_BLOCK],
                                  uint2* __restrict__ spill, uint32_t spill_stride, __amdgpu_buffer_rsrc_t nodes,
                                  __amdgpu_buffer_rsrc_t tris, uint32_t lane, ShadowCounters C, Occ& occlude,
                                  Reach& reach, Exh& exhaust) {
    const uint32_t sub = lane & (G - 1);
    const uint32_t tid = st.scol, gtid = st.gcol;  // the stack the TT_PUSH / TT_POP macros address
    int32_t& stack_size = st.stack_size;
    while (true) {
        const uint64_t lead = __ballot(st.active && sub == 0u);
        const uint32_t n = (uint32_t)__popcll(lead);
        if (n == 0u) return;
        if constexpr (G < 8) {
            if (n * (2 * G) <= TT_WAVE) {
                regroup_shadow<2 * G>(st, lead, lane);
                shadow_wide_phase<STATS, MATCHECK, 2 * G>(A, st, s_stack, spill, spill_stride, nodes, tris, lane, C,
                                                          occlude, reach, exhaust);
                return;
            }
        }
        // ------------------------------------------------------------- node phase
        if (st.active && st.tg.y == 0u) {
            if (st.Reps >= TT_MAX_REPS) {  // :373 loop bound
                st.active = false;
                if (sub == 0u) {
                    if (STATS) C.reps++;
                    exhaust(st);
                }
            } else if (st.cg.y & 0xff000000u) {  // :374-403
                const uint32_t cio = firstbithigh(st.cg.y);
                const uint32_t slot = (cio - 24u) ^ (st.oct & 0xffu);
                const uint32_t rel = __builtin_popcount(st.cg.y & ~(0xffffffffu << slot));
                const uint32_t child = st.cg.x + rel;
                st.cg.y &= ~(1u << cio);
                bool ok = true;
                if (st.cg.y & 0xff000000u) TT_PUSH(st.cg, ok);
                if (ok) {
                    const uint32_t no = node_offset(child);
                    const uint4 n0 = buffer_load16(nodes, no), n1 = buffer_load16(nodes, no + 16u),
                                n2 = buffer_load16(nodes, no + 32u), n3 = buffer_load16(nodes, no + 48u),
                                n4 = buffer_load16(nodes, no + 64u);
                    const uint32_t hitmask =
                        group_or<G>(node_intersect_part<G>(n0, n1, n2, n3, n4, st.ray, st.oct, st.max_distance, sub));
                    st.cg.y = (hitmask & 0xff000000u) | (n0.w >> 24);
                    st.tg.y = hitmask & 0x00ffffffu;
                    st.cg.x = n1.x + (uint32_t)st.NodeOffset;
                    st.tg.x = n1.y + (uint32_t)st.TriOffset;
                    st.Reps++;
                    if (STATS && sub == 0u) C.nodes++;
                } else {
                    st.active = false;
                    if (sub == 0u) {
                        if (STATS) C.ovf++;
                        TT_REPORT_OVERFLOW(A);
                    }
                }
            } else {  // :404-407
                st.tg = st.cg;
                st.cg = make_uint2(0u, 0u);
            }
            if (st.active && st.tg.y != 0u && st.tlas_ss == -1) {  // :411-435 TLAS leaf -> BLAS
                const uint32_t mo = firstbithigh(st.tg.y);
                st.tg.y &= ~(1u << mo);
                const float4* mp = reinterpret_cast<const float4*>(A.leaf + (st.tg.x + mo));  // LeafMesh
                const float4 m0 = mp[0], m1 = mp[1], m2 = mp[2];
                const int4 mo4 = reinterpret_cast<const int4*>(mp)[3];
                st.NodeOffset = mo4.y;
                st.TriOffset = mo4.x;
                bool ok = true;
                if (st.tg.y != 0u) TT_PUSH(st.tg, ok);
                if (ok && (st.cg.y & 0xff000000u)) TT_PUSH(st.cg, ok);
                if (ok) {
                    st.tlas_ss = stack_size;
                    st.MatOffset = mo4.z;
                    const LaneRay& ray = st.ray;
                    LaneRay nr;
                    nr.dx = fma_(m0.z, ray.dz, fma_(m0.y, ray.dy, m0.x * ray.dx));
                    nr.dy = fma_(m1.z, ray.dz, fma_(m1.y, ray.dy, m1.x * ray.dx));
                    nr.dz = fma_(m2.z, ray.dz, fma_(m2.y, ray.dy, m2.x * ray.dx));
                    nr.ox = fma_(m0.z, ray.oz, fma_(m0.y, ray.oy, m0.x * ray.ox)) + m0.w;
                    nr.oy = fma_(m1.z, ray.oz, fma_(m1.y, ray.oy, m1.x * ray.ox)) + m1.w;
                    nr.oz = fma_(m2.z, ray.oz, fma_(m2.y, ray.oy, m2.x * ray.ox)) + m2.w;
                    nr.ix = rcp_rn(nr.dx);
                    nr.iy = rcp_rn(nr.dy);
                    nr.iz = rcp_rn(nr.dz);
                    st.ray = nr;
                    st.oct = octant_inv4(st.ray);
                    st.cg = make_uint2((uint32_t)mo4.w, 0x80000000u);
                    if (STATS && sub == 0u) C.blas++;
                } else {
                    st.active = false;
                    if (sub == 0u) {
                        if (STATS) C.ovf++;
                        TT_REPORT_OVERFLOW(A);
                    }
                }
                st.tg.y = 0u;
            }
        }

        // --------------------------------------------------------- triangle phase
        // :436-446: highest bit first until the first occluder; lane `sub` takes the sub-th triangle
        if (st.active && st.tg.y != 0u) {
            uint32_t m = st.tg.y;
#pragma unroll
            for (uint32_t k = 0; k + 1 < (uint32_t)G; k++)
                if (k < sub && m) m &= ~(1u << firstbithigh(m));
            const bool has = m != 0u;
            bool occ = false;
            float3 f = make_float3(1.0f, 1.0f, 1.0f);  // this lane's glass tint (1: none)
            if (has)
                occ = shadow_triangle<MATCHECK>(tris, A.mat, (int32_t)(st.tg.x + firstbithigh(m)), st.MatOffset, st.ray,
                                                st.max_distance, f);
            // the first occluder in the reference's order (lowest sub), G if none
            const uint32_t first = (uint32_t)group_min_u64<G>(occ ? (uint64_t)sub : (uint64_t)G);
            if (STATS && sub == 0u)
                C.tris += first < (uint32_t)G ? first + 1u : min((uint32_t)__builtin_popcount(st.tg.y), (uint32_t)G);
            if (first < (uint32_t)G) {  // :449-454
                st.active = false;
                if (sub == 0u) {
                    if (STATS) C.occ++;
                    occlude(st);
                }
            } else {
                if (MATCHECK) {  // the tints in the reference's order (lane k holds the k-th triangle)
                    const uint32_t base = lane & ~(uint32_t)(G - 1);
#pragma unroll
                    for (uint32_t k = 0; k < (uint32_t)G; k++) {
                        st.thr.x = st.thr.x * shfl_f(f.x, base + k);
                        st.thr.y = st.thr.y * shfl_f(f.y, base + k);
                        st.thr.z = st.thr.z * shfl_f(f.z, base + k);
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < (uint32_t)G; k++)
                    if (st.tg.y) st.tg.y &= ~(1u << firstbithigh(st.tg.y));
            }
        }

        // ----------------------------------------- advance: pop / finish (:456-494)
        if (st.active && st.tg.y == 0u && (st.cg.y & 0xff000000u) == 0u) {
            if (stack_size != 0) {
                if (stack_size == st.tlas_ss) {
                    st.NodeOffset = (int32_t)A.tlas_base;
                    st.TriOffset = 0;
                    st.tlas_ss = -1;
                    st.ray = st.wray;
                    st.oct = octant_inv4(st.ray);
                }
                TT_POP(st.cg);
            } else {
                st.active = false;
                if (sub == 0u) {
                    if (STATS) C.vis++;
                    reach(st);
                }
            }
        }
    }
}

}  // namespace

// IND: device-resident ray count (tt_trace_shadow_ex_indirect), its own kernel (tt_shadow_kernel_indirect)
template <bool STATS, bool MATCHECK, bool IND>
__device__ __forceinline__ void shadow_body(const ShadowArgs& A) {
    __shared__ uint2 s_stack[TT_LDS_STACK][TT_BLOCK];
    const uint32_t tid = threadIdx.x;
    const uint32_t gtid = blockIdx.x * TT_BLOCK + tid;
    const uint32_t spill_stride = gridDim.x * TT_BLOCK;
    uint2* __restrict__ spill = A.spill;
    (void)gtid;
    (void)spill_stride;
    (void)spill;
    const uint32_t lane = tid & (TT_WAVE - 1);

    uint32_t pool_next = 0, pool_end = 0, more = 1;
    const uint32_t wave_id = blockIdx.x * (TT_BLOCK / TT_WAVE) + (tid >> 6);
    SegState S{blockIdx.x % TT_SEGS, 0u, 0u};
    const uint32_t n_rays = IND ? launch_ray_count(A) : A.n_rays;
    const uint32_t n_tiles = (n_rays + 63u) >> 6;
    const __amdgpu_buffer_rsrc_t nodes = buffer_rsrc(A.nodes, A.n_nodes * (uint32_t)TT_NODE_STRIDE);
    const __amdgpu_buffer_rsrc_t tris = buffer_rsrc(A.tris, A.n_tris * (uint32_t)sizeof(TriPos));

    // a lane without a ray holds tg.y == TT_IDLE (as in tt_trace.hip: a live ray's pending-leaf word never
    // has bit 31 set), so each phase test is one compare of tg.y
    constexpr uint32_t TT_IDLE = 0x80000000u;
    uint32_t ray_index = 0;
    LaneRay ray{}, wray{};
    float max_distance = 0.0f;
    float3 thr = make_float3(1.0f, 1.0f, 1.0f);  // throughput (:361), scaled by glass tints
    uint2 cg = make_uint2(0u, 0u), tg = make_uint2(0u, TT_IDLE);
    uint32_t oct = 0;
    int32_t stack_size = 0, tlas_ss = -1;
    int32_t NodeOffset = 0, TriOffset = 0, MatOffset = 0, Reps = 0;
    uint32_t c_nodes = 0, c_tris = 0, c_blas = 0, c_occ = 0, c_rays = 0, c_vis = 0, c_reps = 0, c_ovf = 0;

    // a finished ray's outputs: occluded (:449-454), Reps exhausted (:373), reached the light (:457-485)
    const bool vis_check = (A.flags & TT_SHADOW_VISIBILITY_CHECK) != 0;
    auto do_occlude = [&](uint32_t ri) {
        if (!vis_check) A.rays[ri].t = 0.0f;
        if (A.visibility) A.visibility[ri] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    };
    auto do_exhaust = [&](uint32_t ri) {  // VisabilityCheckCompute returns true once its loop ends
        if (A.visibility)
            A.visibility[ri] = vis_check ? make_float4(1.0f, 1.0f, 1.0f, 1.0f) : make_float4(0.0f, 0.0f, 0.0f, -1.0f);
    };
    auto do_reach = [&](uint32_t ri, const LaneRay& w, const float3& thr) {  // TerrainExists false
        if (vis_check) {
            if (A.visibility) A.visibility[ri] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
            return;
        }
        const tt_shadow_ray& R = A.rays[ri];
        const uint32_t pix = R.PixelIndex;
        const float t = R.t;
        if (A.visibility) A.visibility[ri] = make_float4(thr.x, thr.y, thr.z, 1.0f);
        if (A.bounce == 0 && A.nee_pos && pix / A.width < A.height) {
            const float d = fabsf(t);
            A.nee_pos[pix] = make_float4(w.ox + w.dx * d, w.oy + w.dy * d, w.oz + w.dz * d, 0.0f);
        }
        if (A.bounce == 0 && t >= 0.0f && A.colors && pix / A.width < A.height) {  // Direct (:469)
            tt_col_data& C = A.colors[pix];
            C.Direct[0] = C.Direct[0] + R.illumination[0] * thr.x;
            C.Direct[1] = C.Direct[1] + R.illumination[1] * thr.y;
            C.Direct[2] = C.Direct[2] + R.illumination[2] * thr.z;
        }
        // the rest of :457-485 (CacheBuffer, Indirect, PrimaryNEERay) runs in tt_shadow_accumulate
    };

    while (true) {
        // ---------------------------------------------------------------- refill
        const uint64_t idle = __ballot((int32_t)tg.y < 0);
        // (two 32-bit SALU counts: a 64-bit count is tested with VALU v_cmp_*_u64)
        const uint32_t n_idle = (uint32_t)__builtin_popcount((uint32_t)idle) + (uint32_t)__builtin_popcount((uint32_t)(idle >> 32));
        const bool pool_dry = !more && pool_next >= pool_end;
        if (n_idle == TT_WAVE && pool_dry) break;
#if TT_WIDE
        // the queue is dry and the live rays fit in 2-lane groups: cooperative drain (tt_wide.h)
        if (pool_dry && TT_WAVE - n_idle <= TT_WIDE_ENTER) {
            ShadowWide st{ray, wray, max_distance, thr, cg, tg, oct, stack_size, tlas_ss, NodeOffset, TriOffset,
                          MatOffset, Reps, ray_index, tid, gtid, (int32_t)tg.y >= 0};
            regroup_shadow<2>(st, __ballot((int32_t)tg.y >= 0), lane);
            auto occ_w = [&](const ShadowWide& w) { do_occlude(w.ray_index); };
            auto reach_w = [&](const ShadowWide& w) { do_reach(w.ray_index, w.wray, w.thr); };
            auto exh_w = [&](const ShadowWide& w) { do_exhaust(w.ray_index); };
            shadow_wide_phase<STATS, MATCHECK, 2>(A, st, s_stack, spill, spill_stride, nodes, tris, lane,
                                                  ShadowCounters{c_nodes, c_tris, c_blas, c_occ, c_vis, c_reps, c_ovf},
                                                  occ_w, reach_w, exh_w);
            break;
        }
#endif
        if (n_idle >= TT_REFILL_MIN && !pool_dry) {
            const uint32_t avail = pool_end - pool_next;
            uint32_t new_base = 0, new_count = 0;
            if (avail < n_idle && more) {
                new_count = sched_reserve(A.ctl, n_rays, n_tiles, lane, n_idle - avail, wave_id, S, new_base);
                more = new_count > 0 ? 1u : 0u;
            }
            const uint32_t take_old = min(avail, n_idle);
            const uint32_t take_new = min(n_idle - take_old, new_count);
            const uint32_t rank = lane_prefix(idle);
            uint32_t widx = 0xffffffffu;
            if (rank < take_old) widx = pool_next + rank;
            else if (rank - take_old < take_new) widx = new_base + (rank - take_old);
            if (new_count > 0) {
                pool_next = new_base + take_new;
                pool_end = new_base + new_count;
            } else {
                pool_next += take_old;
            }
            if ((int32_t)tg.y < 0 && widx != 0xffffffffu) {  // :355-371
                ray_index = widx;
                const uint4* rp = reinterpret_cast<const uint4*>(A.rays + ray_index);
                const uint4 r0 = rp[0], r1 = rp[1];
                ray.ox = __uint_as_float(r0.x);
                ray.oy = __uint_as_float(r0.y);
                ray.oz = __uint_as_float(r0.z);
                ray.dx = __uint_as_float(r1.x);
                ray.dy = __uint_as_float(r1.y);
                ray.dz = __uint_as_float(r1.z);
                // |t| (:356); VisabilityCheckCompute takes its dist as given, throughput 0 (:732)
                // canonicalized once per ray: node_intersect's t_max clamp is a plain v_min_f32
                max_distance = __builtin_canonicalizef(vis_check ? __uint_as_float(r1.w)
                                                                 : fabsf(__uint_as_float(r1.w)));
                thr = vis_check ? make_float3(0.0f, 0.0f, 0.0f) : make_float3(1.0f, 1.0f, 1.0f);
                ray.ix = rcp_rn(ray.dx);
                ray.iy = rcp_rn(ray.dy);
                ray.iz = rcp_rn(ray.dz);
                wray = ray;
                oct = octant_inv4(ray);
                cg = make_uint2(A.tlas_base, 0x80000000u);
                tg = make_uint2(0u, 0u);
                stack_size = 0;
                tlas_ss = -1;
                NodeOffset = (int32_t)A.tlas_base;
                TriOffset = 0;
                MatOffset = 0;
                Reps = 0;
                if (STATS) c_rays++;
            }
        }

        // ------------------------------------------------------------- node phase
        if (tg.y == 0u) {
            if (Reps >= TT_MAX_REPS) {  // :373 loop bound: nothing is written
                tg.y = TT_IDLE;
                if (STATS) c_reps++;
                do_exhaust(ray_index);
            } else if (cg.y & 0xff000000u) {  // :374-403
                const uint32_t cio = firstbithigh(cg.y);
                const uint32_t slot = (cio - 24u) ^ (oct & 0xffu);
                const uint32_t rel = __builtin_popcount(cg.y & ~(0xffffffffu << slot));
                const uint32_t child = cg.x + rel;
                cg.y &= ~(1u << cio);
                bool ok = true;
                if (cg.y & 0xff000000u) TT_PUSH(cg, ok);
                if (ok) {
                    const uint32_t no = node_offset(child);
                    const uint4 n0 = buffer_load16(nodes, no), n1 = buffer_load16(nodes, no + 16u),
                                n2 = buffer_load16(nodes, no + 32u), n3 = buffer_load16(nodes, no + 48u),
                                n4 = buffer_load16(nodes, no + 64u);
                    const uint32_t hitmask = node_intersect(n0, n1, n2, n3, n4, ray, oct, max_distance);
                    cg.y = (hitmask & 0xff000000u) | (n0.w >> 24);
                    tg.y = hitmask & 0x00ffffffu;
                    cg.x = n1.x + (uint32_t)NodeOffset;
                    tg.x = n1.y + (uint32_t)TriOffset;
                    Reps++;
                    if (STATS) c_nodes++;
                } else {
                    tg.y = TT_IDLE;
                    if (STATS) c_ovf++;
                    TT_REPORT_OVERFLOW(A);
                }
            } else {  // :404-407
                tg = cg;
                cg = make_uint2(0u, 0u);
            }
            if ((int32_t)tg.y > 0 && tlas_ss == -1) {  // :411-435 TLAS leaf -> BLAS
                const uint32_t mo = firstbithigh(tg.y);
                tg.y &= ~(1u << mo);
                const float4* mp = reinterpret_cast<const float4*>(A.leaf + (tg.x + mo));  // LeafMesh
                const float4 m0 = mp[0], m1 = mp[1], m2 = mp[2];
                const int4 mo4 = reinterpret_cast<const int4*>(mp)[3];
                NodeOffset = mo4.y;
                TriOffset = mo4.x;
                bool ok = true;
                if (tg.y != 0u) TT_PUSH(tg, ok);
                if (ok && (cg.y & 0xff000000u)) TT_PUSH(cg, ok);
                tg.y = 0u;
                if (ok) {
                    tlas_ss = stack_size;
                    MatOffset = mo4.z;
                    LaneRay nr;
                    nr.dx = fma_(m0.z, ray.dz, fma_(m0.y, ray.dy, m0.x * ray.dx));
                    nr.dy = fma_(m1.z, ray.dz, fma_(m1.y, ray.dy, m1.x * ray.dx));
                    nr.dz = fma_(m2.z, ray.dz, fma_(m2.y, ray.dy, m2.x * ray.dx));
                    nr.ox = fma_(m0.z, ray.oz, fma_(m0.y, ray.oy, m0.x * ray.ox)) + m0.w;
                    nr.oy = fma_(m1.z, ray.oz, fma_(m1.y, ray.oy, m1.x * ray.ox)) + m1.w;
                    nr.oz = fma_(m2.z, ray.oz, fma_(m2.y, ray.oy, m2.x * ray.ox)) + m2.w;
                    nr.ix = rcp_rn(nr.dx);
                    nr.iy = rcp_rn(nr.dy);
                    nr.iz = rcp_rn(nr.dz);
                    ray = nr;
                    oct = octant_inv4(ray);
                    cg = make_uint2((uint32_t)mo4.w, 0x80000000u);
                    if (STATS) c_blas++;
                } else {
                    tg.y = TT_IDLE;
                    if (STATS) c_ovf++;
                    TT_REPORT_OVERFLOW(A);
                }
            }
        }

        // --------------------------------------------------------- triangle phase
        if ((int32_t)tg.y > 0) {  // :436-446, highest bit first, until the first occluder
            const uint32_t ti = firstbithigh(tg.y);
            tg.y &= ~(1u << ti);
            const bool occ =
                shadow_triangle<MATCHECK>(tris, A.mat, (int32_t)(tg.x + ti), MatOffset, ray, max_distance, thr);
            if (STATS) c_tris++;
            if (occ) {  // :449-454
                do_occlude(ray_index);
                tg.y = TT_IDLE;
                if (STATS) c_occ++;
            }
        }

        // ----------------------------------------- advance: pop / finish (:456-494)
        if (tg.y == 0u && (cg.y & 0xff000000u) == 0u) {
            if (stack_size != 0) {
                if (stack_size == tlas_ss) {
                    NodeOffset = (int32_t)A.tlas_base;
                    TriOffset = 0;
                    tlas_ss = -1;
                    ray = wray;
                    oct = octant_inv4(ray);
                }
                TT_POP(cg);
            } else {  // reached the light (TerrainExists false): :457-485
                do_reach(ray_index, wray, thr);
                tg.y = TT_IDLE;
                if (STATS) c_vis++;
            }
        }
    }

    if (STATS) {
        // stats slots as the closest-hit kernel: rays, nodes, tris, blas, hits (= occluded),
        // reps_exhausted, overflow, accepts (= reached the light)
        const uint32_t v[8] = {wave_sum(c_rays), wave_sum(c_nodes), wave_sum(c_tris), wave_sum(c_blas),
                               wave_sum(c_occ),  wave_sum(c_reps),  wave_sum(c_ovf),  wave_sum(c_vis)};
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (v[k]) atomicAdd(&A.ctl->stats[k], (unsigned long long)v[k]);
        }
    }
}

// ---------------------------------------------------------- :457-485 accumulations (row f1)
// The outputs of a ray that reached |t| beyond Direct / NEEPosA: CacheBuffer.CurrentIlluminance,
// Indirect and PrimaryNEERay, with or without the RadianceCache define (include/truetrace_hip.h).
// A streaming pass over the launch's rays after the traversal, driven by its visibility record
// (throughput.xyz, 1 = reached): it keeps the encoders' registers out of the traversal kernel.
constexpr uint32_t TT_ACC_BLOCK = 256;  // streaming pass: plain 256-thread blocks
__global__ __launch_bounds__(TT_ACC_BLOCK) void tt_shadow_accumulate(ShadowArgs A, const float4* __restrict__ vis) {
    const uint32_t ri = blockIdx.x * TT_ACC_BLOCK + threadIdx.x;
    if (ri >= launch_ray_count(A)) return;
    const float4 v = vis[ri];
    if (v.w != 1.0f) return;
    const tt_shadow_ray& R = A.rays[ri];
    const uint32_t pix = R.PixelIndex;
    if (pix / A.width >= A.height) return;  // out-of-range UAV writes are dropped
    const float t = R.t;
    const bool restir = (A.flags & TT_TRACE_USE_RESTIRGI) != 0;
    const bool rc = (A.flags & TT_SHADOW_RADIANCE_CACHE) != 0;
    const float il[3] = {R.illumination[0], R.illumination[1], R.illumination[2]};
    const float th[3] = {v.x, v.y, v.z};
    if (rc && A.cache) {  // :464
        float k[3] = {1.0f, 1.0f, 1.0f};
        if (!(!restir || t >= 0.0f)) {
            const float3 u = tt_enc::unpackRGBE(__float_as_uint(R.LuminanceIncomming));
            k[0] = u.x;
            k[1] = u.y;
            k[2] = u.z;
        }
        uint32_t& ci = A.cache[pix].CurrentIlluminance;
        const float3 d = tt_enc::DecodeRGB(ci);
        ci = tt_enc::EncodeRGB(d.x + (il[0] * th[0]) * k[0], d.y + (il[1] * th[1]) * k[1], d.z + (il[2] * th[2]) * k[2]);
    }
    if (!A.colors) return;
    tt_col_data& C = A.colors[pix];
    if (t >= 0.0f) {  // :466-474 (Direct at bounce 0 was added by the traversal kernel)
        if (A.bounce != 0 && !rc)
            for (int c = 0; c < 3; c++) C.Indirect[c] = C.Indirect[c] + il[c] * th[c];
        return;
    }
    const bool indirect = rc ? (A.bounce != 0 && (restir || C.Data[3] == (float)A.bounce))  // :477
                             : (A.bounce != 0 && (!restir && C.Data[3] == -1.0f));         // :479
    if (indirect) {
        float k[3] = {1.0f, 1.0f, 1.0f};
        if (rc && restir) {
            const float3 u = tt_enc::unpackRGBE(__float_as_uint(R.LuminanceIncomming));
            k[0] = u.x;
            k[1] = u.y;
            k[2] = u.z;
        }
        for (int c = 0; c < 3; c++) C.Indirect[c] = C.Indirect[c] + (il[c] * th[c]) * k[c];
    } else {  // :481 packRGBE(pow(unpackRGBE(PrimaryNEERay), 2.2f) + pow(illumination, rcp(2.2f)) * throughput)
        const float3 p = tt_enc::unpackRGBE(C.PrimaryNEERay);
        const float pv[3] = {p.x, p.y, p.z};
        const float inv22 = 1.0f / 2.2f;
        float o[3];
        for (int c = 0; c < 3; c++) o[c] = tt_enc::pow_pinned(pv[c], 2.2f) + tt_enc::pow_pinned(il[c], inv22) * th[c];
        C.PrimaryNEERay = tt_enc::packRGBE(o[0], o[1], o[2]);
    }
}

hipError_t tt_launch_shadow_accumulate(const ShadowArgs* a, const float4* vis, hipStream_t st) {
    hipLaunchKernelGGL(tt_shadow_accumulate, dim3((a->n_rays + TT_ACC_BLOCK - 1) / TT_ACC_BLOCK), dim3(TT_ACC_BLOCK), 0,
                       st, *a, vis);
    return hipGetLastError();
}

template <bool STATS, bool MATCHECK>
__global__ TT_BOUNDS void tt_shadow_kernel(ShadowArgs A) {
    shadow_body<STATS, MATCHECK, false>(A);
}
template <bool MATCHECK>
__global__ TT_BOUNDS void tt_shadow_kernel_indirect(ShadowArgs A) {
    shadow_body<false, MATCHECK, true>(A);
}

// ------------------------------------------------------------------ launchers
template <bool S, bool M>
static hipError_t launch_shadow(const ShadowArgs& a, uint32_t grid, hipStream_t st) {
    if constexpr (!S) {
        if (a.n_rays_dev) {
            hipLaunchKernelGGL((tt_shadow_kernel_indirect<M>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((tt_shadow_kernel<S, M>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
    return hipGetLastError();
}

hipError_t tt_launch_shadow(const ShadowArgs* a, uint32_t grid, hipStream_t st, int stats, int matcheck) {
    if (stats) return matcheck ? launch_shadow<true, true>(*a, grid, st) : launch_shadow<true, false>(*a, grid, st);
    return matcheck ? launch_shadow<false, true>(*a, grid, st) : launch_shadow<false, false>(*a, grid, st);
}

template <bool S, bool M>
static int shadow_occ() {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tt_shadow_kernel<S, M>, TT_BLOCK, 0) != hipSuccess) b = 1;
    return b;
}

// resident blocks per CU per instantiation, index stats * 2 + matcheck
void tt_shadow_occupancy_table(int* out4) {
    out4[0] = shadow_occ<false, false>();
    out4[1] = shadow_occ<false, true>();
    out4[2] = shadow_occ<true, false>();
    out4[3] = shadow_occ<true, true>();
}
