// tt_wide.h — the drain phase of the closest-hit kernel: G lanes cooperate on one ray.
//
// Once the ray queue is exhausted a persistent wave can no longer refill finished lanes, and the
// launch ends with waves whose few live rays still cost a full wave64 instruction stream per step
// (profiles/r01_diag_*: the last ~30% of a launch runs at 0.6 -> 0.1 active lanes). Here a wave
// whose live rays fit regroups them so that G = 2, 4 or 8 lanes carry each ray (all G lanes hold
// the same traversal state): the eight child slab tests of a node step are split 8/G per lane and
// OR-reduced with DPP, and a triangle pass tests up to G of the leaf's pending triangles at once
// and keeps the closest accepted one (ties: the earliest in the reference's order, which is what
// the sequential strict `t < best.t` loop selects). The per-ray visit order, culling distance,
// Reps count and stack contents are exactly the narrow kernel's, so results stay bit-identical.
// The ray keeps the LDS / spill stack column of the lane it started in.
#ifndef TT_WIDE_H
#define TT_WIDE_H
#include "tt_traverse.h"

#ifndef TT_WIDE
#define TT_WIDE 1          // 0: disable the cooperative drain phase
#endif
#ifndef TT_WIDE_ENTER
#define TT_WIDE_ENTER 32   // enter the drain phase (G = 2) once at most this many rays are live
#endif
// G = 2 lanes per ray: more than 32 live rays do not fit a wave (measured: 48 gives wrong hits)
static_assert(TT_WIDE_ENTER >= 1 && TT_WIDE_ENTER <= 32, "TT_WIDE_ENTER must be in [1, 32]");

namespace {

// everything a ray carries between steps (IntersectionKernels.compute:62-77 + bookkeeping)
struct WideState {
    LaneRay ray, wray;
    Best best;
    uint2 cg, tg;
    uint32_t oct;
    int32_t stack_size, tlas_ss, NodeOffset, TriOffset, MatOffset, mesh_id, Reps;
    uint32_t ray_index, pix;
    float col_w;
    uint32_t scol, gcol;  // LDS stack column (thread in block) and spill column (grid thread)
    bool active;
};

struct Counters {
    uint32_t &nodes, &tris, &blas, &acc, &hits, &reps, &ovf;
};

__device__ __forceinline__ uint32_t shfl_u(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ float shfl_f(float v, uint32_t src) { return __uint_as_float(shfl_u(__float_as_uint(v), src)); }
__device__ __forceinline__ int32_t shfl_i(int32_t v, uint32_t src) { return (int32_t)shfl_u((uint32_t)v, src); }

__device__ __forceinline__ void shfl_ray(LaneRay& r, uint32_t src) {
    r.ox = shfl_f(r.ox, src);
    r.oy = shfl_f(r.oy, src);
    r.oz = shfl_f(r.oz, src);
    r.dx = shfl_f(r.dx, src);
    r.dy = shfl_f(r.dy, src);
    r.dz = shfl_f(r.dz, src);
    r.ix = shfl_f(r.ix, src);
    r.iy = shfl_f(r.iy, src);
    r.iz = shfl_f(r.iz, src);
}

// Regroups the rays led by the lanes in `lead` (wave-uniform) into groups of GN consecutive lanes.
// Must run with every lane of the wave enabled (ds_bpermute reads inactive lanes as zero).
template <int GN>
__device__ __forceinline__ void regroup(WideState& s, uint64_t lead, uint32_t lane) {
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
    s.best.t = shfl_f(s.best.t, src);
    s.best.u = shfl_f(s.best.u, src);
    s.best.v = shfl_f(s.best.v, src);
    s.best.mesh_id = shfl_i(s.best.mesh_id, src);
    s.best.tri_id = shfl_i(s.best.tri_id, src);
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
    s.mesh_id = shfl_i(s.mesh_id, src);
    s.Reps = shfl_i(s.Reps, src);
    s.ray_index = shfl_u(s.ray_index, src);
    s.pix = shfl_u(s.pix, src);
    s.col_w = shfl_f(s.col_w, src);
    s.scol = shfl_u(s.scol, src);
    s.gcol = shfl_u(s.gcol, src);
    s.active = has;
}

// DPP reductions over aligned groups of G lanes (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror)
template <int G>
__device__ __forceinline__ uint32_t group_or(uint32_t v) {
    if (G >= 2) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
    if (G >= 4) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);
    if (G >= 8) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);
    return v;
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_u64(uint64_t k) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)k, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)(k >> 32), CTRL, 0xf, 0xf, false);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    return o < k ? o : k;
}
template <int G>
__device__ __forceinline__ uint64_t group_min_u64(uint64_t k) {
    if (G >= 2) k = dpp_min_u64<0xB1>(k);
    if (G >= 4) k = dpp_min_u64<0x4E>(k);
    if (G >= 8) k = dpp_min_u64<0x141>(k);
    return k;
}

// cwbvh_node_intersect (CommonData.cginc:641-707) restricted to this lane's 8/G child slots
// [sub*8/G, (sub+1)*8/G): the same operations per child as node_intersect, so the OR over the
// group is bit-identical to the full hitmask.
template <int G>
__device__ __forceinline__ uint32_t node_intersect_part(const uint4 n0, const uint4 n1, const uint4 n2,
                                                        const uint4 n3, const uint4 n4, const LaneRay& r,
                                                        uint32_t oct_inv4, float max_distance, uint32_t sub) {
    constexpr uint32_t NC = 8 / G;
    const uint32_t c0 = sub * NC;
    const bool h = c0 >= 4u;  // slots 4-7 live in the second word of each pair
    const uint32_t jb = c0 & 3u;
    const uint32_t w = n0.w;
    const float adjx = __uint_as_float((w & 0xffu) << 23) * r.ix;
    const float adjy = __uint_as_float(((w >> 8) & 0xffu) << 23) * r.iy;
    const float adjz = __uint_as_float(((w >> 16) & 0xffu) << 23) * r.iz;
    const float orgx = r.ix * (__uint_as_float(n0.x) - r.ox);
    const float orgy = r.iy * (__uint_as_float(n0.y) - r.oy);
    const float orgz = r.iz * (__uint_as_float(n0.z) - r.oz);
    const uint32_t meta4 = h ? n1.w : n1.z;
    const uint32_t is_inner4 = (meta4 & (meta4 << 1)) & 0x10101010u;
    const uint32_t inner_mask4 = (is_inner4 >> 1) - (is_inner4 >> 4);
    const uint32_t bit_index4 = (meta4 ^ (oct_inv4 & inner_mask4)) & 0x1f1f1f1fu;
    const uint32_t child_bits4 = (meta4 >> 5) & 0x07070707u;
    const uint32_t qlx = h ? n2.y : n2.x, qhx = h ? n2.w : n2.z;
    const uint32_t qly = h ? n3.y : n3.x, qhy = h ? n3.w : n3.z;
    const uint32_t qlz = h ? n4.y : n4.x, qhz = h ? n4.w : n4.z;
    const bool nx = r.dx < 0.0f, ny = r.dy < 0.0f, nz = r.dz < 0.0f;
    const uint32_t x_min = nx ? qhx : qlx, x_max = nx ? qlx : qhx;
    const uint32_t y_min = ny ? qhy : qly, y_max = ny ? qly : qhy;
    const uint32_t z_min = nz ? qhz : qlz, z_max = nz ? qlz : qhz;
    uint32_t hit_mask = 0;
#pragma unroll
    for (uint32_t k = 0; k < NC; k++) {
        const uint32_t sh = (jb + k) * 8u;
        const float tminx = fma_((float)((x_min >> sh) & 0xffu), adjx, orgx);
        const float tminy = fma_((float)((y_min >> sh) & 0xffu), adjy, orgy);
        const float tminz = fma_((float)((z_min >> sh) & 0xffu), adjz, orgz);
        const float tmaxx = fma_((float)((x_max >> sh) & 0xffu), adjx, orgx);
        const float tmaxy = fma_((float)((y_max >> sh) & 0xffu), adjy, orgy);
        const float tmaxz = fma_((float)((z_max >> sh) & 0xffu), adjz, orgz);
        const float tmin = fmaxf(fmaxf(tminx, tminy), fmaxf(tminz, 1e-8f));
        const float tmax = fminf(fminf(tmaxx, tmaxy), fminf(tmaxz, max_distance));
        const uint32_t bits = ((child_bits4 >> sh) & 0xffu) << ((bit_index4 >> sh) & 0xffu);
        hit_mask |= (tmin < tmax) ? bits : 0u;
    }
    return hit_mask;
}


// The drain loop for groups of G lanes; regroups into 2G-lane groups when the live rays fit and
// returns when every ray of the wave has finished. `finish(st)` writes a finished ray's records,
// `exhaust(st)` sees a ray that ends without a record (the Reps bound or a stack overflow: the
// reference writes nothing for it); both are called on the group's first lane only.
template <bool STATS, bool MATCHECK, int G, class Finish, class Exhaust>
__device__ void wide_phase(const TraceArgs& A, WideState& st, uint2 (*s_stack)[TT_BLOCK], uint2* __restrict__ spill,
                           uint32_t spill_stride, __amdgpu_buffer_rsrc_t nodes, __amdgpu_buffer_rsrc_t tris,
                           uint32_t lane, Counters C, Finish& finish, Exhaust& exhaust) {
    const uint32_t sub = lane & (G - 1);
    const uint32_t base = lane & ~(uint32_t)(G - 1);
    const uint32_t tid = st.scol, gtid = st.gcol;  // the stack the TT_PUSH / TT_POP macros address
    int32_t& stack_size = st.stack_size;
    while (true) {
        const uint64_t lead = __ballot(st.active && sub == 0u);
        const uint32_t n = (uint32_t)__popcll(lead);
        if (n == 0u) return;
        TT_DB(G == 2 ? 14 : G == 4 ? 15 : 16);
        if constexpr (G < 8) {
            if (n * (2 * G) <= TT_WAVE) {
                regroup<2 * G>(st, lead, lane);
                wide_phase<STATS, MATCHECK, 2 * G>(A, st, s_stack, spill, spill_stride, nodes, tris, lane, C, finish,
                                                   exhaust);
                return;
            }
        }
        // ------------------------------------------------------------- node phase
        if (st.active && st.tg.y == 0u) {
            if (st.Reps >= TT_MAX_REPS) {
                st.active = false;  // loop bound hit: the reference writes nothing
                if (STATS && sub == 0u) C.reps++;
                if (sub == 0u) exhaust(st);
            } else if (st.cg.y & 0xff000000u) {  // IntersectionKernels.compute:157-187
                const uint32_t cio = firstbithigh(st.cg.y);
                const uint32_t slot = (cio - 24u) ^ (st.oct & 0xffu);
                const uint32_t rel = __builtin_popcount(st.cg.y & ~(0xffffffffu << slot));
                const uint32_t child = st.cg.x + rel;
                st.cg.y &= ~(1u << cio);
                bool ok = true;
                if (st.cg.y & 0xff000000u) TT_PUSH(st.cg, ok);
                if (ok) {
                    TT_DB(G == 2 ? 20 : G == 4 ? 21 : 22);
                    TT_DL(23, sub == 0u);
                    const uint32_t no = node_offset(child);
                    const uint4 n0 = buffer_load16(nodes, no), n1 = buffer_load16(nodes, no + 16u),
                                n2 = buffer_load16(nodes, no + 32u), n3 = buffer_load16(nodes, no + 48u),
                                n4 = buffer_load16(nodes, no + 64u);
                    const uint32_t hitmask =
                        group_or<G>(node_intersect_part<G>(n0, n1, n2, n3, n4, st.ray, st.oct, st.best.t, sub));
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
                        exhaust(st);
                    }
                }
            } else {  // :188-191
                st.tg = st.cg;
                st.cg = make_uint2(0u, 0u);
            }
            if (st.active && st.tg.y != 0u && st.tlas_ss == -1) {  // :194-219 TLAS leaf -> BLAS
                const uint32_t mo = firstbithigh(st.tg.y);
                st.tg.y &= ~(1u << mo);
                const float4* mp = reinterpret_cast<const float4*>(A.leaf + (st.tg.x + mo));  // LeafMesh
                const float4 m0 = mp[0], m1 = mp[1], m2 = mp[2];
                const int4 mo4 = reinterpret_cast<const int4*>(mp)[3];
                st.mesh_id = reinterpret_cast<const int4*>(mp)[4].x;
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
                        exhaust(st);
                    }
                }
                st.tg.y = 0u;
            }
        }

        // --------------------------------------------------------- triangle phase
        // :220-226 visits the leaf's triangles highest bit first; lane `sub` takes the sub-th of them
        if (st.active && st.tg.y != 0u) {
            TT_DB(G == 2 ? 24 : G == 4 ? 25 : 26);
            TT_DL(27, sub == 0u);
            uint32_t m = st.tg.y;
#pragma unroll
            for (uint32_t k = 0; k + 1 < (uint32_t)G; k++)
                if (k < sub && m) m &= ~(1u << firstbithigh(m));
            const bool has = m != 0u;
            const int32_t tri_id = (int32_t)(st.tg.x + (has ? firstbithigh(m) : 0u));
            TriCand c{0.0f, 0.0f, 0.0f, false, false};
            if (has) c = triangle_candidate<MATCHECK>(tris, A.mat, A.bounce == 0, A.flags, tri_id, st.MatOffset, st.ray,
                                                     st.best.t);
            if (STATS) {  // replay the reference's sequential counting of t-test passes ("accepts")
                float run = st.best.t;
                uint32_t acc = 0;
                const uint32_t f = (c.cand ? 1u : 0u) | (c.accept ? 2u : 0u);
#pragma unroll
                for (uint32_t k = 0; k < (uint32_t)G; k++) {
                    const float tk = shfl_f(c.t, base + k);
                    const uint32_t fk = shfl_u(f, base + k);
                    if ((fk & 1u) && tk < run) {
                        acc++;
                        if (fk & 2u) run = tk;
                    }
                }
                if (sub == 0u) {
                    C.acc += acc;
                    C.tris += min((uint32_t)__builtin_popcount(st.tg.y), (uint32_t)G);
                }
            }
            // closest accepted candidate; equal t -> lowest sub = first in the reference's order
            const uint64_t key = group_min_u64<G>(c.accept ? (((uint64_t)__float_as_uint(c.t) << 32) | sub) : ~0ull);
            if (key != ~0ull) {
                const uint32_t src = base + ((uint32_t)key & (uint32_t)(G - 1));
                st.best.t = __uint_as_float((uint32_t)(key >> 32));
                st.best.u = shfl_f(c.u, src);
                st.best.v = shfl_f(c.v, src);
                st.best.tri_id = shfl_i(tri_id, src);
                st.best.mesh_id = st.mesh_id;
            }
#pragma unroll
            for (uint32_t k = 0; k < (uint32_t)G; k++)
                if (st.tg.y) st.tg.y &= ~(1u << firstbithigh(st.tg.y));
        }

        // ----------------------------------------- advance: pop / finish (:228-251)
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
                if (sub == 0u) finish(st);
                st.active = false;
            }
        }
    }
}

}  // namespace
#endif  // TT_WIDE_H
