// tt_solo.h — one ray per wave ("solo" mode) for the launch's longest rays.
//
// A launch cannot end before its longest ray, and the longest rays are serial chains: with the
// unjittered C2 camera the screen column whose direction.z is exactly -0.0 has NaN
// z slabs (inf * 0), so every box passes in z and each of its ~1,000 rays walks ~900 nodes and
// ~1,600 triangles; one of them exhausts Reps (tools/long_rays.py). In the narrow kernel such a
// ray advances one node or one triangle per wave iteration, behind 63 other lanes' VALU work; in
// the G-lane drain (tt_wide.h) one step still costs a dependent load plus the node test.
//
// Solo mode gives one ray a whole wave and keeps its state wave-uniform (SGPRs, scalar branches):
//  * node step: the 64 lanes form 8 groups of 8; group g holds node `pf_base + g` (lane k of a
//    group tests child slot k), so all eight children of the node just tested are tested at once
//    against the current best.t -- the one the reference visits next is read out with readlane;
//  * lookahead: right after a node test, group g loads node `first_child + g`, so the next
//    descent finds its node already in registers (a DFS pop back into a group whose siblings were
//    loaded hits the same set); only pops into older groups wait for a load, and they load all of
//    that group's siblings at once;
//  * a leaf group's (up to 24) triangles are tested in one pass, lane i = bit i, and the closest
//    accepted one with the earliest reference order (highest bit) wins -- exactly what the
//    sequential strict `t < best.t` loop keeps;
//  * the traversal stack lives in a VGPR across lanes (lane i = entry i), pushed / popped with
//    v_writelane / v_readlane.
// Visit order, culling distance, Reps and the stats counters are the reference's, so results are
// bit-identical to the narrow kernel (every GPU parity test ends its launches in this phase when a
// wave is left with one ray).
#ifndef TT_SOLO_H
#define TT_SOLO_H
// included by tt_wide.h after WideState, Counters and the DPP helpers, before wide_phase

#ifndef TT_SOLO
#define TT_SOLO 0  // 1: solo phase for a wave's last ray (off: its uniform state spills SGPRs and costs occupancy)
#endif

namespace {

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ int32_t rdli(int32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, (int)l); }
__device__ __forceinline__ float rdlf(float v, uint32_t l) { return __uint_as_float(rdl(__float_as_uint(v), l)); }
// v_writelane equivalent: lane `l` (uniform) takes `v`, the others keep `old`
__device__ __forceinline__ uint32_t wrl(uint32_t v, uint32_t l, uint32_t old) {
    return (__lane_id() == l) ? v : old;
}

// Minimum over lanes 0-31 of a float (DPP within each 16-lane row, then two readlanes).
template <int CTRL>
__device__ __forceinline__ float dpp_minf(float v) {
    const float o = __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp((int)0x7f800000, (int)__float_as_uint(v), CTRL,
                                                                         0xf, 0xf, false));
    return fminf(v, o);
}
__device__ __forceinline__ float min32_f(float v) {
    v = dpp_minf<0xB1>(v);
    v = dpp_minf<0x4E>(v);
    v = dpp_minf<0x141>(v);
    v = dpp_minf<0x140>(v);
    return fminf(rdlf(v, 0), rdlf(v, 16));
}

// Triangle bits of a node's leaf children (union over its 8 meta bytes: mask(1/3/7) << offset).
__device__ __forceinline__ uint32_t leaf_tri_bits(uint32_t meta_lo, uint32_t meta_hi) {
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t b = ((j < 4 ? meta_lo : meta_hi) >> ((j & 3) * 8)) & 0xffu;
        const bool inner = (b & 0x18u) == 0x18u;
        if (b != 0u && !inner) bits |= (b >> 5) << (b & 0x1fu);
    }
    return bits & 0x00ffffffu;
}

// Takes the state of the ray in lane `src` (wave-uniform afterwards).
__device__ __forceinline__ void solo_take(WideState& s, uint32_t src) {
    auto ray = [&](LaneRay& r) {
        r.ox = rdlf(r.ox, src); r.oy = rdlf(r.oy, src); r.oz = rdlf(r.oz, src);
        r.dx = rdlf(r.dx, src); r.dy = rdlf(r.dy, src); r.dz = rdlf(r.dz, src);
        r.ix = rdlf(r.ix, src); r.iy = rdlf(r.iy, src); r.iz = rdlf(r.iz, src);
    };
    ray(s.ray);
    ray(s.wray);
    s.best.t = rdlf(s.best.t, src);
    s.best.u = rdlf(s.best.u, src);
    s.best.v = rdlf(s.best.v, src);
    s.best.mesh_id = rdli(s.best.mesh_id, src);
    s.best.tri_id = rdli(s.best.tri_id, src);
    s.cg = make_uint2(rdl(s.cg.x, src), rdl(s.cg.y, src));
    s.tg = make_uint2(rdl(s.tg.x, src), rdl(s.tg.y, src));
    s.oct = rdl(s.oct, src);
    s.stack_size = rdli(s.stack_size, src);
    s.tlas_ss = rdli(s.tlas_ss, src);
    s.NodeOffset = rdli(s.NodeOffset, src);
    s.TriOffset = rdli(s.TriOffset, src);
    s.MatOffset = rdli(s.MatOffset, src);
    s.mesh_id = rdli(s.mesh_id, src);
    s.Reps = rdli(s.Reps, src);
    s.ray_index = rdl(s.ray_index, src);
    s.pix = rdl(s.pix, src);
    s.col_w = rdlf(s.col_w, src);
    s.scol = rdl(s.scol, src);
    s.gcol = rdl(s.gcol, src);
    s.active = true;
}

// Runs the wave-uniform ray `st` to completion. `stk`: lane i holds stack entry i. Must be called
// with every lane of the wave enabled. `finish(st)` runs on lane 0 when the reference would write.
template <bool STATS, bool MATCHECK, class Finish>
__device__ void solo_run(const TraceArgs& A, WideState st, uint2 stk, __amdgpu_buffer_rsrc_t nodes,
                         __amdgpu_buffer_rsrc_t tris, uint32_t lane, Counters C, Finish& finish) {
    const uint32_t grp = lane >> 3, k8 = lane & 7u;
    const bool lead = lane == 0u;
    uint32_t pf_base = 0xffffffffu;  // group g's registers hold node pf_base + g
    uint4 q0 = make_uint4(0u, 0u, 0u, 0u), q1 = q0, q2 = q0, q3 = q0, q4 = q0;
    auto load_group = [&](uint32_t base) {
        const uint32_t no = node_offset(base + grp);
        q0 = buffer_load16(nodes, no);
        q1 = buffer_load16(nodes, no + 16u);
        q2 = buffer_load16(nodes, no + 32u);
        q3 = buffer_load16(nodes, no + 48u);
        q4 = buffer_load16(nodes, no + 64u);
        pf_base = base;
    };
    TriData td{};         // lane i: triangle tg.x + i of the node tested this iteration (prefetched)
    bool write = false;
#ifdef TT_DIAG_SOLO  // cycles (s_memtime) per phase -> diag_times[0..2], iterations [3], node steps [4], tri passes [5], rays [6]
    uint64_t dg_node = 0, dg_tri = 0, dg_adv = 0, dg_it = 0, dg_ns = 0, dg_tp = 0, dg_nwait = 0, dg_twait = 0;
#define TT_SOLO_T() __builtin_amdgcn_s_memtime()
#else
#define TT_SOLO_T() 0ull
#endif
    while (true) {
        [[maybe_unused]] const uint64_t t0 = TT_SOLO_T();
        bool tri_pf = false;
        // ------------------------------------------------------------ node step (:155-219)
        if (st.tg.y == 0u) {
            if (st.Reps >= TT_MAX_REPS) {  // loop bound hit: the reference writes nothing
                if (STATS && lead) C.reps++;
                break;
            }
            if (st.cg.y & 0xff000000u) {
                const uint32_t cio = firstbithigh(st.cg.y);
                const uint32_t slot = (cio - 24u) ^ (st.oct & 0xffu);
                const uint32_t rel = __builtin_popcount(st.cg.y & ~(0xffffffffu << slot));
                const uint32_t base = st.cg.x;
                st.cg.y &= ~(1u << cio);
                if (st.cg.y & 0xff000000u) {
                    if (st.stack_size == TT_STACK_SIZE) {
                        if (lead) {
                            if (STATS) C.ovf++;
                            TT_REPORT_OVERFLOW(A);
                        }
                        break;
                    }
                    stk.x = wrl(st.cg.x, (uint32_t)st.stack_size, stk.x);
                    stk.y = wrl(st.cg.y, (uint32_t)st.stack_size, stk.y);
                    st.stack_size++;
                }
                if (pf_base != base) load_group(base);  // a pop into an older group: load its siblings
#ifdef TT_DIAG_SOLO
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                dg_nwait += TT_SOLO_T() - t0;
#endif
                const uint32_t src = rel * 8u;
                const uint32_t n0w = rdl(q0.w, src), n1x = rdl(q1.x, src), n1y = rdl(q1.y, src);
                if (st.tlas_ss != -1) {
                    // inside a BLAS: issue the loads of every leaf triangle of this node now, so they
                    // arrive while the node test runs (lane i = triangle bit i)
                    const uint32_t leaf = leaf_tri_bits(rdl(q1.z, src), rdl(q1.w, src));
                    if (lane < 24u && ((leaf >> lane) & 1u))
                        td = triangle_load<MATCHECK>(tris, (int32_t)(n1y + (uint32_t)st.TriOffset + lane));
                    tri_pf = true;
                }
                // every group tests its node; the reference visits group `rel`'s
                const uint32_t part = node_intersect_part<8>(q0, q1, q2, q3, q4, st.ray, st.oct, st.best.t, k8);
                const uint32_t hm = rdl(group_or<8>(part), src);
                st.cg = make_uint2(n1x + (uint32_t)st.NodeOffset, (hm & 0xff000000u) | (n0w >> 24));
                st.tg = make_uint2(n1y + (uint32_t)st.TriOffset, hm & 0x00ffffffu);
                st.Reps++;
                if (STATS && lead) C.nodes++;
                if (st.cg.y & 0xff000000u) load_group(st.cg.x);  // lookahead: this node's children
            } else {  // :188-191
                st.tg = st.cg;
                st.cg = make_uint2(0u, 0u);
            }
            if (st.tg.y != 0u && st.tlas_ss == -1) {  // :194-219 TLAS leaf -> BLAS
                const uint32_t mo = firstbithigh(st.tg.y);
                st.tg.y &= ~(1u << mo);
                const float4* mp = reinterpret_cast<const float4*>(A.leaf + (st.tg.x + mo));  // LeafMesh
                const float4 m0 = mp[0], m1 = mp[1], m2 = mp[2];
                const int4 mo4 = reinterpret_cast<const int4*>(mp)[3];
                st.mesh_id = reinterpret_cast<const int4*>(mp)[4].x;
                st.NodeOffset = mo4.y;
                st.TriOffset = mo4.x;
                const int32_t need = (st.tg.y != 0u ? 1 : 0) + ((st.cg.y & 0xff000000u) ? 1 : 0);
                if (st.stack_size + need > TT_STACK_SIZE) {
                    if (lead) {
                        if (STATS) C.ovf++;
                        TT_REPORT_OVERFLOW(A);
                    }
                    break;
                }
                if (st.tg.y != 0u) {
                    stk.x = wrl(st.tg.x, (uint32_t)st.stack_size, stk.x);
                    stk.y = wrl(st.tg.y, (uint32_t)st.stack_size, stk.y);
                    st.stack_size++;
                }
                if (st.cg.y & 0xff000000u) {
                    stk.x = wrl(st.cg.x, (uint32_t)st.stack_size, stk.x);
                    stk.y = wrl(st.cg.y, (uint32_t)st.stack_size, stk.y);
                    st.stack_size++;
                }
                st.tlas_ss = st.stack_size;
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
                st.tg.y = 0u;
                if (STATS && lead) C.blas++;
            }
        }

        [[maybe_unused]] const uint64_t t1 = TT_SOLO_T();
        [[maybe_unused]] const bool tri_now = st.tg.y != 0u;
        // ------------------------------------------- the leaf group's triangles (:220-226)
        if (st.tg.y != 0u) {
            const bool has = lane < 24u && ((st.tg.y >> lane) & 1u);
            const int32_t tri_id = (int32_t)(st.tg.x + lane);
            TriCand c{0.0f, 0.0f, 0.0f, false, false};
#ifdef TT_DIAG_SOLO
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            dg_twait += TT_SOLO_T() - t1;
#endif
            if (has && !tri_pf) td = triangle_load<MATCHECK>(tris, tri_id);
            if (has) c = triangle_test<MATCHECK>(td, A.mat, A.bounce == 0, A.flags, tri_id, st.MatOffset, st.ray, st.best.t);
            if (STATS) {  // the reference's sequential count of t-test passes, highest bit first
                const uint32_t f = (c.cand ? 1u : 0u) | (c.accept ? 2u : 0u);
                float run = st.best.t;
                uint32_t acc = 0;
                uint32_t m = st.tg.y;
                while (m) {
                    const uint32_t b = firstbithigh(m);
                    m &= ~(1u << b);
                    const float tb = rdlf(c.t, b);
                    const uint32_t fb = rdl(f, b);
                    if ((fb & 1u) && tb < run) {
                        acc++;
                        if (fb & 2u) run = tb;
                    }
                }
                if (lead) {
                    C.acc += acc;
                    C.tris += (uint32_t)__builtin_popcount(st.tg.y);
                }
            }
            // closest accepted (accepted t are finite and > 0); equal t -> the highest bit, the one
            // the reference visits first
            const float tmin = min32_f(c.accept ? c.t : __builtin_inff());
            if (tmin != __builtin_inff()) {
                const uint64_t at = __ballot(c.accept && c.t == tmin);
                const uint32_t src = 63u - (uint32_t)__builtin_clzll(at);
                st.best.t = tmin;
                st.best.u = rdlf(c.u, src);
                st.best.v = rdlf(c.v, src);
                st.best.tri_id = (int32_t)(st.tg.x + src);
                st.best.mesh_id = st.mesh_id;
            }
            st.tg.y = 0u;
        }

        [[maybe_unused]] const uint64_t t2 = TT_SOLO_T();
        // ------------------------------------------------ advance: pop / finish (:228-251)
        if ((st.cg.y & 0xff000000u) == 0u) {
            if (st.stack_size != 0) {
                if (st.stack_size == st.tlas_ss) {
                    st.NodeOffset = 0;
                    st.TriOffset = 0;
                    st.tlas_ss = -1;
                    st.ray = st.wray;
                    st.oct = octant_inv4(st.ray);
                }
                st.stack_size--;
                st.cg = make_uint2(rdl(stk.x, (uint32_t)st.stack_size), rdl(stk.y, (uint32_t)st.stack_size));
            } else {
                write = true;
                break;
            }
        }
#ifdef TT_DIAG_SOLO
        const uint64_t t3 = TT_SOLO_T();
        dg_node += t1 - t0;
        dg_tri += t2 - t1;
        dg_adv += t3 - t2;
        dg_it++;
        dg_ns = (uint64_t)st.Reps;
        dg_tp += tri_now ? 1u : 0u;
#endif
    }
#ifdef TT_DIAG_SOLO
    if (lead && A.diag_times) {
        atomicAdd(A.diag_times + 0, (unsigned long long)dg_node);
        atomicAdd(A.diag_times + 1, (unsigned long long)dg_tri);
        atomicAdd(A.diag_times + 2, (unsigned long long)dg_adv);
        atomicAdd(A.diag_times + 3, (unsigned long long)dg_it);
        atomicAdd(A.diag_times + 4, (unsigned long long)dg_ns);
        atomicAdd(A.diag_times + 5, (unsigned long long)dg_tp);
        atomicAdd(A.diag_times + 6, 1ull);
        atomicAdd(A.diag_times + 7, (unsigned long long)dg_nwait);
        atomicAdd(A.diag_times + 8, (unsigned long long)dg_twait);
    }
#endif
    if (write && lead) finish(st);
}

}  // namespace
#endif  // TT_SOLO_H
