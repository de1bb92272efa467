// tt_trace.hip — gfx950 closest-hit CWBVH8 traversal (replaces kernel_trace,
// TrueTrace/Resources/MainCompute/IntersectionKernels.compute:60-260).
//
// Design (MI355X-first, not a translation of the HLSL dispatch):
//  * persistent waves: grid = CUs x resident blocks; rays are dequeued per wave from per-XCD
//    segment counters, TT_CHUNK_BIG at a time with ONE atomic (the reference pops one ray per
//    thread from a single globally-coherent counter, IntersectionKernels.compute:79-81);
//  * lanes that finish are refilled in place (ballot + mbcnt prefix over idle lanes) so the
//    64-wide wave keeps working instead of idling behind its slowest ray;
//  * the 16-entry uint2 traversal stack lives in LDS, [entry][thread] so a wave's 64 stack
//    accesses hit 64 distinct banks (ds_read_b64/ds_write_b64, conflict-free);
//  * 80-B nodes are five 16-B loads; triangles use a 48-B traversal layout (three 16-B loads)
//    derived from AggTris at upload;
//  * the per-ray visit order, the culling distance and the strict t < best.t acceptance are
//    exactly the reference's, so t / primID / instID are bit-identical to the oracle.
// Numerics follow include/truetrace_hip.h (compiled with -ffp-contract=off).
#include "tt_wide.h"

namespace {
// :229-241 + set() CommonData.cginc:430-434: the hit record and _PrimaryTriangleInfo of a finished
// ray (wr = the world-space ray, ray2). Returns whether the ray hit something.
template <int INFO>
__device__ __forceinline__ bool write_record(const TraceArgs& A, uint32_t ray_index, uint32_t pix, float col_w,
                                             const Best& best, const LaneRay& wr) {
    tt_ray_data* R = A.rays + ray_index;
    if (INFO != 0) {
        // (pix % W, pix / W) with pix / W < H is the texel at index pix: no division needed
        if (pix < A.n_pixels) {
            uint4 o;
            bool write = false;
            if (INFO == 1) {
                const int32_t to = A.mesh[best.mesh_id].TriOffset;
                o = make_uint4((uint32_t)best.mesh_id, (uint32_t)(best.tri_id - to),
                               __float_as_uint(best.u), __float_as_uint(best.v));
                write = true;
            } else {
                const float w = col_w;
                if (w == -1.0f || (float)A.bounce == w) {
                    write = true;
                    const bool miss = best.t == A.far_plane;
                    if ((A.flags & TT_TRACE_USE_RESTIRGI) && !miss) {
                        const int32_t to = A.mesh[best.mesh_id].TriOffset;
                        o.x = (uint32_t)best.mesh_id;
                        o.y = (uint32_t)(best.tri_id - to);
                        o.z = (uint32_t)(best.u * 65535.0f) | ((uint32_t)(best.v * 65535.0f) << 16);
                    } else if ((A.flags & TT_TRACE_USE_ASVGF) || !miss) {
                        o.x = __float_as_uint(wr.dx);
                        o.y = __float_as_uint(wr.dy);
                        o.z = __float_as_uint(wr.dz);
                    } else {
                        o.x = __float_as_uint(wr.dx * best.t + wr.ox);
                        o.y = __float_as_uint(wr.dy * best.t + wr.oy);
                        o.z = __float_as_uint(wr.dz * best.t + wr.oz);
                    }
                    o.w = miss ? 1u : 0u;
                }
            }
            if (write) reinterpret_cast<uint4*>(A.info)[pix] = o;
        }
    }
    const uint32_t uv = (uint32_t)(best.u * 65535.0f) | ((uint32_t)(best.v * 65535.0f) << 16);
    const uint4 hit = make_uint4((uint32_t)best.mesh_id, (uint32_t)best.tri_id, __float_as_uint(best.t), uv);
    reinterpret_cast<uint4*>(R)[2] = hit;
    if (A.hits_out) {  // the compact record stream (multi-GPU gather): a raw buffer store, 32-bit offset
        const u32x4 v = {hit.x, hit.y, hit.z, hit.w};
        __builtin_amdgcn_raw_buffer_store_b128(v, buffer_rsrc(A.hits_out, 0x7fffffff), (ray_index - A.ray_offset) << 4,
                                               0, 0);
    }
    return best.t != A.far_plane;
}

// A ray that ends without a record (the Reps bound, IntersectionKernels.compute:155, or a stack
// overflow) leaves RayData.hits as it was; the compact stream (tt_trace_closest_hits) promises the
// same bytes as RayData.hits, so it gets the unchanged word (a rare path: one 16-B load).
__device__ __forceinline__ void keep_record(const TraceArgs& A, uint32_t ray_index) {
    if (A.hits_out) {
        const uint4 h = reinterpret_cast<const uint4*>(A.rays + ray_index)[2];
        const u32x4 v = {h.x, h.y, h.z, h.w};
        __builtin_amdgcn_raw_buffer_store_b128(v, buffer_rsrc(A.hits_out, 0x7fffffff), (ray_index - A.ray_offset) << 4,
                                               0, 0);
    }
}

// TT_TRACE_ADAPTIVE_ORDER: a finished (or Reps-exhausted) ray's cost -- its Reps count -- into its
// ray chunk's entry of the launch's cost map (no-return atomic max; tt_order.hip sorts the next
// launch's chunks by it). The ray chunk is the 8x8 pixel tile in the full-frame swizzle, else
// (ray index - offset) / 64. Rays below TT_ORDER_MIN_REPS skip the atomic: chunks whose rays are all
// cheap keep cost 0 and their natural order, and a launch issues few atomics.
static_assert(TT_CHUNK_BIG == 64, "the adaptive order maps one dequeue (TT_CHUNK_BIG rays) to one 64-ray chunk");
#ifndef TT_ORDER_MIN_REPS
#define TT_ORDER_MIN_REPS 32
#endif
__device__ __forceinline__ void record_chunk_cost(const TraceArgs& A, bool swizzle, uint32_t ray_index, int32_t reps) {
    if (reps < TT_ORDER_MIN_REPS) return;
    const uint32_t local = ray_index - A.ray_offset;
    uint32_t c = local >> 6;
    if (swizzle) {
        const uint32_t py = fastdiv(local, A.div_width), px = local - py * A.width;
        c = (py >> 3) * (A.width >> 3) + (px >> 3);
    }
    atomicMax(A.chunk_cost + c, (uint32_t)reps);
}
}  // namespace


// TT_ROOT_LEAF (TraceArgs::root, tt_device.h): the root of a one-leaf TLAS is stepped when a ray starts
// and the TLAS leaf -> BLAS switch follows before the loop's node step, so the ray's first node step in
// the loop is already its BLAS root (one loop iteration less per ray).
namespace {
// node_intersect (tt_traverse.h) for the root's one child: the same operations in the same order
__device__ __forceinline__ bool root_leaf_hit(const RootLeaf& R, const LaneRay& r, float max_distance) {
    const float adjx = __uint_as_float(rl_byte(R.e, 0) << 23) * r.ix;
    const float adjy = __uint_as_float(rl_byte(R.e, 1) << 23) * r.iy;
    const float adjz = __uint_as_float(rl_byte(R.e, 2) << 23) * r.iz;
    const float orgx = r.ix * (R.px - r.ox);
    const float orgy = r.iy * (R.py - r.oy);
    const float orgz = r.iz * (R.pz - r.oz);
    const bool nx = r.dx < 0.0f, ny = r.dy < 0.0f, nz = r.dz < 0.0f;
    const uint32_t x_min = rl_byte(nx ? R.qhi : R.qlo, 0), x_max = rl_byte(nx ? R.qlo : R.qhi, 0);
    const uint32_t y_min = rl_byte(ny ? R.qhi : R.qlo, 1), y_max = rl_byte(ny ? R.qlo : R.qhi, 1);
    const uint32_t z_min = rl_byte(nz ? R.qhi : R.qlo, 2), z_max = rl_byte(nz ? R.qlo : R.qhi, 2);
    const float tminx = fma_((float)x_min, adjx, orgx);
    const float tminy = fma_((float)y_min, adjy, orgy);
    const float tminz = fma_((float)z_min, adjz, orgz);
    const float tmaxx = fma_((float)x_max, adjx, orgx);
    const float tmaxy = fma_((float)y_max, adjy, orgy);
    const float tmaxz = fma_((float)z_max, adjz, orgz);
    const float tmin = fmaxf(fmaxf(tminx, tminy), fmaxf(tminz, 1e-8f));
    float tmaxz_c;
    asm("v_min_f32 %0, %1, %2" : "=v"(tmaxz_c) : "v"(tmaxz), "v"(max_distance));
    const float tmax = fminf(fminf(tmaxx, tmaxy), tmaxz_c);
    return tmin < tmax;
}
}  // namespace


// INFO: 0 = no _PrimaryTriangleInfo, 1 = bounce 0 form, 2 = bounce > 0 form (GlobalColors).
// IND: the ray count is device-resident (tt_trace_closest_indirect): instantiated as its own kernel
// (tt_trace_kernel_indirect), so the direct launches keep exactly their code and kernel names.
// ORD: TT_TRACE_ADAPTIVE_ORDER (tt_trace_kernel_ord): chunks are dequeued in A.order (when set) and
// every ray's Reps count goes into the tile cost map.
template <bool STATS, bool MATCHECK, int INFO, bool IND, bool ORD>
__device__ __forceinline__ void trace_body(const TraceArgs& A) {
    __shared__ uint2 s_stack[TT_LDS_STACK][TT_BLOCK];
    const uint32_t tid = threadIdx.x;
    zero_next_control(A.ctl_next, tid);
    const uint32_t gtid = blockIdx.x * TT_BLOCK + tid;
    const uint32_t spill_stride = gridDim.x * TT_BLOCK;
    uint2* __restrict__ spill = A.spill;
    (void)gtid;
    (void)spill_stride;
    (void)spill;
    const uint32_t lane = tid & (TT_WAVE - 1);
#ifdef TT_DIAG_BLOCKS
    if (tid < TT_DB_N) tt_db[tid] = 0ull;
    __syncthreads();
#endif

    // wave-uniform scheduler state: a private pool [pool_next, pool_end) of work indices, refilled
    // from segment `seg` (segments = contiguous 1/TT_SEGS slices of the work range, dealt to XCD
    // groups by blockIdx % TT_SEGS for L2 locality; exhausted segments are stolen from in turn)
    uint32_t pool_next = 0, pool_end = 0, more = 1;
    const uint32_t wave_id = blockIdx.x * (TT_BLOCK / TT_WAVE) + (tid >> 6);
    SegState S{blockIdx.x % TT_SEGS, 0u, 0u};
    const uint32_t n_rays = IND ? launch_ray_count(A) : A.n_rays;
    const uint32_t n_tiles = (n_rays + 63u) >> 6;
    // work index -> ray index in 8x8 screen tiles: full-frame primary batches only (a device count
    // decides at run time)
    const bool swizzle = IND ? (A.tile_swizzle && n_rays == A.n_pixels) : (A.tile_swizzle != 0u);
    const __amdgpu_buffer_rsrc_t nodes = buffer_rsrc(A.nodes, A.n_nodes * (uint32_t)TT_NODE_STRIDE);
    const __amdgpu_buffer_rsrc_t tris = buffer_rsrc(A.tris, A.n_tris * (uint32_t)sizeof(TriPos));

    // lane traversal state (IntersectionKernels.compute:62-77). A lane without a ray (idle, finished or
    // ended) holds tg.y == TT_IDLE: the pending-leaf word of a live ray never has bit 31 set (hit bits
    // 0-23 only), so "active" needs no register of its own and every phase test of the loop is one
    // compare of tg.y: at the loop top (tg.y == 0), leaf triangles pending ((int)tg.y > 0), idle (< 0).
    constexpr uint32_t TT_IDLE = 0x80000000u;
    uint32_t ray_index = 0;
    uint32_t pix = 0;    // RayData.PixelIndex, kept from the ray load
    float col_w = 0.0f;  // GlobalColors[pix].Data.w (INFO == 2), loaded when the ray starts
    bool pending = false;  // finished, record not yet written (TT_DEFER_FINISH)
    LaneRay ray{}, wray{};
    Best best{};
    uint2 cg = make_uint2(0u, 0u), tg = make_uint2(0u, TT_IDLE);
    uint32_t oct = 0;
    int32_t stack_size = 0, tlas_ss = -1;
    int32_t NodeOffset = 0, TriOffset = 0, MatOffset = 0, mesh_id = -1, Reps = 0;
    uint32_t c_nodes = 0, c_tris = 0, c_blas = 0, c_acc = 0, c_rays = 0, c_hits = 0, c_reps = 0, c_ovf = 0;
    uint32_t d_iter = 0, d_node_lanes = 0, d_node_iters = 0, d_tri_lanes = 0, d_tri_iters = 0, d_active_lanes = 0;
    uint32_t d_lead_same = 0, d_uniform = 0;  // node-step uniformity (lanes sharing the first lane's node)
    // the world-space ray (ray2, IntersectionKernels.compute:151), kept in registers
    auto world_ray = [&]() -> LaneRay { return wray; };

#if TT_ROOT_LEAF
    const bool rl_ok = A.root.ok != 0u;  // a kernel argument: wave-uniform
#endif
    // :194-219 TLAS leaf -> BLAS (the lane is at TLAS level with pending leaf bits in tg)
    auto enter_blas = [&]() {
            TT_DB(8);
            const uint32_t mo = firstbithigh(tg.y);
            tg.y &= ~(1u << mo);
            const float4* mp = reinterpret_cast<const float4*>(A.leaf + (tg.x + mo));  // LeafMesh
            const float4 m0 = mp[0], m1 = mp[1], m2 = mp[2];
            const int4 mo4 = reinterpret_cast<const int4*>(mp)[3];
            const int4 mo5 = reinterpret_cast<const int4*>(mp)[4];
            mesh_id = mo5.x;
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
                keep_record(A, ray_index);
            }
    };
    // :229-241: the finished ray's hit record and _PrimaryTriangleInfo
    auto finish_ray = [&]() {
        const bool hit = write_record<INFO>(A, ray_index, pix, col_w, best, world_ray());
        if (STATS) c_hits += hit ? 1u : 0u;
        (void)hit;
        if (ORD) record_chunk_cost(A, swizzle, ray_index, Reps);
    };
    while (true) {
        TT_DB(0);
        // ---------------------------------------------------------------- refill
        const uint64_t idle = __ballot((int32_t)tg.y < 0);
        // (two 32-bit counts: written as __popcll, the compiler keeps the count 64-bit and tests it with two
        // VALU v_cmp_*_u64 per iteration)
        const uint32_t n_idle = (uint32_t)__builtin_popcount((uint32_t)idle) + (uint32_t)__builtin_popcount((uint32_t)(idle >> 32));
        const bool pool_dry = !more && pool_next >= pool_end;
#if TT_DRAIN_PRIO
        // a draining wave issues ahead of the waves of launches still in their bulk (other parts / frames)
        if (pool_dry) __builtin_amdgcn_s_setprio(TT_DRAIN_PRIO);
#endif
        // the queue is dry and the live rays fit in 2-lane groups: cooperative drain (tt_wide.h)
        const bool to_wide = TT_WIDE && pool_dry && n_idle < TT_WAVE && TT_WAVE - n_idle <= TT_WIDE_ENTER;
        // finished rays write their records in batches, right before their lanes are refilled
        if ((n_idle == TT_WAVE && pool_dry) || (n_idle >= TT_REFILL_MIN && !pool_dry) || to_wide) {
            if (pending) {
                TT_DB(1);
                finish_ray();
                pending = false;
            }
        }
        if (n_idle == TT_WAVE && pool_dry) break;
#if TT_WIDE
        if (to_wide) {
            TT_DB(13);
            WideState st{ray, world_ray(), best, cg, tg, oct, stack_size, tlas_ss, NodeOffset, TriOffset, MatOffset,
                         mesh_id, Reps, ray_index, pix, col_w, tid, gtid, (int32_t)tg.y >= 0};
            regroup<2>(st, __ballot((int32_t)tg.y >= 0), lane);
            auto finish_wide = [&](const WideState& w) {
                const bool hit = write_record<INFO>(A, w.ray_index, w.pix, w.col_w, w.best, w.wray);
                if (STATS) c_hits += hit ? 1u : 0u;
                if (ORD) record_chunk_cost(A, swizzle, w.ray_index, w.Reps);
            };
            auto exhaust_wide = [&](const WideState& w) {
                keep_record(A, w.ray_index);
                if (ORD) record_chunk_cost(A, swizzle, w.ray_index, w.Reps);
            };
            wide_phase<STATS, MATCHECK, 2>(A, st, s_stack, spill, spill_stride, nodes, tris, lane,
                                           Counters{c_nodes, c_tris, c_blas, c_acc, c_hits, c_reps, c_ovf},
                                           finish_wide, exhaust_wide);
            break;
        }
#endif
        if (n_idle >= TT_REFILL_MIN && !pool_dry) {
            TT_DB(2);
#if TT_LONG_PRIO
            // a wave carrying a long ray (>= TT_LONG_PRIO node steps so far) issues ahead of the others until
            // its next refill without one: the long ray's dependent chain, not the wave's share of issue,
            // is what sets a small launch's length (the degenerate-direction rays)
            if (__ballot((int32_t)tg.y >= 0 && Reps >= TT_LONG_PRIO) != 0ull) __builtin_amdgcn_s_setprio(TT_LONG_PRIO_LEVEL);
            else __builtin_amdgcn_s_setprio(0);
#endif
            // wave-uniform: take from the wave's pool first, then one dequeue for the rest
            const uint32_t avail = pool_end - pool_next;
            uint32_t new_base = 0, new_count = 0;
            if (avail < n_idle && more) {
                new_count = sched_reserve(A.ctl, n_rays, n_tiles, lane, n_idle - avail, wave_id, S, new_base);
                more = new_count > 0 ? 1u : 0u;
                // a reservation is one whole 64-ray work chunk (TT_CHUNK_BIG, chunk-aligned segments): the
                // adaptive order maps it to the ray chunk it dequeues (one wave-uniform load)
                if (ORD && A.order && new_count > 0)
                    new_base = (__builtin_amdgcn_readfirstlane(A.order[new_base >> 6]) << 6) | (new_base & 63u);
            }
            const uint32_t take_old = min(avail, n_idle);
            const uint32_t take_new = min(n_idle - take_old, new_count);
            const uint32_t rank = lane_prefix(idle);
            uint32_t widx = 0xffffffffu;
            if (rank < take_old) widx = pool_next + rank;
            else if (rank - take_old < take_new) widx = new_base + (rank - take_old);
            if (new_count > 0) {  // the old pool was fully consumed (avail < n_idle)
                pool_next = new_base + take_new;
                pool_end = new_base + new_count;
            } else {
                pool_next += take_old;
            }
#if TT_UNIFORM_POOL  // keep the wave-uniform scheduler state in SGPRs (the loop head's tests become SALU)
            pool_next = __builtin_amdgcn_readfirstlane(pool_next);
            pool_end = __builtin_amdgcn_readfirstlane(pool_end);
            more = __builtin_amdgcn_readfirstlane(more);
#endif
            if ((int32_t)tg.y < 0 && widx != 0xffffffffu) {
                TT_DB(4);
                TT_DL(19, true);
                // work index -> ray index (8x8 screen tiles for full-frame primary batches)
                uint32_t local = widx;
                if (swizzle) {
                    const uint32_t tw = A.width >> 3;
                    const uint32_t t = widx >> 6, l = widx & 63u;
                    const uint32_t ty = fastdiv(t, A.div_tiles), tx = t - ty * tw;
                    local = (ty * 8u + (l >> 3)) * A.width + tx * 8u + (l & 7u);
                }
                ray_index = A.ray_offset + local;
                const uint4* rp = reinterpret_cast<const uint4*>(A.rays + ray_index);
                const uint4 r0 = rp[0], r1 = rp[1];
                pix = r0.w;
                if (INFO == 2) col_w = (pix < A.n_pixels) ? A.colors[pix].Data[3] : 0.0f;
                ray.ox = __uint_as_float(r0.x);
                ray.oy = __uint_as_float(r0.y);
                ray.oz = __uint_as_float(r0.z);
                ray.dx = __uint_as_float(r1.x);
                ray.dy = __uint_as_float(r1.y);
                ray.dz = __uint_as_float(r1.z);
                ray.ix = rcp_rn(ray.dx);
                ray.iy = rcp_rn(ray.dy);
                ray.iz = rcp_rn(ray.dz);
                wray = ray;
                oct = octant_inv4(ray);
                best.t = A.far_plane;
                best.u = 0.0f;
                best.v = 0.0f;
                best.mesh_id = 0;
                best.tri_id = -1;
                cg = make_uint2(A.tlas_base, 0x80000000u);  // the TLAS root: node 0 of the context's TLAS
                tg = make_uint2(0u, 0u);
                stack_size = 0;
                tlas_ss = -1;
                NodeOffset = (int32_t)A.tlas_base;  // TLAS level (0, or a frame-slot TLAS's region)
                TriOffset = 0;
                MatOffset = 0;
                mesh_id = -1;
                Reps = 0;
                if (STATS) c_rays++;
#if TT_ROOT_LEAF
                if (rl_ok) {  // the root's node step, then the TLAS leaf -> BLAS switch
                    const RootLeaf& RL = A.root;
                    const bool hit = root_leaf_hit(RL, ray, best.t);
                    cg = make_uint2(RL.base_child, 0u);  // (hitmask & 0xff000000) | imask: both 0
                    tg = make_uint2(RL.base_tri, hit ? RL.bits : 0u);
                    Reps = 1;
                    if (STATS) c_nodes++;
                    // a ray that hits the root's leaf switches to its BLAS before this iteration's node step
                    // (here, with the started lanes only: a TLAS-level lane has no pending leaf bits at the
                    // loop top otherwise, so no per-iteration test is needed)
                    if (hit) enter_blas();
                }
#endif
            }
        }

        // ------------------------------------------------------------- node phase
        if (STATS) {  // SIMD-efficiency diagnostics (wave-uniform; lane 0 accumulates)
            const uint64_t nm = __ballot(tg.y == 0u && Reps < TT_MAX_REPS && (cg.y & 0xff000000u));
            const uint64_t am = __ballot((int32_t)tg.y >= 0);  // outside the lane-0 branch: a ballot there sees lane 0 only
            if (lane == 0) {
                d_iter++;
                d_node_lanes += (uint32_t)__popcll(nm);
                d_node_iters += nm ? 1u : 0u;
                d_active_lanes += (uint32_t)__popcll(am);
            }
        }
        // A lane is at the top of the reference's loop exactly when no leaf triangles are pending.
        if (tg.y == 0u) {
            TT_DB(5);
            if (Reps >= TT_MAX_REPS) {
                tg.y = TT_IDLE;  // loop bound hit: the reference writes nothing
                if (STATS) c_reps++;
                keep_record(A, ray_index);
                if (ORD) record_chunk_cost(A, swizzle, ray_index, Reps);
            } else if (cg.y & 0xff000000u) {  // IntersectionKernels.compute:157-187
                const uint32_t cio = firstbithigh(cg.y);
                const uint32_t slot = (cio - 24u) ^ (oct & 0xffu);
                const uint32_t rel = __builtin_popcount(cg.y & ~(0xffffffffu << slot));
                const uint32_t child = cg.x + rel;
                cg.y &= ~(1u << cio);
                bool ok = true;
                if (cg.y & 0xff000000u) {
                    TT_DB(7);
                    TT_PUSH(cg, ok);
                }
                if (ok) {
                    TT_DB(6);
                    TT_DL(17, true);
                    if (STATS) {  // how many node-phase lanes visit the same node as the first one
                        const uint32_t lead = __builtin_amdgcn_readfirstlane(child);
                        const uint64_t same = __ballot(child == lead), all = __ballot(true);
                        d_lead_same += child == lead ? 1u : 0u;
                        d_uniform += (same == all && lane == (uint32_t)__builtin_ctzll(all)) ? 1u : 0u;
                    }
                    const uint32_t no = node_offset(child);
                    const uint4 n0 = buffer_load16<TT_NODE_CPOL>(nodes, no), n1 = buffer_load16<TT_NODE_CPOL>(nodes, no + 16u),
                                n2 = buffer_load16<TT_NODE_CPOL>(nodes, no + 32u),
                                n3 = buffer_load16<TT_NODE_CPOL>(nodes, no + 48u),
                                n4 = buffer_load16<TT_NODE_CPOL>(nodes, no + 64u);
                    const uint32_t hitmask = node_intersect(n0, n1, n2, n3, n4, ray, oct, best.t);
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
                    keep_record(A, ray_index);
                }
            } else {  // :188-191
                tg = cg;
                cg = make_uint2(0u, 0u);
            }
            if ((int32_t)tg.y > 0 && tlas_ss == -1) enter_blas();  // :194-219 TLAS leaf -> BLAS
        }

        if (STATS) {
            const uint64_t tm = __ballot((int32_t)tg.y > 0);
            if (lane == 0) {
                d_tri_lanes += (uint32_t)__popcll(tm);
                d_tri_iters += tm ? 1u : 0u;
            }
        }
        // --------------------------------------------------------- triangle phase
        if ((int32_t)tg.y > 0) {  // :220-226, highest bit first, one triangle per pass
            TT_DB(9);
            TT_DL(18, true);
            const uint32_t ti = firstbithigh(tg.y);
            tg.y &= ~(1u << ti);
            const bool acc = intersect_triangle<MATCHECK>(tris, A.mat, A.bounce == 0, A.flags, (int32_t)(tg.x + ti),
                                                          mesh_id, MatOffset, ray, best);
            if (STATS) {
                c_tris++;
                c_acc += acc ? 1u : 0u;
            }
        }

        // ----------------------------------------- advance: pop / finish (:228-251)
        // One place for every lane whose group is used up, whether it came from a node step or
        // from its last triangle this pass (equivalent order: the reference pops right after).
        if (tg.y == 0u && (cg.y & 0xff000000u) == 0u) {
            TT_DB(10);
            if (stack_size != 0) {
                TT_DB(11);
                if (stack_size == tlas_ss) {
                    TT_DB(12);
                    NodeOffset = (int32_t)A.tlas_base;
                    TriOffset = 0;
                    tlas_ss = -1;
                    ray = world_ray();
                    oct = octant_inv4(ray);
                }
                TT_POP(cg);
            } else {
                pending = true;  // written at the next refill (or when the wave drains)
                tg.y = TT_IDLE;
            }
        }
    }

#ifdef TT_DIAG_BLOCKS
    __syncthreads();
    if (tid < TT_DB_N && A.diag_times && tt_db[tid]) atomicAdd(A.diag_times + tid, tt_db[tid]);
#endif
    if (STATS) {
        const uint32_t v[8] = {wave_sum(c_rays), wave_sum(c_nodes), wave_sum(c_tris), wave_sum(c_blas),
                               wave_sum(c_hits), wave_sum(c_reps), wave_sum(c_ovf), wave_sum(c_acc)};
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (v[k]) atomicAdd(&A.ctl->stats[k], (unsigned long long)v[k]);
            const uint32_t d[6] = {d_iter, d_node_iters, d_node_lanes, d_tri_iters, d_tri_lanes, d_active_lanes};
#pragma unroll
            for (int k = 0; k < 6; k++) atomicAdd(&A.ctl->diag[k], (unsigned long long)d[k]);
        }
        const uint32_t ls = wave_sum(d_lead_same), un = wave_sum(d_uniform);
        if (lane == 0) {
            atomicAdd(&A.ctl->diag[6], (unsigned long long)ls);
            atomicAdd(&A.ctl->diag[7], (unsigned long long)un);
        }
    }
}

template <bool STATS, bool MATCHECK, int INFO>
__global__ TT_BOUNDS void tt_trace_kernel(TraceArgs A) {
    trace_body<STATS, MATCHECK, INFO, false, false>(A);
}
template <bool MATCHECK, int INFO>
__global__ TT_BOUNDS void tt_trace_kernel_indirect(TraceArgs A) {
    trace_body<false, MATCHECK, INFO, true, false>(A);
}
// (held at 5 waves per SIMD like the direct kernels: the cost record would otherwise cost INFO = 2 a
// wave; the material-check forms keep the default bounds, which do not spill VGPRs)
template <int INFO>
__global__ __launch_bounds__(TT_BLOCK) __attribute__((amdgpu_waves_per_eu(5))) void tt_trace_kernel_ord(TraceArgs A) {
    trace_body<false, false, INFO, false, true>(A);
}
template <int INFO>
__global__ TT_BOUNDS void tt_trace_kernel_ord_mat(TraceArgs A) {
    trace_body<false, true, INFO, false, true>(A);
}

// ------------------------------------------------------------------ launchers
template <bool S, bool M, int I>
static hipError_t launch_one(const TraceArgs& a, uint32_t grid, hipStream_t st) {
    if constexpr (!S) {
        if (a.n_rays_dev) {  // stats launches never take a device count (tt_api.hip refuses them)
            hipLaunchKernelGGL((tt_trace_kernel_indirect<M, I>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
            return hipGetLastError();
        }
        if (a.chunk_cost) {  // TT_TRACE_ADAPTIVE_ORDER (never with stats or a device count)
            if (M) hipLaunchKernelGGL((tt_trace_kernel_ord_mat<I>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
            else hipLaunchKernelGGL((tt_trace_kernel_ord<I>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((tt_trace_kernel<S, M, I>), dim3(grid), dim3(TT_BLOCK), 0, st, a);
    return hipGetLastError();
}

template <bool S, bool M>
static hipError_t launch_info(const TraceArgs& a, int info, uint32_t grid, hipStream_t st) {
    if (info == 0) return launch_one<S, M, 0>(a, grid, st);
    if (info == 1) return launch_one<S, M, 1>(a, grid, st);
    return launch_one<S, M, 2>(a, grid, st);
}

hipError_t tt_launch_trace(const TraceArgs& a, bool stats, bool matcheck, int info, uint32_t grid,
                           hipStream_t st) {
    if (stats) return matcheck ? launch_info<true, true>(a, info, grid, st) : launch_info<true, false>(a, info, grid, st);
    return matcheck ? launch_info<false, true>(a, info, grid, st) : launch_info<false, false>(a, info, grid, st);
}

// Occupancy (resident blocks per CU) of every instantiation: they differ in registers, so each
// launch sizes its persistent grid from its own entry.
template <bool S, bool M, int I>
static int occ_one() {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tt_trace_kernel<S, M, I>, TT_BLOCK, 0) != hipSuccess) b = 1;
    return b;
}
template <bool M, int I>
static int occ_ord() {
    int b = 0;
    const hipError_t e = M ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tt_trace_kernel_ord_mat<I>, TT_BLOCK, 0)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tt_trace_kernel_ord<I>, TT_BLOCK, 0);
    return e == hipSuccess ? b : 1;
}
// index = stats*6 + matcheck*3 + info; 12 + matcheck*3 + info: the adaptive-order kernels
hipError_t tt_trace_occupancy_table(int* out18) {
    int* out12 = out18;
    out12[0] = occ_one<false, false, 0>();
    out12[1] = occ_one<false, false, 1>();
    out12[2] = occ_one<false, false, 2>();
    out12[3] = occ_one<false, true, 0>();
    out12[4] = occ_one<false, true, 1>();
    out12[5] = occ_one<false, true, 2>();
    out12[6] = occ_one<true, false, 0>();
    out12[7] = occ_one<true, false, 1>();
    out12[8] = occ_one<true, false, 2>();
    out12[9] = occ_one<true, true, 0>();
    out12[10] = occ_one<true, true, 1>();
    out12[11] = occ_one<true, true, 2>();
    out18[12] = occ_ord<false, 0>();
    out18[13] = occ_ord<false, 1>();
    out18[14] = occ_ord<false, 2>();
    out18[15] = occ_ord<true, 0>();
    out18[16] = occ_ord<true, 1>();
    out18[17] = occ_ord<true, 2>();
    return hipGetLastError();
}

uint32_t tt_trace_block_size() { return TT_BLOCK; }
uint32_t tt_trace_chunk_rays() { return TT_CHUNK_BIG; }
uint32_t tt_trace_lds_bytes() { return (uint32_t)(TT_LDS_STACK * TT_BLOCK * sizeof(uint2)); }
uint32_t tt_trace_spill_entries() {
    return TT_LDS_STACK >= TT_STACK_SIZE ? 0u : (uint32_t)(TT_STACK_SIZE - TT_LDS_STACK);
}
