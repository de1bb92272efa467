// tt_order.hip — the adaptive dequeue order of TT_TRACE_ADAPTIVE_ORDER launches.
//
// A persistent trace launch ends when its last ray finishes, and a launch's longest rays are
// serial chains of dependent node / triangle fetches (up to ~1 us each when they miss the L2s).
// When such a ray is dequeued late it becomes the launch's tail: on the Bistro-shaped C4 scene a
// 1080p primary launch spends ~0.2 ms of its ~1.06 ms finishing rays that started late
// (profiles/r03/exp_lpt_temporal_c4_c2.txt: longest-chunk-first with the exact costs 0.82 ms, with
// the costs of ANOTHER jittered frame 0.83-0.85 ms -- frames are temporally coherent).
//
// The flagged trace kernel (tt_trace_kernel_ord) records, per 64-ray chunk (the 8x8 pixel tile in
// the full-frame swizzle, else records [64 m, 64 m + 64) of the batch), the largest Reps count of
// its rays that reached TT_ORDER_MIN_REPS; before the next flagged launch of the same bounce index
// this kernel sorts each scheduler segment's chunks by those costs, longest first, and the trace
// kernel maps each dequeue (one whole chunk) through the result. A compacted bounce list shifts
// from frame to frame, so its chunk m is only approximately the previous frame's chunk m: a hint,
// which is all an order needs (results never depend on it).
//
// One block per segment (TT_SEGS, the work ranges the trace kernel's XCD groups dequeue from, so
// each segment keeps its screen band and its L2): a counting sort over OKEYS cost buckets in LDS.
// The histogram and the scatter run in rounds of OB consecutive chunks with a barrier between
// rounds, so chunks of equal cost keep their natural (spatial) order up to a permutation inside
// one round. A launch whose ray count is not a multiple of 64 keeps its partial last chunk last
// (only the last work chunk is partial, and it must stay the partial one).
#include "tt_traverse.h"

namespace {
constexpr uint32_t OB = 256;      // threads per block: small, so the kernel fits beside a running trace
constexpr uint32_t OKEYS = 1024;  // cost buckets (Reps <= TT_MAX_REPS = 1000 fits)
constexpr uint32_t OITEMS = 8;    // chunks per thread per batch: their key loads are in flight together

__device__ __forceinline__ uint32_t chunk_key(const OrderArgs& A, uint32_t m) {
    const uint32_t c = A.cost[m];
    return c < A.hot ? 0u : min(c, OKEYS - 1u);  // below `hot`: one bucket, sorted last, natural order
}

__global__ __launch_bounds__(OB) void tt_order_kernel(OrderArgs A) {
    __shared__ uint32_t s_off[OKEYS];
    __shared__ uint32_t s_wsum[OB / TT_WAVE];
    const uint32_t tid = threadIdx.x, s = blockIdx.x;
    // the map the coming trace fills
    for (uint32_t i = s * OB + tid; i < A.n_chunks; i += TT_SEGS * OB) A.cost_clear[i] = 0u;
    for (uint32_t i = tid; i < OKEYS; i += OB) s_off[i] = 0u;
    __syncthreads();
    const uint32_t lo = (uint32_t)((uint64_t)A.n_chunks * s / TT_SEGS);
    uint32_t hi = (uint32_t)((uint64_t)A.n_chunks * (s + 1) / TT_SEGS);
    if (s == TT_SEGS - 1 && (A.n_rays & 63u) && hi > lo) {
        A.order[hi - 1] = hi - 1;  // the partial chunk stays last
        hi--;
    }
    if (hi <= lo) return;
    const uint32_t n = hi - lo;
    // pass 1: histogram
    for (uint32_t b = 0; b < n; b += OB * OITEMS) {
        uint32_t k[OITEMS];
#pragma unroll
        for (uint32_t i = 0; i < OITEMS; i++) {
            const uint32_t j = b + i * OB + tid;
            k[i] = j < n ? chunk_key(A, lo + j) : OKEYS;
        }
#pragma unroll
        for (uint32_t i = 0; i < OITEMS; i++)
            if (k[i] < OKEYS) atomicAdd(&s_off[k[i]], 1u);
    }
    __syncthreads();
    // exclusive scan in DESCENDING key order: bucket k starts after every bucket k' > k.
    // Thread t owns buckets [1023 - 4t - 3, 1023 - 4t] (4 per thread).
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        c[i] = s_off[OKEYS - 1u - (tid * 4u + i)];
        sum += c[i];
    }
    const uint32_t lane = tid & (TT_WAVE - 1), w = tid >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < TT_WAVE; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d, TT_WAVE);
        if (lane >= (uint32_t)d) incl += v;
    }
    if (lane == TT_WAVE - 1) s_wsum[w] = incl;
    __syncthreads();
    uint32_t base = incl - sum;
    for (uint32_t i = 0; i < w; i++) base += s_wsum[i];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s_off[OKEYS - 1u - (tid * 4u + i)] = base;
        base += c[i];
    }
    __syncthreads();
    // pass 2: scatter, one round of OB consecutive chunks at a time
    for (uint32_t b = 0; b < n; b += OB * OITEMS) {
        uint32_t k[OITEMS];
#pragma unroll
        for (uint32_t i = 0; i < OITEMS; i++) {
            const uint32_t j = b + i * OB + tid;
            k[i] = j < n ? chunk_key(A, lo + j) : OKEYS;
        }
#pragma unroll
        for (uint32_t i = 0; i < OITEMS; i++) {
            if (k[i] < OKEYS) {
                const uint32_t pos = atomicAdd(&s_off[k[i]], 1u);
                A.order[lo + pos] = lo + b + i * OB + tid;
            }
            __syncthreads();
        }
    }
}
}  // namespace

hipError_t tt_launch_order(const OrderArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(tt_order_kernel, dim3(TT_SEGS), dim3(OB), 0, st, a);
    return hipGetLastError();
}
