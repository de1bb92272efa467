// tt_group.hip — multi-GPU tile-sharded frames behind the C ABI (include/truetrace_hip.h, "multi-GPU
// tile-sharded frames").
//
// The reference traces a frame on one GPU: RayTracingMaster.RenderImage issues Generate, then per bounce
// kernel_trace / kernel_shade (RayTracingMaster.cs:954-1007). Here the frame is cut into tile x tile
// screen tiles dealt round-robin over the group's ranks; each member generates its tiles' camera rays
// (tt_generate_list_kernel: bit for bit Generate's rays of those pixels), traces them with
// tt_trace_closest_hits (the 16-B records written contiguously into the member's send buffer), and ONE
// RCCL gather -- ncclSend from every rank, ncclRecv of every rank's block on rank 0, fused in one
// ncclGroupStart/End -- brings them to rank 0, where tt_group_scatter_kernel puts them back in screen
// order. The scene is replicated per device (a Sponza / Bistro / San Miguel CWBVH is well under 2 GB
// of a 288 GB HBM3E device), so nothing else crosses xGMI. The bounce chain (enqueue + indirect trace)
// stays on each member's device.
//
// Per member and frame slot: one context (slot 0 lends its scene to the others, tt_ctx_share_scene) on a
// dedicated hardware-queue stream (tt_stream_create), the slot's ray buffer, send buffer and device
// bounce count. Per member: one communication stream for the gather. Frame k runs on slot k % slots, so a
// member's frame k + 1 primary launch overlaps frame k's bounce drain and gather. A group of one rank traces
// the identity pixel order straight into the caller's hits_out / info_out (no gather, no scatter).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/truetrace_hip.h"

hipError_t tt_launch_generate_list(const float* c2w, const float* ip, const uint32_t* pixels, uint32_t n,
                                   uint32_t batch, uint32_t w, uint32_t h, float near_plane, float far_plane,
                                   int32_t jitter, int32_t frames, int32_t max_bounce, tt_ray_data* rays,
                                   hipStream_t st);

#define TT_GROUP_MAX_SLOTS 8u

namespace {

// ------------------------------------------------------------------ RCCL, resolved at run time
// dlopen by soname: a process that already holds an RCCL (PyTorch's torch/lib/librccl.so has the same
// soname librccl.so.1) gets that one, so one process never runs two RCCL copies; otherwise the system's.
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto get = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                all = false;
                r.why += std::string(" missing ") + name;
            }
        };
        get(r.GetUniqueId, "ncclGetUniqueId");
        get(r.CommInitRank, "ncclCommInitRank");
        get(r.CommInitAll, "ncclCommInitAll");
        get(r.CommDestroy, "ncclCommDestroy");
        get(r.GroupStart, "ncclGroupStart");
        get(r.GroupEnd, "ncclGroupEnd");
        get(r.Send, "ncclSend");
        get(r.Recv, "ncclRecv");
        get(r.GetErrorString, "ncclGetErrorString");
        r.ok = all;
    });
    return r;
}

// ------------------------------------------------------------------ kernels
// Back to screen order on rank 0. The gathered records are rank-major blocks, rank q's block its B frames'
// records back to back, each frame in the member's trace order; record j of the rank-order concatenation of the
// members' pixel lists (pixel order[j], of rank q, its l-th) sits for frame b at base[j] + b * stride[j]
// (base = B * shard_off[q] + l, stride = shard_n[q]): frame b's record goes to out[b * WH + order[j]]. With
// _PrimaryTriangleInfo gathered too (TT_GROUP_INFO) the info texels follow all records at recv + B * WH.
__global__ __launch_bounds__(256) void tt_group_scatter_kernel(const uint4* __restrict__ recv,
                                                               const uint32_t* __restrict__ order,
                                                               const uint32_t* __restrict__ base,
                                                               const uint32_t* __restrict__ stride, uint32_t wh,
                                                               uint32_t batch, uint4* __restrict__ out,
                                                               uint4* __restrict__ info_out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= wh * batch) return;
    const uint32_t b = t / wh, j = t - b * wh;
    const uint32_t src = base[j] + b * stride[j], dst = b * wh + order[j];
    out[dst] = recv[src];
    if (info_out) info_out[dst] = recv[(size_t)wh * batch + src];
}
// A member's _PrimaryTriangleInfo texels (written at their pixels of the B-frames-tall screen by the primary trace)
// packed in its ray order behind its hit records, so they travel with them.
__global__ __launch_bounds__(256) void tt_group_pack_info_kernel(const uint4* __restrict__ info_full,
                                                                 const uint32_t* __restrict__ pixels, uint32_t n,
                                                                 uint32_t batch, uint32_t wh, uint4* __restrict__ dst) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n * batch) return;
    const uint32_t b = r / n;
    dst[r] = info_full[pixels[r - b * n] + b * wh];
}

// ------------------------------------------------------------------ shard arithmetic
void tile_pixels(uint32_t W, uint32_t H, uint32_t tile, uint32_t world, uint32_t rank, std::vector<uint32_t>& out) {
    out.clear();
    if (world == 1) {  // the identity: the trace kernel's own full-frame 8x8 swizzle keeps waves coherent
        out.resize((size_t)W * H);
        for (uint32_t i = 0; i < W * H; i++) out[i] = i;
        return;
    }
    const uint32_t tx = (W + tile - 1) / tile, ty = (H + tile - 1) / tile;
    for (uint32_t t = rank; t < tx * ty; t += world) {
        const uint32_t x0 = (t % tx) * tile, y0 = (t / tx) * tile;
        const uint32_t x1 = std::min(x0 + tile, W), y1 = std::min(y0 + tile, H);
        for (uint32_t by = y0; by < y1; by += 8)
            for (uint32_t bx = x0; bx < x1; bx += 8)
                for (uint32_t y = by; y < std::min(by + 8, y1); y++)
                    for (uint32_t x = bx; x < std::min(bx + 8, x1); x++) out.push_back(y * W + x);
    }
}

uint64_t tile_count(uint32_t W, uint32_t H, uint32_t tile, uint32_t world, uint32_t rank) {
    if (world == 1) return (uint64_t)W * H;
    const uint32_t tx = (W + tile - 1) / tile, ty = (H + tile - 1) / tile;
    uint64_t n = 0;
    for (uint32_t t = rank; t < tx * ty; t += world) {
        const uint32_t x0 = (t % tx) * tile, y0 = (t / tx) * tile;
        n += (uint64_t)(std::min(x0 + tile, W) - x0) * (std::min(y0 + tile, H) - y0);
    }
    return n;
}

template <class T>
struct Dev {
    T* p = nullptr;
    hipError_t alloc(size_t n) {
        return hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(1, n) * sizeof(T));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
};

struct Member {
    int device = 0;
    uint32_t rank = 0;
    uint32_t n = 0;  // primary rays (pixels of its tiles)
    tt_ctx* ctx[TT_GROUP_MAX_SLOTS] = {};
    void* stream[TT_GROUP_MAX_SLOTS] = {};
    void* comm_stream = nullptr;
    ncclComm_t comm = nullptr;
    Dev<tt_ray_data> rays[TT_GROUP_MAX_SLOTS];
    Dev<uint4> send[TT_GROUP_MAX_SLOTS];       // hit records [0, B n) (+ info texels [B n, 2 B n) with TT_GROUP_INFO)
    Dev<uint4> info_full[TT_GROUP_MAX_SLOTS];  // TT_GROUP_INFO: the primary trace's _PrimaryTriangleInfo, B W H
    Dev<uint32_t> count[TT_GROUP_MAX_SLOTS];  // bounce-1 survivors of the slot's last frame
    Dev<uint32_t> pixels;
    hipEvent_t ev_prim[TT_GROUP_MAX_SLOTS] = {};  // the slot's primary records are final
    hipEvent_t ev_sent[TT_GROUP_MAX_SLOTS] = {};  // the gather that last read the slot's send buffer is done
    bool sent_used[TT_GROUP_MAX_SLOTS] = {};
};

}  // namespace

struct tt_group {
    uint32_t W = 0, H = 0, tile = 64, slots = 2, flags = 0, world = 0;
    uint32_t B = 1;  // frames per call (tt_group_config.batch)
    bool bounce = false, copy = false, info = false;
    bool direct = false;  // one rank: traced straight into the caller's outputs (tt_group_trace_frame)
    std::vector<Member> m;
    std::vector<uint64_t> shard_n, shard_off;  // per rank
    // rank 0's side (when this process holds it: member 0)
    bool root = false;
    Dev<uint4> recv[TT_GROUP_MAX_SLOTS];  // B W H hit records in rank order (+ B W H info texels, TT_GROUP_INFO)
    Dev<uint32_t> order, base, stride;    // the scatter's tables (tt_group_scatter_kernel)
    Dev<uint4> stage;  // screen-order records for a host hits_out (copied back by a synchronous frame)
    uint64_t frame = 0;
    std::string err;
};

namespace {

tt_status gfail(tt_group* g, tt_status s, const char* fmt, ...) {
    if (g) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        g->err = buf;
    }
    return s;
}

#define G_HIP(g, call)                                                                                      \
    do {                                                                                                    \
        hipError_t e_ = (call);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return gfail(g, e_ == hipErrorOutOfMemory ? TT_ERR_OOM : TT_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)
#define G_NCCL(g, call)                                                                                     \
    do {                                                                                                    \
        ncclResult_t r_ = (call);                                                                           \
        if (r_ != ncclSuccess) return gfail(g, TT_ERR_HIP, "%s: %s", #call, rccl().GetErrorString(r_));     \
    } while (0)
#define G_TT(g, m, call)                                                                                    \
    do {                                                                                                    \
        tt_status s_ = (call);                                                                              \
        if (s_ != TT_OK) return gfail(g, s_, "%s: %s", #call, tt_last_error((m)));                          \
    } while (0)

bool check_config(const tt_group_config* cfg, std::string& why) {
    if (!cfg) return why = "null config", false;
    if (!cfg->width || !cfg->height) return why = "zero screen size", false;
    if ((uint64_t)cfg->width * cfg->height > (1ull << 27)) return why = "screen above 2^27 pixels", false;
    const uint32_t tile = cfg->tile ? cfg->tile : 64;
    if (tile % 8) return why = "tile must be a multiple of 8", false;
    if (cfg->slots > TT_GROUP_MAX_SLOTS) return why = "at most 8 slots", false;
    if (cfg->flags & ~(uint32_t)(TT_GROUP_COPY_GATHER | TT_GROUP_BOUNCE | TT_GROUP_INFO)) return why = "unknown flags", false;
    const uint32_t B = cfg->batch ? cfg->batch : 1;
    if (B > 16) return why = "at most 16 frames per call", false;
    // (the batch is one screen B frames tall: its pixels and a member's B n rays per launch stay below 2^27)
    if ((uint64_t)cfg->width * cfg->height * B > (1ull << 27)) return why = "batch x screen above 2^27 pixels", false;
    return true;
}

// everything but the communicators: shard sizes, per-member contexts / streams / buffers, rank 0's side
tt_status setup(tt_group* g, const tt_group_config* cfg) {
    g->W = cfg->width;
    g->H = cfg->height;
    g->tile = cfg->tile ? cfg->tile : 64;
    g->slots = cfg->slots ? cfg->slots : 2;
    g->flags = cfg->flags;
    g->bounce = (cfg->flags & TT_GROUP_BOUNCE) != 0;
    g->copy = (cfg->flags & TT_GROUP_COPY_GATHER) != 0;
    g->info = (cfg->flags & TT_GROUP_INFO) != 0;
    g->B = cfg->batch ? cfg->batch : 1;
    // TT_GROUP_FORCE_GATHER=1 keeps a one-rank group on the gather + scatter path (tools/group_scale.py: one GPU
    // standing in for one rank of an N-GPU node)
    const char* fg = std::getenv("TT_GROUP_FORCE_GATHER");
    g->direct = g->world == 1 && !(fg && std::atoi(fg) != 0);
    const size_t K = g->info ? 2 : 1;  // records per ray in the gather
    const uint64_t WH = (uint64_t)g->W * g->H, B = g->B;
    g->shard_n.resize(g->world);
    g->shard_off.resize(g->world);
    uint64_t off = 0;
    for (uint32_t r = 0; r < g->world; r++) {
        g->shard_n[r] = tile_count(g->W, g->H, g->tile, g->world, r);
        g->shard_off[r] = off;
        off += g->shard_n[r];
    }
    std::vector<uint32_t> pix;
    for (Member& mb : g->m) {
        G_HIP(g, hipSetDevice(mb.device));
        tile_pixels(g->W, g->H, g->tile, g->world, mb.rank, pix);
        mb.n = (uint32_t)pix.size();
        G_HIP(g, mb.pixels.alloc(pix.size()));
        if (!pix.empty()) G_HIP(g, hipMemcpy(mb.pixels.p, pix.data(), 4 * pix.size(), hipMemcpyHostToDevice));
        G_TT(g, nullptr, tt_stream_create(mb.device, &mb.comm_stream));
        for (uint32_t s = 0; s < g->slots; s++) {
            G_TT(g, nullptr, tt_stream_create(mb.device, &mb.stream[s]));
            tt_config c{};
            c.device = mb.device;
            c.stream = mb.stream[s];
            if (tt_ctx_create(&c, &mb.ctx[s]) != TT_OK) return gfail(g, TT_ERR_HIP, "tt_ctx_create on device %d", mb.device);
            (void)tt_ctx_set_timing(mb.ctx[s], 0);  // no per-launch event pair (a host turns it on per context)
            if (B > 1) (void)tt_ctx_set_frame_pixels(mb.ctx[s], (uint32_t)WH);
            G_HIP(g, hipSetDevice(mb.device));
            // GlobalRays of the B-frames-tall screen: the primary rays at [0, B n), bounce 1 at [B W H, + B n)
            G_HIP(g, mb.rays[s].alloc(B * (WH + mb.n)));
            if (!g->direct) {  // (a one-rank group traces straight into the caller's buffers: tt_group_trace_frame)
                G_HIP(g, mb.send[s].alloc(K * B * mb.n));
                if (g->info) G_HIP(g, mb.info_full[s].alloc(B * WH));
            }
            G_HIP(g, mb.count[s].alloc(1));
            G_HIP(g, hipMemset(mb.count[s].p, 0, 4));
            G_HIP(g, hipEventCreateWithFlags(&mb.ev_prim[s], hipEventDisableTiming));
            G_HIP(g, hipEventCreateWithFlags(&mb.ev_sent[s], hipEventDisableTiming));
        }
    }
    if (g->root && !g->direct) {
        Member& r0 = g->m[0];
        G_HIP(g, hipSetDevice(r0.device));
        std::vector<uint32_t> order, base, stride;
        order.reserve(WH);
        base.reserve(WH);
        stride.reserve(WH);
        for (uint32_t r = 0; r < g->world; r++) {
            tile_pixels(g->W, g->H, g->tile, g->world, r, pix);
            order.insert(order.end(), pix.begin(), pix.end());
            for (uint32_t l = 0; l < (uint32_t)pix.size(); l++) {
                base.push_back((uint32_t)(B * g->shard_off[r] + l));
                stride.push_back((uint32_t)g->shard_n[r]);
            }
        }
        G_HIP(g, g->order.alloc(order.size()));
        G_HIP(g, hipMemcpy(g->order.p, order.data(), 4 * order.size(), hipMemcpyHostToDevice));
        G_HIP(g, g->base.alloc(base.size()));
        G_HIP(g, hipMemcpy(g->base.p, base.data(), 4 * base.size(), hipMemcpyHostToDevice));
        G_HIP(g, g->stride.alloc(stride.size()));
        G_HIP(g, hipMemcpy(g->stride.p, stride.data(), 4 * stride.size(), hipMemcpyHostToDevice));
        for (uint32_t s = 0; s < g->slots; s++) G_HIP(g, g->recv[s].alloc(K * B * WH));
    }
    return TT_OK;
}

void teardown(tt_group* g) {
    for (Member& mb : g->m) {
        (void)hipSetDevice(mb.device);
        for (uint32_t s = 0; s < TT_GROUP_MAX_SLOTS; s++)
            if (mb.stream[s]) (void)hipStreamSynchronize(static_cast<hipStream_t>(mb.stream[s]));
        if (mb.comm_stream) (void)hipStreamSynchronize(static_cast<hipStream_t>(mb.comm_stream));
    }
    for (Member& mb : g->m) {
        (void)hipSetDevice(mb.device);
        if (mb.comm) (void)rccl().CommDestroy(mb.comm);
        mb.comm = nullptr;
        for (uint32_t s = TT_GROUP_MAX_SLOTS; s-- > 0;)  // borrowers before the lender (slot 0)
            if (mb.ctx[s]) (void)tt_ctx_destroy(mb.ctx[s]);
        for (uint32_t s = 0; s < TT_GROUP_MAX_SLOTS; s++) {
            mb.rays[s].release();
            mb.send[s].release();
            mb.info_full[s].release();
            mb.count[s].release();
            if (mb.ev_prim[s]) (void)hipEventDestroy(mb.ev_prim[s]);
            if (mb.ev_sent[s]) (void)hipEventDestroy(mb.ev_sent[s]);
            if (mb.stream[s]) (void)tt_stream_destroy(mb.stream[s]);
        }
        mb.pixels.release();
        if (mb.comm_stream) (void)tt_stream_destroy(mb.comm_stream);
    }
    if (!g->m.empty()) (void)hipSetDevice(g->m[0].device);
    for (uint32_t s = 0; s < TT_GROUP_MAX_SLOTS; s++) g->recv[s].release();
    g->order.release();
    g->base.release();
    g->stride.release();
    g->stage.release();
    (void)hipGetLastError();
}

int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

// 1: device memory of `device`; 0: host memory (pageable or pinned); -1: device memory of another device
int where(const void* p, int device) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return a.device == device ? 1 : -1;
    return 0;
}

}  // namespace

extern "C" {

tt_status tt_group_tile_pixels(uint32_t width, uint32_t height, uint32_t tile, uint32_t world, uint32_t rank,
                               uint32_t* pixels, uint32_t max, uint32_t* n) {
    if (!n || (max && !pixels) || !width || !height || !world || rank >= world || !tile || tile % 8 ||
        (uint64_t)width * height > 0xffffffffull)
        return TT_ERR_INVALID_ARG;
    std::vector<uint32_t> pix;
    tile_pixels(width, height, tile, world, rank, pix);
    const size_t k = std::min<size_t>(pix.size(), max);
    if (k) std::memcpy(pixels, pix.data(), 4 * k);
    *n = (uint32_t)pix.size();
    return TT_OK;
}

tt_status tt_group_create(const int32_t* devices, uint32_t n, const tt_group_config* cfg, tt_group** out) {
    if (!out) return TT_ERR_INVALID_ARG;
    *out = nullptr;
    std::string why;
    if (!devices || !n || !check_config(cfg, why)) return TT_ERR_INVALID_ARG;
    const int ndev = device_count();
    if (ndev == 0) return TT_ERR_NO_DEVICE;
    const bool copy = (cfg->flags & TT_GROUP_COPY_GATHER) != 0;
    for (uint32_t i = 0; i < n; i++) {
        if (devices[i] < 0 || devices[i] >= ndev) return TT_ERR_INVALID_ARG;
        for (uint32_t j = 0; j < i && !copy; j++)
            if (devices[j] == devices[i]) return TT_ERR_INVALID_ARG;  // RCCL: one rank per device
    }
    if (!copy && !rccl().ok) return TT_ERR_UNSUPPORTED;
    tt_group* g = new tt_group();
    g->world = n;
    g->root = true;
    g->m.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        g->m[i].device = devices[i];
        g->m[i].rank = i;
    }
    tt_status st = setup(g, cfg);
    if (st == TT_OK && !copy) {
        std::vector<ncclComm_t> comms(n);
        std::vector<int> devs(devices, devices + n);
        const ncclResult_t r = rccl().CommInitAll(comms.data(), (int)n, devs.data());
        if (r != ncclSuccess) {
            st = gfail(g, TT_ERR_HIP, "ncclCommInitAll: %s", rccl().GetErrorString(r));
        } else {
            for (uint32_t i = 0; i < n; i++) g->m[i].comm = comms[i];
        }
    }
    if (st != TT_OK) {
        teardown(g);
        delete g;
        return st;
    }
    *out = g;
    return TT_OK;
}

tt_status tt_group_unique_id(uint8_t id[128]) {
    if (!id) return TT_ERR_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    if (!rccl().ok) return TT_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (rccl().GetUniqueId(&u) != ncclSuccess) return TT_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return TT_OK;
}

tt_status tt_group_create_rank(const uint8_t id[128], uint32_t world, uint32_t rank, int32_t device,
                               const tt_group_config* cfg, tt_group** out) {
    if (!out) return TT_ERR_INVALID_ARG;
    *out = nullptr;
    std::string why;
    if (!id || !world || rank >= world || !check_config(cfg, why)) return TT_ERR_INVALID_ARG;
    if (cfg->flags & TT_GROUP_COPY_GATHER) return TT_ERR_INVALID_ARG;  // copies need one process
    const int ndev = device_count();
    if (ndev == 0) return TT_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return TT_ERR_INVALID_ARG;
    if (!rccl().ok) return TT_ERR_UNSUPPORTED;
    tt_group* g = new tt_group();
    g->world = world;
    g->root = rank == 0;
    g->m.resize(1);
    g->m[0].device = device;
    g->m[0].rank = rank;
    tt_status st = setup(g, cfg);
    if (st == TT_OK) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        (void)hipSetDevice(device);
        const ncclResult_t r = rccl().CommInitRank(&g->m[0].comm, (int)world, u, (int)rank);
        if (r != ncclSuccess) st = gfail(g, TT_ERR_HIP, "ncclCommInitRank: %s", rccl().GetErrorString(r));
    }
    if (st != TT_OK) {
        teardown(g);
        delete g;
        return st;
    }
    *out = g;
    return TT_OK;
}

tt_status tt_group_destroy(tt_group* g) {
    if (!g) return TT_ERR_INVALID_ARG;
    teardown(g);
    delete g;
    return TT_OK;
}

const char* tt_group_last_error(const tt_group* g) { return g ? g->err.c_str() : "null group"; }

uint32_t tt_group_local_members(const tt_group* g) { return g ? (uint32_t)g->m.size() : 0u; }

tt_ctx* tt_group_member_ctx(tt_group* g, uint32_t m) {
    return (g && m < g->m.size()) ? g->m[m].ctx[0] : nullptr;
}

}  // extern "C"

namespace {
// An upload to every member's scene context (slot 0). The other slots borrow its scene, and a lender with
// borrowers refuses uploads: they let go first and share the new scene after (up = the upload per member).
template <class Up>
tt_status reupload(tt_group* g, Up up) {
    for (Member& mb : g->m)
        for (uint32_t s = 1; s < g->slots; s++) {
            if (mb.ctx[s]) (void)tt_ctx_destroy(mb.ctx[s]);
            mb.ctx[s] = nullptr;
        }
    for (Member& mb : g->m) {
        tt_ctx* c0 = mb.ctx[0];
        G_TT(g, c0, up(c0));
        for (uint32_t s = 1; s < g->slots; s++) {
            tt_config c{};
            c.device = mb.device;
            c.stream = mb.stream[s];
            if (tt_ctx_create(&c, &mb.ctx[s]) != TT_OK) return gfail(g, TT_ERR_HIP, "tt_ctx_create on device %d", mb.device);
            (void)tt_ctx_set_timing(mb.ctx[s], 0);
            if (g->B > 1) (void)tt_ctx_set_frame_pixels(mb.ctx[s], g->W * g->H);
            G_TT(g, mb.ctx[s], tt_ctx_share_scene(mb.ctx[s], c0));
        }
    }
    return TT_OK;
}
}  // namespace

extern "C" {

tt_status tt_group_scene_upload(tt_group* g, const tt_cwbvh_node* nodes, uint32_t n_nodes, const tt_cuda_triangle* tris,
                                uint32_t n_tris, const int32_t* tlas, uint32_t n_tlas, const tt_mesh_data* md,
                                uint32_t n_mesh, const tt_material* mats, uint32_t n_mat) {
    if (!g) return TT_ERR_INVALID_ARG;
    return reupload(g, [&](tt_ctx* c) {
        return tt_scene_upload(c, nodes, n_nodes, tris, n_tris, tlas, n_tlas, md, n_mesh, mats, n_mat);
    });
}

tt_status tt_group_scene_upload_alpha_atlas(tt_group* g, const uint8_t* texels, uint32_t width, uint32_t height) {
    if (!g) return TT_ERR_INVALID_ARG;
    return reupload(g, [&](tt_ctx* c) { return tt_scene_upload_alpha_atlas(c, texels, width, height); });
}

tt_status tt_group_scene_upload_texture_atlas(tt_group* g, const uint16_t* rgba_half, uint32_t width, uint32_t height) {
    if (!g) return TT_ERR_INVALID_ARG;
    return reupload(g, [&](tt_ctx* c) { return tt_scene_upload_texture_atlas(c, rgba_half, width, height); });
}

// Per-frame scene updates on every member's scene context (AssetManager.cs:1760-1825 per device): the slots
// borrow that scene, and the library orders each update after their traces already issued and before the
// ones issued after it (tt_ctx_share_scene), so a host calls these between frames with no synchronisation.
tt_status tt_group_scene_update_meshdata(tt_group* g, uint32_t first, uint32_t count, const tt_mesh_data* md) {
    if (!g) return TT_ERR_INVALID_ARG;
    for (Member& mb : g->m) G_TT(g, mb.ctx[0], tt_scene_update_meshdata(mb.ctx[0], first, count, md));
    return TT_OK;
}

tt_status tt_group_scene_update_nodes(tt_group* g, uint32_t first, uint32_t count, const tt_cwbvh_node* nodes) {
    if (!g) return TT_ERR_INVALID_ARG;
    for (Member& mb : g->m) G_TT(g, mb.ctx[0], tt_scene_update_nodes(mb.ctx[0], first, count, nodes));
    return TT_OK;
}

tt_status tt_group_tlas_refit(tt_group* g, uint32_t n_tlas_nodes, const float* mesh_aabbs, uint32_t n_mesh,
                              uint32_t flags) {
    if (!g) return TT_ERR_INVALID_ARG;
    if (flags & TT_TRACE_DEVICE_PTRS)  // (one device array cannot serve every member's device)
        return gfail(g, TT_ERR_INVALID_ARG, "tt_group_tlas_refit takes host mesh AABBs");
    for (Member& mb : g->m)
        G_TT(g, mb.ctx[0], tt_tlas_refit(mb.ctx[0], n_tlas_nodes, mesh_aabbs, n_mesh, flags & TT_TRACE_ASYNC));
    return TT_OK;
}

tt_status tt_group_trace_frame(tt_group* g, const tt_camera* cam, uint32_t* hits_out, uint32_t* info_out,
                               uint32_t flags) {
    if (!g) return TT_ERR_INVALID_ARG;
    if (!cam) return gfail(g, TT_ERR_INVALID_ARG, "null camera");
    if (cam->width != g->W || cam->height != g->H)
        return gfail(g, TT_ERR_INVALID_ARG, "camera is %ux%u, the group's screen %ux%u", cam->width, cam->height, g->W, g->H);
    if (cam->far_plane != cam->far_plane) return gfail(g, TT_ERR_INVALID_ARG, "far_plane is NaN");
    bool host_out = false;
    if (g->root) {
        if (!hits_out) return gfail(g, TT_ERR_INVALID_ARG, "rank 0 needs hits_out");
        if (reinterpret_cast<uintptr_t>(hits_out) % 16) return gfail(g, TT_ERR_INVALID_ARG, "hits_out must be 16-byte aligned");
        const int w = where(hits_out, g->m[0].device);
        if (w < 0) return gfail(g, TT_ERR_INVALID_ARG, "hits_out is device memory of another device than rank 0's (%d)",
                                g->m[0].device);
        if (w == 0 && (flags & TT_TRACE_ASYNC))
            return gfail(g, TT_ERR_INVALID_ARG, "a host hits_out needs a synchronous frame (no TT_TRACE_ASYNC)");
        host_out = w == 0;
        if (g->info) {  // the info texels' buffer: the same kind of memory as hits_out
            if (!info_out) return gfail(g, TT_ERR_INVALID_ARG, "TT_GROUP_INFO: rank 0 needs info_out");
            if (reinterpret_cast<uintptr_t>(info_out) % 16) return gfail(g, TT_ERR_INVALID_ARG, "info_out must be 16-byte aligned");
            if (where(info_out, g->m[0].device) != w)
                return gfail(g, TT_ERR_INVALID_ARG, "info_out must be the same kind of memory as hits_out");
        }
        if (host_out && !g->stage.p) {
            G_HIP(g, hipSetDevice(g->m[0].device));
            G_HIP(g, g->stage.alloc((g->info ? 2 : 1) * (size_t)g->B * g->W * g->H));
        }
    }
    const uint32_t s = (uint32_t)(g->frame % g->slots);
    const bool async = (flags & TT_TRACE_ASYNC) != 0;
    const uint32_t tflags = TT_TRACE_DEVICE_PTRS | TT_TRACE_ASYNC;
    const uint32_t B = g->B, WH = g->W * g->H, HB = g->H * B;  // the batch traces as one W x B H screen
    // A group of one rank (world 1) traces the identity pixel order: ray b n + j is pixel j of frame b, so its
    // records and info texels are already in hits_out / info_out order -- the trace writes them there directly
    // and there is nothing to gather or scatter (host outputs: through the staging buffer).
    const bool direct = g->direct;
    // 1. every member: Generate its tiles of the B frames, trace them (records into its send buffer)
    for (Member& mb : g->m) {
        hipStream_t st = static_cast<hipStream_t>(mb.stream[s]);
        G_HIP(g, hipSetDevice(mb.device));
        // the send buffer is free again once the gather that last read it is done (rank 0's copies: its event)
        if (mb.sent_used[s] && !direct)
            G_HIP(g, hipStreamWaitEvent(st, g->copy ? g->m[0].ev_sent[s] : mb.ev_sent[s], 0));
        G_HIP(g, tt_launch_generate_list(cam->cam_to_world, cam->cam_inv_proj, mb.pixels.p, mb.n, B, g->W, g->H,
                                         cam->near_plane, cam->far_plane, cam->jitter, cam->frames_accumulated,
                                         cam->max_bounce, mb.rays[s].p, st));
        tt_trace_params p{};
        p.n_rays = B * mb.n;
        p.bounce = 0;
        p.far_plane = cam->far_plane;
        p.screen_width = g->W;
        p.screen_height = HB;
        p.flags = tflags;
        if (direct) {
            uint4* oh = host_out ? g->stage.p : reinterpret_cast<uint4*>(hits_out);
            uint4* oi = !g->info ? nullptr : host_out ? g->stage.p + (size_t)B * WH : reinterpret_cast<uint4*>(info_out);
            G_TT(g, mb.ctx[s], tt_trace_closest_hits(mb.ctx[s], &p, mb.rays[s].p, reinterpret_cast<uint32_t*>(oi), nullptr,
                                                     reinterpret_cast<uint32_t*>(oh)));
            if (host_out) {
                G_HIP(g, hipMemcpyAsync(hits_out, oh, (size_t)B * WH * 16, hipMemcpyDeviceToHost, st));
                if (g->info) G_HIP(g, hipMemcpyAsync(info_out, oi, (size_t)B * WH * 16, hipMemcpyDeviceToHost, st));
            }
            continue;
        }
        if (mb.n) G_TT(g, mb.ctx[s], tt_trace_closest_hits(mb.ctx[s], &p, mb.rays[s].p,
                                                           g->info ? reinterpret_cast<uint32_t*>(mb.info_full[s].p) : nullptr,
                                                           nullptr, reinterpret_cast<uint32_t*>(mb.send[s].p)));
        if (g->info && mb.n) {
            hipLaunchKernelGGL(tt_group_pack_info_kernel, dim3((B * mb.n + 255u) / 256u), dim3(256), 0, st,
                               mb.info_full[s].p, mb.pixels.p, mb.n, B, WH, mb.send[s].p + (size_t)B * mb.n);
            G_HIP(g, hipGetLastError());
        }
        G_HIP(g, hipEventRecord(mb.ev_prim[s], st));
    }
    // 2. the gather: one fused RCCL group (or device copies) on the communication streams; a rank's message is
    // its B frames' records back to back (and as many info texels after them)
    const size_t info_at = (size_t)B * WH;  // the info texels' region of rank 0's receive buffer
    if (direct) {
        // (nothing crosses devices)
    } else if (!g->copy) {
        for (Member& mb : g->m) {
            G_HIP(g, hipSetDevice(mb.device));
            G_HIP(g, hipStreamWaitEvent(static_cast<hipStream_t>(mb.comm_stream), mb.ev_prim[s], 0));
        }
        G_NCCL(g, rccl().GroupStart());
        ncclResult_t r = ncclSuccess;
        for (Member& mb : g->m) {
            hipStream_t cs = static_cast<hipStream_t>(mb.comm_stream);
            const size_t cnt = (size_t)B * mb.n * 4;  // uint32 words of the rank's records
            if (r == ncclSuccess && mb.n) r = rccl().Send(mb.send[s].p, cnt, ncclUint32, 0, mb.comm, cs);
            if (r == ncclSuccess && mb.n && g->info)
                r = rccl().Send(mb.send[s].p + (size_t)B * mb.n, cnt, ncclUint32, 0, mb.comm, cs);
            if (mb.rank == 0)
                for (uint32_t q = 0; q < g->world && r == ncclSuccess; q++)
                    if (g->shard_n[q]) {
                        const size_t at = (size_t)B * g->shard_off[q], qcnt = (size_t)B * g->shard_n[q] * 4;
                        r = rccl().Recv(g->recv[s].p + at, qcnt, ncclUint32, (int)q, mb.comm, cs);
                        if (r == ncclSuccess && g->info)  // (messages between one pair match in call order)
                            r = rccl().Recv(g->recv[s].p + info_at + at, qcnt, ncclUint32, (int)q, mb.comm, cs);
                    }
        }
        const ncclResult_t re = rccl().GroupEnd();
        if (r != ncclSuccess || re != ncclSuccess)
            return gfail(g, TT_ERR_HIP, "RCCL gather: %s", rccl().GetErrorString(r != ncclSuccess ? r : re));
        for (Member& mb : g->m) {
            G_HIP(g, hipSetDevice(mb.device));
            G_HIP(g, hipEventRecord(mb.ev_sent[s], static_cast<hipStream_t>(mb.comm_stream)));
            mb.sent_used[s] = true;
        }
    } else {
        Member& r0 = g->m[0];
        hipStream_t cs = static_cast<hipStream_t>(r0.comm_stream);
        G_HIP(g, hipSetDevice(r0.device));
        for (Member& mb : g->m) {
            G_HIP(g, hipStreamWaitEvent(cs, mb.ev_prim[s], 0));
            const size_t at = (size_t)B * g->shard_off[mb.rank], bytes = (size_t)B * mb.n * 16;
            if (mb.n) G_HIP(g, hipMemcpyAsync(g->recv[s].p + at, mb.send[s].p, bytes, hipMemcpyDeviceToDevice, cs));
            if (mb.n && g->info)
                G_HIP(g, hipMemcpyAsync(g->recv[s].p + info_at + at, mb.send[s].p + (size_t)B * mb.n, bytes,
                                        hipMemcpyDeviceToDevice, cs));
        }
        G_HIP(g, hipEventRecord(r0.ev_sent[s], cs));
        for (Member& mb : g->m) mb.sent_used[s] = true;
    }
    // rank 0: back to screen order (after its communication stream's receives)
    if (g->root && !direct) {
        Member& r0 = g->m[0];
        G_HIP(g, hipSetDevice(r0.device));
        uint4* oh = host_out ? g->stage.p : reinterpret_cast<uint4*>(hits_out);
        uint4* oi = !g->info ? nullptr : host_out ? g->stage.p + info_at : reinterpret_cast<uint4*>(info_out);
        hipLaunchKernelGGL(tt_group_scatter_kernel, dim3((B * WH + 255u) / 256u), dim3(256), 0,
                           static_cast<hipStream_t>(r0.comm_stream), g->recv[s].p, g->order.p, g->base.p, g->stride.p,
                           WH, B, oh, oi);
        G_HIP(g, hipGetLastError());
        if (host_out) {
            G_HIP(g, hipMemcpyAsync(hits_out, g->stage.p, info_at * 16, hipMemcpyDeviceToHost,
                                    static_cast<hipStream_t>(r0.comm_stream)));
            if (g->info)
                G_HIP(g, hipMemcpyAsync(info_out, g->stage.p + info_at, info_at * 16, hipMemcpyDeviceToHost,
                                        static_cast<hipStream_t>(r0.comm_stream)));
        }
    }
    // 3. bounce 1 on every member's own device (the gather reads only the send buffers, so it overlaps); with
    // B > 1 the enqueue draws frame b's directions from its frame-local pixel at frames + b (frame_pixels = W H)
    if (g->bounce) {
        for (Member& mb : g->m) {
            if (!mb.n) continue;
            tt_trace_params p{};
            p.n_rays = B * mb.n;
            p.bounce = 0;
            p.far_plane = cam->far_plane;
            p.screen_width = g->W;
            p.screen_height = HB;
            p.flags = tflags;
            G_TT(g, mb.ctx[s], tt_enqueue_diffuse_bounce_indirect(mb.ctx[s], &p, nullptr, mb.rays[s].p,
                                                                  cam->frames_accumulated, cam->max_bounce,
                                                                  mb.count[s].p));
            p.bounce = 1;
            G_TT(g, mb.ctx[s], tt_trace_closest_indirect(mb.ctx[s], &p, mb.count[s].p, mb.rays[s].p, nullptr, nullptr));
        }
    }
    g->frame++;
    if (!async) return tt_group_sync(g);
    return TT_OK;
}

tt_status tt_group_sync(tt_group* g) {
    if (!g) return TT_ERR_INVALID_ARG;
    for (Member& mb : g->m) {
        G_HIP(g, hipSetDevice(mb.device));
        for (uint32_t s = 0; s < g->slots; s++) G_HIP(g, hipStreamSynchronize(static_cast<hipStream_t>(mb.stream[s])));
        G_HIP(g, hipStreamSynchronize(static_cast<hipStream_t>(mb.comm_stream)));
    }
    for (Member& mb : g->m)
        for (uint32_t s = 0; s < g->slots; s++) {
            uint64_t ov = 0;
            if (mb.ctx[s] && tt_async_overflows(mb.ctx[s], &ov) != TT_OK)
                return gfail(g, TT_ERR_STACK_OVERFLOW, "member %d: %llu rays overflowed the traversal stack", (int)mb.rank,
                             (unsigned long long)ov);
        }
    return TT_OK;
}

tt_status tt_group_frame_rays(tt_group* g, uint32_t m, uint32_t* n_primary, uint32_t* n_bounce, tt_ray_data** rays_dev) {
    if (!g) return TT_ERR_INVALID_ARG;
    if (m >= g->m.size()) return gfail(g, TT_ERR_INVALID_ARG, "member %u of %zu", m, g->m.size());
    if (g->frame == 0) return gfail(g, TT_ERR_INVALID_ARG, "no frame traced yet");
    Member& mb = g->m[m];
    const uint32_t s = (uint32_t)((g->frame - 1) % g->slots);
    G_HIP(g, hipSetDevice(mb.device));
    G_HIP(g, hipStreamSynchronize(static_cast<hipStream_t>(mb.stream[s])));
    uint32_t nb = 0;
    if (g->bounce) G_HIP(g, hipMemcpy(&nb, mb.count[s].p, 4, hipMemcpyDeviceToHost));
    if (n_primary) *n_primary = g->B * mb.n;
    if (n_bounce) *n_bounce = nb;
    if (rays_dev) *rays_dev = mb.rays[s].p;
    return TT_OK;
}

}  // extern "C"
