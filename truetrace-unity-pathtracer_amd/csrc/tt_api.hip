// tt_api.hip — the C ABI of include/truetrace_hip.h: context lifecycle, scene upload with
// structural validation, trace dispatch (the kernel_trace replacement) and the normal resolve.
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "tt_device.h"
#include "tt_refit.h"

#define TT_RING 256u
// Overlay regions behind a scene's nodes (tt_ctx_share_blas): this many frame-slot TLASes per lender
#ifndef TT_TLAS_SLOTS
#define TT_TLAS_SLOTS 8u
#endif

hipError_t tt_launch_trace(const TraceArgs& a, bool stats, bool matcheck, int info, uint32_t grid, hipStream_t st);
uint32_t tt_trace_chunk_rays();
hipError_t tt_trace_occupancy_table(int* out18);
hipError_t tt_launch_shadow(const ShadowArgs* a, uint32_t grid, hipStream_t st, int stats, int matcheck);
hipError_t tt_launch_shadow_accumulate(const ShadowArgs* a, const float4* vis, hipStream_t st);
void tt_shadow_occupancy_table(int* out4);
uint32_t tt_trace_block_size();
uint32_t tt_trace_spill_entries();
uint32_t tt_trace_lds_bytes();
hipError_t tt_launch_generate(const float* c2w, const float* ip, uint32_t w, uint32_t h, float near_plane, float far_plane,
                              int32_t jitter, int32_t frames, int32_t max_bounce, tt_ray_data* rays, hipStream_t st);
hipError_t tt_launch_bounce(tt_ray_data* rays, uint32_t src_off, uint32_t dst_off, uint32_t n, float far_plane,
                            int32_t cur_bounce, int32_t frames, int32_t max_bounce, const tt_cuda_triangle* tris,
                            const tt_mesh_data* md, uint32_t* counter, hipStream_t st, const uint32_t* n_dev,
                            uint32_t* n_next_dev, uint32_t* ctl_next, uint32_t ctl_next_words,
                            uint32_t frame_pixels);
uint32_t tt_bounce_tiles(uint32_t n);
hipError_t tt_launch_resolve(const tt_ray_data* rays, uint32_t ray_offset, uint32_t n, float far_plane,
                             const tt_cuda_triangle* tris, uint32_t n_tris, const tt_mesh_data* md, uint32_t n_mesh,
                             float* out, hipStream_t st);
hipError_t tt_launch_rcp_selftest(unsigned long long* d_bad, hipStream_t st);

namespace {

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        n = count;
        return hipSuccess;
    }
    bool own = true;  // false: borrowed from another context's scene (tt_ctx_share_scene), never freed here
    void release() {
        if (p && own) (void)hipFree(p);
        p = nullptr;
        n = 0;
        own = true;
    }
    void borrow(const DevBuf& o) {
        release();
        p = o.p;
        n = o.n;
        own = false;
    }
};

struct SceneHost {
    std::vector<tt_cwbvh_node> nodes;
    std::vector<int32_t> tlas;
    std::vector<tt_mesh_data> mesh;
    uint32_t n_tris = 0;
    uint32_t n_mat = 0;
    std::vector<uint32_t> matdat;  // only kept when a material sets the Invisible flag
    bool any_shadow_skip = false;  // IsBackground / ShadowCaster present (shadow material checks)
    bool any_atlas_shadow = false; // specTrans == 1 present (shadow glass tint: needs the texture atlas)
    bool any_cutout = false;       // Cutout materials present (need the alpha atlas)
    std::vector<CutoutMat> cut;    // per material, when any_cutout
    std::vector<GlassMat> glass;   // per material, when any_atlas_shadow
    // incremental per-frame updates (tt_scene_update_*): what the last full validation established
    struct BlasKey {
        uint32_t root, node_offset, tri_offset;
        bool operator<(const BlasKey& o) const {
            return root != o.root ? root < o.root : node_offset != o.node_offset ? node_offset < o.node_offset
                                                                                  : tri_offset < o.tri_offset;
        }
        bool operator==(const BlasKey& o) const {
            return root == o.root && node_offset == o.node_offset && tri_offset == o.tri_offset;
        }
    };
    std::vector<BlasKey> blas_ok;       // sorted: (root, NodeOffset, TriOffset) triples walked and valid
    std::vector<uint8_t> is_tlas_node;  // node reached by the TLAS-level walk
    std::vector<uint32_t> tlas_nodes;   // the same, as a list
    std::vector<uint8_t> is_blas_node;  // node reached by a validated BLAS walk (never TLAS-only updated)
};

}  // namespace

struct tt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 0;
    int blocks_per_cu = 0;
    uint32_t grid = 0;
    uint32_t grid_of[18] = {};  // resident persistent grid per kernel instantiation (12..17: adaptive order)
    uint32_t shadow_grid_of[4] = {};  // the same for the any-hit kernel (stats * 2 + matcheck)
    TraceControl* ctl = nullptr;  // two control blocks: a trace launch uses one and zeroes the other
    uint32_t* sticky = nullptr;   // stack overflows of every launch since the last tt_async_overflows
    uint32_t ctl_cur = 0;          // the block the next launch uses
    bool ctl_zero[2] = {false, false};  // known zero when the next launch on the stream runs
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // last launch (aliases into the ring)
    hipEvent_t ring0[256] = {}, ring1[256] = {};
    uint32_t ring_n = 0, ring_base = 0;
    bool timing = true;  // tt_ctx_set_timing: asynchronous launches record their HIP-event pair
    uint32_t frame_pixels = 0;  // tt_ctx_set_frame_pixels: batched frames' bounce random numbers (0: off)
    bool lib_stream = false;    // stream is one of tt_stream_create's (tt_shutdown / the exit teardown may end it)
    std::string err;
    // scene
    bool has_scene = false;
    bool any_invisible = false;
    bool any_shadow_skip = false;  // some material is IsBackground / ShadowCaster
    bool any_atlas_shadow = false; // some material has specTrans == 1 (shadow tint needs the texture atlas)
    bool any_cutout = false;       // some material is Cutout (needs the alpha atlas)
    SceneHost host;
    DevBuf<tt_cwbvh_node> nodes;
    DevBuf<uint8_t> nodes_k;    // TT_NODE_STRIDE != 80: the kernels' strided copy of `nodes`
    DevBuf<tt_cuda_triangle> tris_raw;
    DevBuf<TriPos> tris;
    DevBuf<int32_t> tlas;
    DevBuf<tt_mesh_data> mesh_raw;
    DevBuf<MeshGpu> mesh;
    DevBuf<LeafMesh> leaf;
    DevBuf<uint32_t> mat_tag;
    DevBuf<CutoutMat> mat_cut;
    DevBuf<GlassMat> mat_glass;
    DevBuf<uint2> tex;          // _TextureAtlas, decoded RGBA half texels
    uint32_t tex_w = 0, tex_h = 0;
    DevBuf<uint8_t> atlas;      // _AlphaAtlas (R8)
    uint32_t atlas_w = 0, atlas_h = 0;
    // TT_ROOT_LEAF: node 0 as the device holds it is known on the host (upload, node updates); a device
    // refit of the TLAS rewrites it without a read-back, so the fast root step is off until the next update
    bool root_known = false;
    // TLAS refit (f4): plan valid for (scene generation, n_tlas_nodes)
    RefitDev refit;
    uint64_t scene_gen = 0, refit_gen = ~0ull;
    uint32_t refit_n_tlas = 0;
    DevBuf<float> st_boxes;
    // BLAS refit (f4, deforming / skinned meshes): one prepared plan + triangle boxes per mesh
    struct BlasRefit {
        RefitDev dev;
        uint32_t n_nodes = 0;  // nodes the plan covers, from the mesh's first node
        uint64_t gen = ~0ull;
        uint32_t node_base = ~0u;  // the mesh's NodeOffset the plan was built for
        DevBuf<float> boxes;
    };

    std::map<uint32_t, BlasRefit> blas_refit;
    DevBuf<float> st_vtx;
    DevBuf<int32_t> st_idx, st_leaf;
    // host-pointer staging
    uint64_t max_rays = 0;
    DevBuf<tt_ray_data> st_rays;
    DevBuf<uint32_t> st_info;
    DevBuf<tt_col_data> st_colors;
    DevBuf<float> st_normals;
    DevBuf<uint32_t> counter;   // bounce enqueue counters: two blocks of counter_words, used in turn
    uint32_t counter_words = 0, counter_cur = 0;
    DevBuf<uint2> spill;        // deep traversal-stack entries (tt_trace_spill_entries() per thread)
    uint32_t spill_threads = 0; // grid threads the spill area is sized for (max over all grids)
    DevBuf<tt_shadow_ray> st_shadow;
    DevBuf<float4> st_vis;
    DevBuf<float4> st_nee;
    DevBuf<tt_cache_data> st_cache;
    unsigned long long last_diag[8] = {};
    // pinned host staging for the asynchronous per-frame updates: two slots, each reused once the
    // copy enqueued from it has completed (its event)
    struct Pinned {
        void* p = nullptr;
        size_t n = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
    };
    Pinned pin[2];
    uint32_t pin_cur = 0;
    // TT_TRACE_ADAPTIVE_ORDER: per bounce index (min(bounce, 7)), the last flagged launch's per-tile
    // costs and the order buffer the next one dequeues in (tt_order.hip)
    struct OrderSlot {
        DevBuf<uint32_t> cost[2];  // cost[cur]: the last launch's costs (when valid)
        DevBuf<uint32_t> order;
        uint32_t cur = 0, w = 0, h = 0;
        uint32_t n_chunks = 0;     // chunks of the last flagged launch (tt_trace_chunk_costs)
        bool valid = false;
    };
    OrderSlot ord[8];
    // tt_ctx_share_scene: a borrower traces its lender's scene buffers (read-only) on its own stream
    tt_ctx* lender = nullptr;  // set on a borrower
    int borrowers = 0;         // on a lender: contexts currently tracing its scene
    // node array sizes: the scene's nodes, and the device array (+ TT_TLAS_SLOTS overlay regions of
    // tlas_res nodes each behind them, tt_ctx_share_blas)
    uint32_t n_nodes_scene = 0, n_nodes_dev = 0, tlas_res = 0;
    // tt_ctx_share_blas: a borrower with a TLAS of its own (a frame slot's TLAS refit and _MeshData rewrite
    // never wait for, or are seen by, the other slots): its TLAS nodes [0, n_tlas_own) live in overlay region
    // ovl_slot of the lender's node array, at kernel node index tlas_base; TLASBVH8Indices, _MeshData and the
    // derived MeshGpu / LeafMesh records are its own buffers. host.nodes then holds only those TLAS nodes.
    bool ovl = false;
    uint32_t ovl_slot = 0, tlas_base = 0, n_tlas_own = 0;
    uint32_t ovl_used = 0;     // lender: overlay regions in use (bit per slot)
    // Cross-stream order of a shared scene (the reference rewrites the TLAS and _MeshData every frame,
    // then dispatches, AssetManager.cs:1821-1825): a lender mutation waits for the borrowers' launches
    // already enqueued, and a borrower launch waits for the lender's mutations already enqueued. An
    // overlay borrower reads only the lender's BLAS part, so it orders only against BLAS-side mutations.
    // The lender's share state below (and its host node 0, which plain borrowers read for TT_ROOT_LEAF) is
    // guarded by `mu`, so a lender and its borrowers may be driven from different host threads; `mu` is held
    // across each read / write section (SceneRead / SceneWrite), so their enqueues are atomic against each
    // other. Recursive: a section's own calls (the root-leaf copy, the refit's bookkeeping) lock it again.
    std::recursive_mutex mu;
    std::vector<tt_ctx*> borrower_list;  // lender: the contexts tracing its scene
    hipEvent_t ev_scene = nullptr;       // lender: after its last scene mutation (recorded while borrowed)
    uint64_t scene_mut = 0;              // lender: mutations recorded in ev_scene so far
    hipEvent_t ev_blas = nullptr;        // lender: after its last BLAS-side mutation (overlay borrowers wait)
    uint64_t blas_mut = 0;               // lender: BLAS-side mutations recorded in ev_blas so far
    hipEvent_t ev_read = nullptr;        // borrower: recorded on its stream by a lender mutation (SceneWrite)
    uint64_t read_seq = 0;               // borrower: read sections enqueued so far
    uint64_t read_waited = 0;            // borrower: reads the lender's stream already waits for
    uint64_t mut_waited = 0;             // borrower: lender mutations this stream already waits for
};

// Scene-mutating calls are refused on a borrower (update the lender), and reallocating ones on a
// lender that has borrowers (their pointers would dangle). TT_REFUSE_BORROWER_TLAS lets an overlay
// borrower (tt_ctx_share_blas) mutate its own TLAS-side state.
#define TT_REFUSE_BORROWER(c)                                                                              \
    do {                                                                                                   \
        if ((c)->lender) return fail((c), TT_ERR_INVALID_ARG, "this context traces a shared scene: update the context it shares from"); \
    } while (0)
#define TT_REFUSE_BORROWER_TLAS(c)                                                                         \
    do {                                                                                                   \
        if ((c)->lender && !(c)->ovl) return fail((c), TT_ERR_INVALID_ARG, "this context traces a shared scene: update the context it shares from"); \
    } while (0)
#define TT_REFUSE_LENDER(c)                                                                                \
    do {                                                                                                   \
        if ((c)->borrowers > 0) return fail((c), TT_ERR_INVALID_ARG, "other contexts share this scene: destroy them (or re-share) first"); \
    } while (0)

// Per-call timing ring entries (tt_timing_read) around device work issued on the context stream.
// (with timing off -- tt_ctx_set_timing -- the calls that use these record nothing: they are all asynchronous
// or report no kernel time)
static hipError_t ring_open(tt_ctx* c, uint32_t& slot) {
    slot = c->ring_n % TT_RING;
    if (!c->timing) return hipSuccess;
    return hipEventRecord(c->ring0[slot], c->stream);
}
static hipError_t ring_close(tt_ctx* c, uint32_t slot) {
    if (!c->timing) return hipSuccess;
    const hipError_t e = hipEventRecord(c->ring1[slot], c->stream);
    c->ring_n++;
    c->ev0 = c->ring0[slot];
    c->ev1 = c->ring1[slot];
    return e;
}

// Shared-scene ordering (tt_ctx_share_scene / tt_ctx_share_blas). A borrower's enqueues that read the
// lender's scene buffers form a read section, a lender's scene mutation a write section; both hold the
// lender's mutex from first to last enqueue, so sections of the contexts sharing one scene are atomic
// against each other whichever host threads drive them. A read section makes the borrower's stream wait
// for the lender mutations enqueued before it (one wait per new mutation) and counts one read. A write
// section makes the lender's stream wait for every borrower stream with reads counted since the last such
// wait, by recording an event on that stream right then -- one record per borrower per mutation and
// nothing per launch (round 5 recorded one after every borrower launch: with the launch-timing pair, the
// per-launch markers cost 15-20% of a strong-scaled rank's frame, profiles/r05/events/) -- and, at its end,
// records the mutation for later readers. An overlay borrower (tt_ctx_share_blas) reads only the lender's
// BLAS part, so it orders only against BLAS-side mutations.
static hipError_t lazy_event(hipEvent_t& ev) {
    return ev ? hipSuccess : hipEventCreateWithFlags(&ev, hipEventDisableTiming);
}
// TT_NO_SCENE_ORDER: a diagnostic variant build only (make variant NAME=noorder VFLAGS=-DTT_NO_SCENE_ORDER): the
// sections take the lock but order nothing, to show the ordering tests fail without them.
#ifndef TT_NO_SCENE_ORDER
#define TT_NO_SCENE_ORDER 0
#endif
class SceneRead {
  public:
    explicit SceneRead(tt_ctx* c) : L_(c->lender) {
        if (!L_) return;
        if (TT_NO_SCENE_ORDER) {
            L_->mu.lock();
            return;
        }
        L_->mu.lock();
        const uint64_t seq = c->ovl ? L_->blas_mut : L_->scene_mut;
        if (seq != c->mut_waited) {
            err = hipStreamWaitEvent(c->stream, c->ovl ? L_->ev_blas : L_->ev_scene, 0);
            if (err == hipSuccess) c->mut_waited = seq;
        }
        c->read_seq++;
    }
    SceneRead(const SceneRead&) = delete;
    SceneRead& operator=(const SceneRead&) = delete;
    ~SceneRead() { end(); }
    void end() {
        if (L_) L_->mu.unlock();
        L_ = nullptr;
    }
    hipError_t err = hipSuccess;

  private:
    tt_ctx* L_;
};
// blas: the mutation touches what overlay borrowers read too (BLAS nodes, triangles); otherwise only the
// lender's TLAS-side state (TLAS nodes, _MeshData), which only plain borrowers read. active = false: no
// section (an overlay borrower's own TLAS-side state is read by nobody else).
class SceneWrite {
  public:
    SceneWrite(tt_ctx* c, bool blas, bool active = true) : c_(active ? c : nullptr), blas_(blas) {
        if (!c_) return;
        c_->mu.lock();
        if (TT_NO_SCENE_ORDER) return;
        for (tt_ctx* b : c_->borrower_list) {
            if (b->read_seq == b->read_waited || (b->ovl && !blas_)) continue;
            if ((err = lazy_event(b->ev_read)) != hipSuccess || (err = hipEventRecord(b->ev_read, b->stream)) != hipSuccess ||
                (err = hipStreamWaitEvent(c_->stream, b->ev_read, 0)) != hipSuccess)
                return;
            b->read_waited = b->read_seq;
        }
    }
    SceneWrite(const SceneWrite&) = delete;
    SceneWrite& operator=(const SceneWrite&) = delete;
    ~SceneWrite() {
        if (c_) c_->mu.unlock();
    }
    // after the mutation is enqueued: records it for the borrowers (a later borrower syncs the stream when
    // it shares, so nothing is recorded without one) and leaves the section
    hipError_t end() {
        if (!c_) return hipSuccess;
        hipError_t e = hipSuccess;
        if (!c_->borrower_list.empty() && !TT_NO_SCENE_ORDER) {
            e = lazy_event(c_->ev_scene);
            if (e == hipSuccess) e = hipEventRecord(c_->ev_scene, c_->stream);
            if (e == hipSuccess) c_->scene_mut++;
            if (e == hipSuccess && blas_) {
                e = lazy_event(c_->ev_blas);
                if (e == hipSuccess) e = hipEventRecord(c_->ev_blas, c_->stream);
                if (e == hipSuccess) c_->blas_mut++;
            }
        }
        c_->mu.unlock();
        c_ = nullptr;
        return e;
    }
    hipError_t err = hipSuccess;

  private:
    tt_ctx* c_;
    bool blas_;
};
// The node array the kernels read: the reference's (80-B stride) or its strided copy, refreshed on the
// context stream after every write to `nodes` (device node indices [first, first + count): a frame slot's
// TLAS sits at tlas_base).
static const uint4* kernel_nodes(const tt_ctx* c) {
    return TT_NODE_STRIDE == 80 ? reinterpret_cast<const uint4*>(c->nodes.p) : reinterpret_cast<const uint4*>(c->nodes_k.p);
}
static hipError_t refresh_node_copy(tt_ctx* c, uint32_t first, uint32_t count) {
    if (TT_NODE_STRIDE == 80 || count == 0) return hipSuccess;
    return hipMemcpy2DAsync(c->nodes_k.p + (size_t)first * TT_NODE_STRIDE, TT_NODE_STRIDE, c->nodes.p + first,
                            sizeof(tt_cwbvh_node), sizeof(tt_cwbvh_node), count, hipMemcpyDeviceToDevice, c->stream);
}
static void unlink_borrower(tt_ctx* b) {
    tt_ctx* L = b->lender;
    if (!L) return;
    std::lock_guard<std::recursive_mutex> lk(L->mu);
    L->borrowers--;
    L->borrower_list.erase(std::remove(L->borrower_list.begin(), L->borrower_list.end(), b), L->borrower_list.end());
    if (b->ovl) L->ovl_used &= ~(1u << b->ovl_slot);
    b->lender = nullptr;
    b->ovl = false;
    b->tlas_base = 0;
}

namespace {

tt_status fail(tt_ctx* c, tt_status s, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return s;
}

tt_status hip_fail(tt_ctx* c, hipError_t e, const char* what) {
    return fail(c, e == hipErrorOutOfMemory ? TT_ERR_OOM : TT_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define TT_HIP(c, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(c, e_, #call); \
    } while (0)

// Structural validation of everything the trace kernel can reach (IntersectBVH's index
// arithmetic, IntersectionKernels.compute:157-213): every reachable node, triangle, TLAS slot
// and mesh record must be in range, so the GPU kernel needs no per-access bounds checks.
struct Validator {
    const SceneHost& s;
    // the nodes a walk reads: TLAS-level walks tl[0, n_tl), BLAS-level walks bl[0, n_bl). A context's own
    // scene: both are its host.nodes. An overlay borrower (tt_ctx_share_blas): its TLAS copy, and the lender's
    // nodes and material words, exactly as its kernels address them (TLAS at tlas_base, BLASes shared).
    const tt_cwbvh_node* tl;
    uint32_t n_tl;
    const tt_cwbvh_node* bl;
    uint32_t n_bl;
    const std::vector<uint32_t>* matdat;
    std::vector<uint32_t> epoch_of;
    uint32_t epoch = 0;
    std::string why;
    explicit Validator(const SceneHost& h)
        : s(h), tl(h.nodes.data()), n_tl((uint32_t)h.nodes.size()), bl(h.nodes.data()), n_bl((uint32_t)h.nodes.size()),
          matdat(&h.matdat), epoch_of(h.nodes.size(), 0u) {}
    Validator(const SceneHost& own, const SceneHost& blas)
        : s(own), tl(own.nodes.data()), n_tl((uint32_t)own.nodes.size()), bl(blas.nodes.data()),
          n_bl((uint32_t)blas.nodes.size()), matdat(&blas.matdat),
          epoch_of(std::max(own.nodes.size(), blas.nodes.size()), 0u) {}

    uint32_t max_matdat = 0;
    std::vector<uint32_t> tlas_visit;  // nodes reached by the last TLAS-level walk
    std::vector<uint32_t> blas_visit;  // nodes reached by the BLAS-level walks of this validator
    std::vector<SceneHost::BlasKey> keys;  // BLAS (root, NodeOffset, TriOffset) walked by run()
    bool walk(uint32_t root, uint32_t node_offset, uint32_t tri_offset, bool tlas_level) {
        epoch++;
        max_matdat = 0;
        if (tlas_level) tlas_visit.clear();
        std::vector<uint32_t> work{root};
        while (!work.empty()) {
            const uint32_t ni = work.back();
            work.pop_back();
            if (ni >= (tlas_level ? n_tl : n_bl)) {
                why = "node index " + std::to_string(ni) + " out of range" +
                      (tlas_level && tl != bl ? " of the context's own TLAS nodes" : "");
                return false;
            }
            if (epoch_of[ni] == epoch) continue;
            epoch_of[ni] = epoch;
            if (tlas_level) tlas_visit.push_back(ni);
            else blas_visit.push_back(ni);
            const tt_cwbvh_node& n = tlas_level ? tl[ni] : bl[ni];
            const uint32_t imask = n.e_imask >> 24;
            for (int k = 0; k < 8; k++) {
                const uint32_t meta = (n.meta[k >> 2] >> ((k & 3) * 8)) & 0xffu;
                const uint32_t low5 = meta & 0x1fu, bits = (meta >> 5) & 7u;
                const bool inner = (meta & 0x18u) == 0x18u;
                if (inner) {
                    if (bits != 1u) {
                        why = "inner meta with child bits != 1";
                        return false;
                    }
                    const uint32_t slot = low5 - 24u;
                    const uint32_t child = n.base_child + node_offset + (uint32_t)__builtin_popcount(imask & ((1u << slot) - 1u));
                    work.push_back(child);
                } else if (bits) {
                    const uint32_t top = low5 + (31u - (uint32_t)__builtin_clz(bits));
                    if (top >= 24u) {
                        why = "leaf meta spills into the internal-child bits";
                        return false;
                    }
                    for (uint32_t b = 0; b < 3; b++) {
                        if (!((bits >> b) & 1u)) continue;
                        const uint64_t t = (uint64_t)n.base_tri + tri_offset + low5 + b;
                        if (tlas_level) {
                            if (t >= s.tlas.size()) {
                                why = "TLAS leaf slot out of range";
                                return false;
                            }
                            const int32_t m = s.tlas[t];
                            if (m < 0 || (size_t)m >= s.mesh.size()) {
                                why = "TLASBVH8Indices entry out of range";
                                return false;
                            }
                        } else if (t >= s.n_tris) {
                            why = "triangle index out of range";
                            return false;
                        } else if (!matdat->empty()) {
                            max_matdat = std::max(max_matdat, (*matdat)[(size_t)t]);
                        }
                    }
                }
            }
        }
        return true;
    }

    // one mesh record's BLAS (IntersectionKernels.compute:197-213 reach it through the TLAS)
    bool walk_mesh(const tt_mesh_data& md) {
        if (md.NodeOffset < 0 || md.TriOffset < 0) {
            why = "negative mesh offsets";
            return false;
        }
        return walk((uint32_t)(md.mesh_data_bvh_offsets & 0x7fffffff), (uint32_t)md.NodeOffset,
                    (uint32_t)md.TriOffset, false);
    }

    bool run() {
        if (n_tl == 0 || n_bl == 0 || s.mesh.empty()) {
            why = "empty scene";
            return false;
        }
        if (!walk(0, 0, 0, true)) return false;
        // every mesh record reachable through the TLAS (validate them all: cheap, and update
        // paths may re-point TLAS leaves)
        struct Seen {
            uint64_t key;
            uint32_t root, max_matdat;
        };
        std::vector<Seen> seen;
        for (size_t m = 0; m < s.mesh.size(); m++) {
            const tt_mesh_data& md = s.mesh[m];
            const uint32_t root = (uint32_t)(md.mesh_data_bvh_offsets & 0x7fffffff);
            if (md.NodeOffset < 0 || md.TriOffset < 0) {
                why = "negative mesh offsets";
                return false;
            }
            const uint64_t key = ((uint64_t)(uint32_t)md.NodeOffset << 32) | (uint32_t)md.TriOffset;
            uint32_t mm = 0;
            bool dup = false;
            for (auto& p : seen)
                if (p.key == key && p.root == root) {
                    dup = true;
                    mm = p.max_matdat;
                }
            if (!dup) {
                if (!walk(root, (uint32_t)md.NodeOffset, (uint32_t)md.TriOffset, false)) return false;
                mm = max_matdat;
                seen.push_back(Seen{key, root, mm});
                keys.push_back(SceneHost::BlasKey{root, (uint32_t)md.NodeOffset, (uint32_t)md.TriOffset});
            }

        }
        std::sort(keys.begin(), keys.end());
        return true;
    }
};

// Records what a full validation established, for the incremental per-frame update paths.
void remember_validation(SceneHost& h, const Validator& v) {
    h.blas_ok = v.keys;
    h.is_tlas_node.assign(h.nodes.size(), 0u);
    h.tlas_nodes = v.tlas_visit;
    for (uint32_t n : h.tlas_nodes) h.is_tlas_node[n] = 1u;
    h.is_blas_node.assign(h.nodes.size(), 0u);
    for (uint32_t n : v.blas_visit) h.is_blas_node[n] = 1u;
}

tt_status check_scene(const tt_cwbvh_node* nodes, uint32_t n_nodes, const tt_cuda_triangle* tris, uint32_t n_tris,
                      const int32_t* tlas, uint32_t n_tlas, const tt_mesh_data* md, uint32_t n_mesh,
                      const tt_material* mats, uint32_t n_mat, SceneHost& h, std::vector<uint32_t>& tags,
                      bool& any_invisible, std::string& why) {
    if (!nodes || !n_nodes || !tris || !n_tris || !tlas || !n_tlas || !md || !n_mesh || (n_mat && !mats)) {
        why = "null or empty buffer";
        return TT_ERR_INVALID_ARG;
    }
    if ((uint64_t)n_nodes * std::max<uint64_t>(sizeof(tt_cwbvh_node), TT_NODE_STRIDE) >= (1ull << 32) ||
        (uint64_t)n_tris * 48u >= (1ull << 32)) {
        why = "node or triangle array of 4 GiB or more (the trace kernel addresses them with 32-bit offsets)";
        return TT_ERR_INVALID_ARG;
    }
    h.nodes.assign(nodes, nodes + n_nodes);
    h.tlas.assign(tlas, tlas + n_tlas);
    h.mesh.assign(md, md + n_mesh);
    h.n_tris = n_tris;
    h.n_mat = n_mat;
    any_invisible = false;
    tags.assign(std::max<uint32_t>(n_mat, 1u), 0u);
    for (uint32_t m = 0; m < n_mat; m++) {
        tags[m] = mats[m].Tag & ~((1u << TT_MATWORD_CUTOUT) | (1u << TT_MATWORD_GLASS));
        if (mats[m].specTrans == 1.0f) tags[m] |= 1u << TT_MATWORD_GLASS;  // stained-glass shadow tint
        if (mats[m].MatType == TT_MAT_CUTOUT_INDEX) {  // alpha test, IntersectionKernels.compute:35-40
            tags[m] |= 1u << TT_MATWORD_CUTOUT;
            h.any_cutout = true;
        }
        any_invisible |= ((mats[m].Tag >> TT_FLAG_INVISIBLE) & 1u) != 0;
        h.any_shadow_skip |= (((mats[m].Tag >> TT_FLAG_IS_BACKGROUND) | (mats[m].Tag >> TT_FLAG_SHADOW_CASTER)) & 1u) != 0;
        h.any_atlas_shadow |= mats[m].specTrans == 1.0f;
    }
    if (h.any_cutout) {
        h.cut.assign(n_mat, CutoutMat{});
        for (uint32_t m = 0; m < n_mat; m++) {
            CutoutMat& r = h.cut[m];
            r.alpha_tex[0] = mats[m].AlphaTex[0];
            r.alpha_tex[1] = mats[m].AlphaTex[1];
            r.cutoff = mats[m].AlphaCutoff;
            for (int k = 0; k < 4; k++) r.scale[k] = mats[m].AlbedoTexScale[k];
        }
    }
    if (h.any_atlas_shadow) {
        h.glass.assign(n_mat, GlassMat{});
        for (uint32_t m = 0; m < n_mat; m++) {
            GlassMat& r = h.glass[m];
            r.albedo_tex[0] = mats[m].AlbedoTex[0];
            r.albedo_tex[1] = mats[m].AlbedoTex[1];
            for (int k = 0; k < 3; k++) r.color[k] = mats[m].surfaceColor[k];
            for (int k = 0; k < 4; k++) r.scale[k] = mats[m].AlbedoTexScale[k];
        }
    }
    if (any_invisible) {
        h.matdat.resize(n_tris);
        for (uint32_t t = 0; t < n_tris; t++) h.matdat[t] = tris[t].MatDat;
    }
    Validator v(h);
    if (!v.run()) {
        why = v.why;
        return TT_ERR_INVALID_ARG;
    }
    remember_validation(h, v);
    return TT_OK;
}

__host__ __device__ inline void derive_mesh(const tt_mesh_data& in, MeshGpu& o) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) o.m[r * 4 + c] = in.W2L[c * 4 + r];
    o.TriOffset = in.TriOffset;
    o.NodeOffset = in.NodeOffset;
    o.MaterialOffset = in.MaterialOffset;
    o.root = in.mesh_data_bvh_offsets & 0x7fffffff;
}

// LeafMesh[i] = the mesh record TLASBVH8Indices[i] names (indices were validated at upload)
std::vector<LeafMesh> derive_leaves(const std::vector<int32_t>& tlas, const std::vector<tt_mesh_data>& md) {
    std::vector<LeafMesh> out(std::max<size_t>(1, tlas.size()));
    for (size_t i = 0; i < tlas.size(); i++) {
        LeafMesh& l = out[i];
        std::memset(&l, 0, sizeof(l));
        const int32_t m = tlas[i];
        if (m >= 0 && (size_t)m < md.size()) derive_mesh(md[(size_t)m], l.m);
        l.mesh_id = m;
    }
    return out;
}

void derive_tri(const tt_cuda_triangle& t, TriPos& o) {
    o.p0x = t.pos0[0];
    o.p0y = t.pos0[1];
    o.p0z = t.pos0[2];
    o.e1x = t.posedge1[0];
    o.e1y = t.posedge1[1];
    o.e1z = t.posedge1[2];
    o.e2x = t.posedge2[0];
    o.e2y = t.posedge2[1];
    o.e2z = t.posedge2[2];
    o.matdat = t.MatDat;
    o.pad0 = o.pad1 = 0;
}

// The traversal records of updated _MeshData entries [first, first + count) (derive_mesh), and
// every TLAS leaf record whose TLASBVH8Indices entry names one of them (derive_leaves).
// src: records [first, first + count), read in place from the pinned staging buffer (host memory the
// GPU reads over the bus: no copy operation on the stream), also stored to _MeshData (raw).
__global__ void tt_update_mesh_kernel(const tt_mesh_data* __restrict__ src, tt_mesh_data* __restrict__ raw,
                                      MeshGpu* __restrict__ mesh, LeafMesh* __restrict__ leaf,
                                      const int32_t* __restrict__ tlas, uint32_t n_tlas, uint32_t first, uint32_t count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const tt_mesh_data r = src[i];
        raw[first + i] = r;
        MeshGpu g;
        derive_mesh(r, g);
        mesh[first + i] = g;
    }
    if (i < n_tlas) {
        const int32_t m = tlas[i];
        if (m >= 0 && (uint32_t)m - first < count) {
            LeafMesh l;
            derive_mesh(src[(uint32_t)m - first], l.m);
            l.mesh_id = m;
            l.pad[0] = l.pad[1] = l.pad[2] = 0;
            leaf[i] = l;
        }
    }
}

bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

}  // namespace

extern "C" {

int32_t tt_abi_version(void) { return TT_ABI_VERSION; }

int32_t tt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

const char* tt_last_error(const tt_ctx* c) { return c ? c->err.c_str() : "null context"; }

}  // extern "C"

// Streams made by tt_stream_create that the caller has not destroyed yet. A queue created with a CU mask
// that is still alive when the HIP runtime's own static destructors run takes the process down in
// __cxa_finalize (SIGSEGV, gpurun_out/qmap.out under rocprofv3), so the library destroys what is left
// from an exit handler. It is registered after the first stream is made -- after the HIP runtime has
// initialised and registered its own destructors -- and exit handlers run in reverse order of
// registration, so it runs before the runtime tears down. A host that destroys its streams (or a
// Unity domain reload that misses StreamDestroy) is covered either way.
namespace {
std::mutex g_streams_mu;
std::vector<std::pair<int, hipStream_t>> g_streams;
// streams the teardown (tt_shutdown, the exit handlers) destroyed under a context still holding them: such a
// context refuses launches and skips the stream sync in tt_ctx_destroy (a host's static destructors may
// destroy contexts after the teardown ran)
std::vector<hipStream_t> g_dead;
std::atomic<uint32_t> g_dead_n{0};
bool g_streams_handler = false;

void release_live_streams() {
    std::vector<std::pair<int, hipStream_t>> live;
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        live.swap(g_streams);
        for (auto& ds : live) g_dead.push_back(ds.second);
        g_dead_n.store((uint32_t)g_dead.size());
    }
    for (auto& ds : live) {
        if (hipSetDevice(ds.first) != hipSuccess) continue;
        (void)hipStreamSynchronize(ds.second);
        (void)hipStreamDestroy(ds.second);
    }
    (void)hipGetLastError();
}

// The atexit form. exit() has already destroyed the exiting thread's thread_locals when atexit handlers
// run, and a profiler that wraps the HIP API (rocprofv3) keeps per-thread state its stream calls need
// ("'get_stream_stack()' Must be non nullptr", profiles/r05/lifecycle/atexit_only_abort_under_rocprofv3.txt):
// so the teardown runs on a fresh thread, whose thread state is created on its first HIP call.
void release_live_streams_at_exit() {
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        if (g_streams.empty()) return;
    }
    std::thread t(release_live_streams);
    t.join();
}

bool stream_dead(hipStream_t s) {
    if (g_dead_n.load(std::memory_order_relaxed) == 0) return false;
    std::lock_guard<std::mutex> lk(g_streams_mu);
    return std::find(g_dead.begin(), g_dead.end(), s) != g_dead.end();
}
bool is_lib_stream(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_streams_mu);
    return std::any_of(g_streams.begin(), g_streams.end(), [s](const std::pair<int, hipStream_t>& ds) { return ds.second == s; });
}
}  // namespace

// a context whose library stream the teardown destroyed refuses every launch
#define TT_REFUSE_DEAD_STREAM(c)                                                                            \
    do {                                                                                                    \
        if ((c)->lib_stream && stream_dead((c)->stream))                                                    \
            return fail((c), TT_ERR_INVALID_ARG, "the context's stream was destroyed by tt_shutdown / the exit teardown"); \
    } while (0)

extern "C" {

}  // extern "C"

namespace {
// A profiler that wraps the HIP API (rocprofv3's tool) keeps per-thread state that its stream calls need
// ("'get_stream_stack()' Must be non nullptr"), and exit() destroys a thread's thread_local objects BEFORE it
// runs any atexit handler: from the atexit handler alone, the hipStreamDestroy calls abort under the tool.
// So the teardown is armed a second way: a thread_local guard, constructed on the first launch on one of the
// library's streams (after the tool's own per-thread state exists, so destroyed before it: glibc runs a
// thread's TLS destructors in reverse order of construction), whose destructor tears the streams down when
// the MAIN thread's thread_locals are destroyed -- i.e. from exit() -- and does nothing when another thread
// ends (the process goes on). The atexit handler stays for a process whose launches all came from other
// threads; a second run finds the list empty.
bool stream_exit_handler_on() {
    static const bool on = [] {  // TT_STREAM_EXIT_HANDLER=0: diagnosis only (the exit-time teardown off)
        const char* e = std::getenv("TT_STREAM_EXIT_HANDLER");
        return !(e && e[0] == '0');
    }();
    return on;
}
struct MainThreadExitGuard {
    ~MainThreadExitGuard() {
        if ((pid_t)syscall(SYS_gettid) == getpid()) release_live_streams();
    }
};
void note_stream_launch(hipStream_t s) {
    thread_local bool armed = false;
    if (armed || !stream_exit_handler_on()) return;
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        if (std::none_of(g_streams.begin(), g_streams.end(), [s](const std::pair<int, hipStream_t>& ds) { return ds.second == s; }))
            return;
    }
    armed = true;
    thread_local MainThreadExitGuard guard;
    (void)&guard;
}
}  // namespace

extern "C" {

tt_status tt_shutdown(void) {
    release_live_streams();
    return TT_OK;
}

uint32_t tt_stream_live_count(void) {
    std::lock_guard<std::mutex> lk(g_streams_mu);
    return (uint32_t)g_streams.size();
}

tt_status tt_stream_create(int32_t device, void** stream) {
    if (!stream) return TT_ERR_INVALID_ARG;
    *stream = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return TT_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) return TT_ERR_INVALID_ARG;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return TT_ERR_HIP;
    hipDeviceProp_t prop;
    hipStream_t s = nullptr;
    tt_status st = TT_OK;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        st = TT_ERR_HIP;
    } else {
        // every CU enabled: the mask only exists to get a HW queue that no other stream shares
        std::vector<uint32_t> mask(((uint32_t)prop.multiProcessorCount + 31u) / 32u, 0xffffffffu);
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            st = TT_ERR_HIP;
        }
    }
    (void)hipSetDevice(prev);  // the caller's current device is left as it was
    if (st == TT_OK) {
        *stream = s;
        std::lock_guard<std::mutex> lk(g_streams_mu);
        g_streams.emplace_back(device, s);
        // (a new stream may reuse a destroyed one's handle)
        g_dead.erase(std::remove(g_dead.begin(), g_dead.end(), s), g_dead.end());
        g_dead_n.store((uint32_t)g_dead.size());
        if (!g_streams_handler && stream_exit_handler_on())
            g_streams_handler = std::atexit(release_live_streams_at_exit) == 0;
    }
    return st;
}

tt_status tt_stream_destroy(void* stream) {
    if (!stream) return TT_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        auto it = std::find_if(g_streams.begin(), g_streams.end(),
                               [s](const std::pair<int, hipStream_t>& ds) { return ds.second == s; });
        if (it == g_streams.end()) return TT_ERR_INVALID_ARG;  // not ours, or destroyed already
        g_streams.erase(it);
    }
    const hipError_t a = hipStreamSynchronize(s);
    const hipError_t b = hipStreamDestroy(s);
    return (a == hipSuccess && b == hipSuccess) ? TT_OK : TT_ERR_HIP;
}

tt_status tt_ctx_create(const tt_config* cfg, tt_ctx** out) {
    if (!cfg || !out) return TT_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return TT_ERR_NO_DEVICE;
    }
    if (cfg->device < 0 || cfg->device >= ndev) return TT_ERR_INVALID_ARG;
    tt_ctx* c = new tt_ctx();
    c->device = cfg->device;
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) {
        delete c;
        return TT_ERR_HIP;
    }
    if (cfg->stream) {
        c->stream = static_cast<hipStream_t>(cfg->stream);
        c->lib_stream = is_lib_stream(c->stream);
    } else {
        // blocking (default-flag) stream: ordered with the legacy NULL stream, so callers that
        // fill device buffers on it (torch's default stream) cannot race the engine
        if (hipStreamCreate(&c->stream) != hipSuccess) {
            delete c;
            return TT_ERR_HIP;
        }
        c->own_stream = true;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
        tt_ctx_destroy(c);
        return TT_ERR_HIP;
    }
    c->num_cus = prop.multiProcessorCount;
    int occ[18];
    (void)tt_trace_occupancy_table(occ);
    // Residency check beyond the occupancy API: measured on MI355X, five 32-KiB-LDS blocks were
    // not co-resident (the fifth started only when another exited), consistent with the LDS being
    // allocated per half-CU (2 x 80 KiB). Size every persistent grid so all its blocks are resident.
    const uint32_t lds_block = tt_trace_lds_bytes();
    const int lds_cap = lds_block ? 2 * (int)((80u * 1024u) / lds_block) : 8;
    int knob = 0;
    if (const char* e = std::getenv("TT_BLOCKS_PER_CU")) knob = std::atoi(e);  // tuning/diagnostic knob
    // at most 32 waves per CU (8 blocks of 4 waves at the default 256-thread block)
    const int wpb = (int)std::max(1u, tt_trace_block_size() / 64u);
    const int block_cap = std::max(1, 32 / wpb);
    for (int k = 0; k < 18; k++) {
        int b = std::max(1, std::min(std::min(occ[k], lds_cap), block_cap));
        if (knob > 0 && knob < b) b = knob;
        c->grid_of[k] = (uint32_t)(c->num_cus * b);
    }
    int socc[4];
    tt_shadow_occupancy_table(socc);
    for (int k = 0; k < 4; k++) {
        int b = std::max(1, std::min(std::min(socc[k], lds_cap), block_cap));
        if (knob > 0 && knob < b) b = knob;
        c->shadow_grid_of[k] = (uint32_t)(c->num_cus * b);
    }
    c->blocks_per_cu = (int)(c->grid_of[1] / c->num_cus);
    c->grid = c->grid_of[1];
    uint32_t max_grid = 0;
    for (int k = 0; k < 18; k++) max_grid = std::max(max_grid, c->grid_of[k]);
    for (int k = 0; k < 4; k++) max_grid = std::max(max_grid, c->shadow_grid_of[k]);
    c->spill_threads = max_grid * tt_trace_block_size();
    // two control blocks + the sticky overflow counter behind them
    if (hipMalloc(reinterpret_cast<void**>(&c->ctl), 2 * sizeof(TraceControl) + 256) != hipSuccess) {
        tt_ctx_destroy(c);
        return TT_ERR_OOM;
    }
    c->sticky = reinterpret_cast<uint32_t*>(c->ctl + 2);
    if (hipMemset(c->ctl, 0, 2 * sizeof(TraceControl) + 256) != hipSuccess) {
        tt_ctx_destroy(c);
        return TT_ERR_HIP;
    }
    for (uint32_t i = 0; i < TT_RING; i++) {
        if (hipEventCreate(&c->ring0[i]) != hipSuccess || hipEventCreate(&c->ring1[i]) != hipSuccess) {
            tt_ctx_destroy(c);
            return TT_ERR_HIP;
        }
    }
    if (const uint32_t se = tt_trace_spill_entries()) {
        if (c->spill.alloc((size_t)se * c->spill_threads) != hipSuccess) {
            tt_ctx_destroy(c);
            return TT_ERR_OOM;
        }
    }
    c->max_rays = cfg->max_rays;
    if (c->max_rays) {
        if (c->st_rays.alloc(c->max_rays) != hipSuccess) {
            tt_ctx_destroy(c);
            return TT_ERR_OOM;
        }
    }
    *out = c;
    return TT_OK;
}

tt_status tt_ctx_destroy(tt_ctx* c) {
    if (!c) return TT_ERR_INVALID_ARG;
    if (c->borrowers > 0) return fail(c, TT_ERR_INVALID_ARG, "other contexts share this scene: destroy them first");
    (void)hipSetDevice(c->device);
    if (c->stream && !(c->lib_stream && stream_dead(c->stream))) (void)hipStreamSynchronize(c->stream);
    unlink_borrower(c);
    if (c->ev_scene) (void)hipEventDestroy(c->ev_scene);
    if (c->ev_blas) (void)hipEventDestroy(c->ev_blas);
    if (c->ev_read) (void)hipEventDestroy(c->ev_read);
    c->nodes.release();
    c->nodes_k.release();
    c->tris_raw.release();
    c->tris.release();
    c->tlas.release();
    c->mesh_raw.release();
    c->mesh.release();
    c->mat_tag.release();
    c->mat_cut.release();
    c->mat_glass.release();
    c->leaf.release();
    c->atlas.release();
    c->tex.release();
    tt_refit_free(c->refit);
    for (auto& kv : c->blas_refit) {
        tt_refit_free(kv.second.dev);
        kv.second.boxes.release();
    }
    c->st_vtx.release();
    c->st_idx.release();
    c->st_leaf.release();
    c->st_boxes.release();
    c->st_rays.release();
    c->st_shadow.release();
    c->st_vis.release();
    c->st_nee.release();
    c->st_cache.release();
    c->st_info.release();
    c->st_colors.release();
    c->st_normals.release();
    c->counter.release();
    c->spill.release();
    for (auto& os : c->ord) {  // TT_TRACE_ADAPTIVE_ORDER state
        os.cost[0].release();
        os.cost[1].release();
        os.order.release();
    }
    if (c->ctl) (void)hipFree(c->ctl);
    for (uint32_t i = 0; i < TT_RING; i++) {
        if (c->ring0[i]) (void)hipEventDestroy(c->ring0[i]);
        if (c->ring1[i]) (void)hipEventDestroy(c->ring1[i]);
    }
    for (auto& pn : c->pin) {
        if (pn.p) (void)hipHostFree(pn.p);
        if (pn.ev) (void)hipEventDestroy(pn.ev);
    }
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return TT_OK;
}

tt_status tt_ctx_set_timing(tt_ctx* c, int32_t enabled) {
    if (!c) return TT_ERR_INVALID_ARG;
    c->timing = enabled != 0;
    return TT_OK;
}

tt_status tt_ctx_set_frame_pixels(tt_ctx* c, uint32_t frame_pixels) {
    if (!c) return TT_ERR_INVALID_ARG;
    if (frame_pixels > 0x7fffffffu) return fail(c, TT_ERR_INVALID_ARG, "frame_pixels above 2^31 - 1");
    c->frame_pixels = frame_pixels;
    return TT_OK;
}

tt_status tt_timing_reset(tt_ctx* c) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_HIP(c, hipStreamSynchronize(c->stream));
    c->ring_base = c->ring_n;
    return TT_OK;
}

tt_status tt_timing_read(tt_ctx* c, float* ms, uint32_t max, uint32_t* n) {
    if (!c || !n || (max && !ms)) return TT_ERR_INVALID_ARG;
    TT_HIP(c, hipStreamSynchronize(c->stream));
    const uint32_t total = c->ring_n - c->ring_base;
    const uint32_t avail = std::min(total, TT_RING);
    const uint32_t k = std::min(avail, max);
    for (uint32_t i = 0; i < k; i++) {
        const uint32_t slot = (c->ring_n - avail + i) % TT_RING;
        TT_HIP(c, hipEventElapsedTime(&ms[i], c->ring0[slot], c->ring1[slot]));
    }
    *n = k;
    return TT_OK;
}

tt_status tt_trace_diagnostics(const tt_ctx* c, uint64_t* out8) {
    if (!c || !out8) return TT_ERR_INVALID_ARG;
    for (int k = 0; k < 8; k++) out8[k] = c->last_diag[k];
    return TT_OK;
}

tt_status tt_selftest_rcp(tt_ctx* c, uint64_t* mismatches) {
    if (!c || !mismatches) return TT_ERR_INVALID_ARG;
    TT_HIP(c, hipSetDevice(c->device));
    DevBuf<unsigned long long> bad;
    struct Release {
        DevBuf<unsigned long long>& b;
        ~Release() { b.release(); }
    } release{bad};
    TT_HIP(c, bad.alloc(1));
    TT_HIP(c, hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), c->stream));
    TT_HIP(c, tt_launch_rcp_selftest(bad.p, c->stream));
    unsigned long long h = 0;
    TT_HIP(c, hipMemcpyAsync(&h, bad.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
    TT_HIP(c, hipStreamSynchronize(c->stream));
    *mismatches = (uint64_t)h;
    return TT_OK;
}

void* tt_ctx_stream(tt_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

tt_status tt_async_overflows(tt_ctx* c, uint64_t* count) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_HIP(c, hipStreamSynchronize(c->stream));
    uint32_t n = 0;
    TT_HIP(c, hipMemcpy(&n, c->sticky, sizeof(n), hipMemcpyDeviceToHost));
    TT_HIP(c, hipMemset(c->sticky, 0, sizeof(n)));
    if (count) *count = n;
    if (n) return fail(c, TT_ERR_STACK_OVERFLOW, "%u rays needed more than %d traversal stack entries", n, TT_STACK_SIZE);
    return TT_OK;
}

tt_status tt_sync(tt_ctx* c) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

namespace {
tt_status refresh_leaves(tt_ctx* c);
}

tt_status tt_scene_upload(tt_ctx* c, const tt_cwbvh_node* nodes, uint32_t n_nodes, const tt_cuda_triangle* tris,
                          uint32_t n_tris, const int32_t* tlas, uint32_t n_tlas, const tt_mesh_data* md,
                          uint32_t n_mesh, const tt_material* mats, uint32_t n_mat) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_REFUSE_BORROWER(c);
    TT_REFUSE_LENDER(c);
    if (!nodes || !n_nodes || !tris || !n_tris || !tlas || !n_tlas || !md || !n_mesh || (n_mat && !mats))
        return fail(c, TT_ERR_INVALID_ARG, "tt_scene_upload: null or empty buffer");
    TT_HIP(c, hipSetDevice(c->device));
    c->has_scene = false;
    SceneHost h;
    std::vector<uint32_t> tags;
    bool any_invisible = false;
    std::string why;
    const tt_status vs = check_scene(nodes, n_nodes, tris, n_tris, tlas, n_tlas, md, n_mesh, mats, n_mat, h, tags,
                                     any_invisible, why);
    if (vs != TT_OK) return fail(c, vs, "scene validation failed: %s", why.c_str());
    std::vector<TriPos> tp(n_tris);
    for (uint32_t t = 0; t < n_tris; t++) derive_tri(tris[t], tp[t]);
    std::vector<MeshGpu> mg(n_mesh);
    for (uint32_t m = 0; m < n_mesh; m++) derive_mesh(md[m], mg[m]);
    c->nodes.release();
    c->tris_raw.release();
    c->tris.release();
    c->tlas.release();
    c->mesh_raw.release();
    c->mesh.release();
    c->mat_tag.release();
    c->mat_cut.release();
    c->mat_glass.release();
    // the TLAS region (every node the TLAS-level walk reaches lies in [0, tlas_res)) and TT_TLAS_SLOTS overlay
    // regions of that size behind the scene's nodes, for frame slots with TLASes of their own
    uint32_t tlas_res = 0;
    for (uint32_t n : h.tlas_nodes) tlas_res = std::max(tlas_res, n + 1u);
    if (((uint64_t)n_nodes + (uint64_t)TT_TLAS_SLOTS * tlas_res) * TT_NODE_STRIDE >= (1ull << 32))
        tlas_res = 0;  // no overlay regions (a node array near the 32-bit limit of the kernels' buffer loads)
    const uint32_t n_nodes_dev = n_nodes + TT_TLAS_SLOTS * tlas_res;
    hipError_t e;
    if ((e = c->nodes.alloc(n_nodes_dev)) != hipSuccess || (e = c->tris_raw.alloc(n_tris)) != hipSuccess ||
        (e = c->tris.alloc(n_tris)) != hipSuccess || (e = c->tlas.alloc(n_tlas)) != hipSuccess ||
        (e = c->mesh_raw.alloc(n_mesh)) != hipSuccess || (e = c->mesh.alloc(n_mesh)) != hipSuccess ||
        (e = c->mat_tag.alloc(tags.size())) != hipSuccess)
        return hip_fail(c, e, "scene allocation");
    TT_HIP(c, hipMemcpy(c->nodes.p, nodes, sizeof(tt_cwbvh_node) * n_nodes, hipMemcpyHostToDevice));
    if (TT_NODE_STRIDE != 80) {
        c->nodes_k.release();
        if ((e = c->nodes_k.alloc((size_t)n_nodes_dev * TT_NODE_STRIDE)) != hipSuccess) return hip_fail(c, e, "node copy");
        TT_HIP(c, hipMemsetAsync(c->nodes_k.p, 0, (size_t)n_nodes_dev * TT_NODE_STRIDE, c->stream));
        TT_HIP(c, refresh_node_copy(c, 0, n_nodes));
        TT_HIP(c, hipStreamSynchronize(c->stream));
    }
    TT_HIP(c, hipMemcpy(c->tris_raw.p, tris, sizeof(tt_cuda_triangle) * n_tris, hipMemcpyHostToDevice));
    TT_HIP(c, hipMemcpy(c->tris.p, tp.data(), sizeof(TriPos) * n_tris, hipMemcpyHostToDevice));
    TT_HIP(c, hipMemcpy(c->tlas.p, tlas, sizeof(int32_t) * n_tlas, hipMemcpyHostToDevice));
    TT_HIP(c, hipMemcpy(c->mesh_raw.p, md, sizeof(tt_mesh_data) * n_mesh, hipMemcpyHostToDevice));
    TT_HIP(c, hipMemcpy(c->mesh.p, mg.data(), sizeof(MeshGpu) * n_mesh, hipMemcpyHostToDevice));
    TT_HIP(c, hipMemcpy(c->mat_tag.p, tags.data(), sizeof(uint32_t) * tags.size(), hipMemcpyHostToDevice));
    if (h.any_cutout) {
        if ((e = c->mat_cut.alloc(h.cut.size())) != hipSuccess) return hip_fail(c, e, "cutout records");
        TT_HIP(c, hipMemcpy(c->mat_cut.p, h.cut.data(), sizeof(CutoutMat) * h.cut.size(), hipMemcpyHostToDevice));
    }
    if (h.any_atlas_shadow) {
        if ((e = c->mat_glass.alloc(h.glass.size())) != hipSuccess) return hip_fail(c, e, "glass records");
        TT_HIP(c, hipMemcpy(c->mat_glass.p, h.glass.data(), sizeof(GlassMat) * h.glass.size(), hipMemcpyHostToDevice));
    }
    c->host = std::move(h);
    c->n_nodes_scene = n_nodes;
    c->n_nodes_dev = n_nodes_dev;
    c->tlas_res = tlas_res;
    c->ovl_used = 0;
    c->root_known = true;
    c->any_invisible = any_invisible;
    c->scene_gen++;
    c->any_shadow_skip = c->host.any_shadow_skip;
    c->any_cutout = c->host.any_cutout;
    c->any_atlas_shadow = c->host.any_atlas_shadow;
    c->leaf.release();
    {
        const tt_status st = refresh_leaves(c);
        if (st != TT_OK) return st;
    }
    c->has_scene = true;
    return TT_OK;
}

tt_status tt_scene_upload_alpha_atlas(tt_ctx* c, const uint8_t* texels, uint32_t width, uint32_t height) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_BORROWER(c);
    TT_REFUSE_LENDER(c);
    if (!texels || width == 0 || height == 0 || (uint64_t)width * height > 0x7fffffffull)
        return fail(c, TT_ERR_INVALID_ARG, "tt_scene_upload_alpha_atlas: empty or oversized atlas");
    TT_HIP(c, hipSetDevice(c->device));
    c->atlas.release();
    c->atlas_w = c->atlas_h = 0;
    TT_HIP(c, c->atlas.alloc((size_t)width * height));
    TT_HIP(c, hipMemcpy(c->atlas.p, texels, (size_t)width * height, hipMemcpyHostToDevice));
    c->atlas_w = width;
    c->atlas_h = height;
    return TT_OK;
}

tt_status tt_scene_upload_texture_atlas(tt_ctx* c, const uint16_t* rgba_half, uint32_t width, uint32_t height) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_BORROWER(c);
    TT_REFUSE_LENDER(c);
    if (!rgba_half || width == 0 || height == 0 || (uint64_t)width * height > 0x7fffffffull / 8u)
        return fail(c, TT_ERR_INVALID_ARG, "tt_scene_upload_texture_atlas: empty or oversized atlas");
    TT_HIP(c, hipSetDevice(c->device));
    c->tex.release();
    c->tex_w = c->tex_h = 0;
    TT_HIP(c, c->tex.alloc((size_t)width * height));
    TT_HIP(c, hipMemcpy(c->tex.p, rgba_half, (size_t)width * height * 8u, hipMemcpyHostToDevice));
    c->tex_w = width;
    c->tex_h = height;
    return TT_OK;
}

}  // extern "C"

namespace {
// The host mirror a borrower keeps of its lender's scene: scalars and material records, never the node array
// or the validation bookkeeping (an overlay borrower adds its own TLAS-side arrays, tt_ctx_share_blas)
void copy_host_light(SceneHost& d, const SceneHost& s) {
    d = SceneHost{};
    d.n_tris = s.n_tris;
    d.n_mat = s.n_mat;
    d.any_shadow_skip = s.any_shadow_skip;
    d.any_atlas_shadow = s.any_atlas_shadow;
    d.any_cutout = s.any_cutout;
    d.cut = s.cut;
    d.glass = s.glass;
}

// Checks shared by tt_ctx_share_scene / tt_ctx_share_blas; then dst's previous scene ties are cut and the
// lender's read-only buffers borrowed (everything but the TLAS-side buffers an overlay owns).
tt_status share_begin(tt_ctx* dst, tt_ctx* src) {
    if (dst == src) return fail(dst, TT_ERR_INVALID_ARG, "a context cannot share its own scene");
    if (!src->has_scene) return fail(dst, TT_ERR_NO_SCENE, "the source context has no scene");
    if (src->lender) return fail(dst, TT_ERR_INVALID_ARG, "the source context shares another context's scene");
    if (dst->borrowers > 0) return fail(dst, TT_ERR_INVALID_ARG, "other contexts share this context's scene");
    if (dst->device != src->device) return fail(dst, TT_ERR_INVALID_ARG, "the contexts are on different devices");
    TT_HIP(dst, hipSetDevice(dst->device));
    TT_HIP(dst, hipStreamSynchronize(dst->stream));  // nothing of dst's still reads its old scene
    TT_HIP(dst, hipStreamSynchronize(src->stream));  // src's upload / updates have landed
    unlink_borrower(dst);
    dst->nodes.borrow(src->nodes);
    dst->nodes_k.borrow(src->nodes_k);
    dst->tris_raw.borrow(src->tris_raw);
    dst->tris.borrow(src->tris);
    dst->mat_tag.borrow(src->mat_tag);
    dst->mat_cut.borrow(src->mat_cut);
    dst->mat_glass.borrow(src->mat_glass);
    dst->tex.borrow(src->tex);
    dst->atlas.borrow(src->atlas);
    dst->tex_w = src->tex_w;
    dst->tex_h = src->tex_h;
    dst->atlas_w = src->atlas_w;
    dst->atlas_h = src->atlas_h;
    dst->any_invisible = src->any_invisible;
    dst->any_shadow_skip = src->any_shadow_skip;
    dst->any_atlas_shadow = src->any_atlas_shadow;
    dst->any_cutout = src->any_cutout;
    dst->n_nodes_scene = src->n_nodes_scene;
    dst->n_nodes_dev = src->n_nodes_dev;
    dst->tlas_res = 0;  // a borrower never lends
    dst->ovl = false;
    dst->tlas_base = 0;
    dst->n_tlas_own = 0;
    dst->root_known = false;
    return TT_OK;
}

void share_link(tt_ctx* dst, tt_ctx* src) {
    std::lock_guard<std::recursive_mutex> lk(src->mu);
    dst->has_scene = true;
    dst->scene_gen++;
    dst->lender = src;
    src->borrowers++;
    src->borrower_list.push_back(dst);
    if (dst->ovl) src->ovl_used |= 1u << dst->ovl_slot;
    dst->mut_waited = dst->ovl ? src->blas_mut : src->scene_mut;  // src's stream was synchronized above
    dst->read_waited = dst->read_seq;
}
}  // namespace

extern "C" {

// Traces on `dst` read `src`'s scene buffers (nodes, triangles, TLAS, mesh and leaf records, materials,
// atlases) instead of a copy: two contexts tracing concurrently (the two-part layout) then share one
// cache footprint. The borrowed buffers are read-only for `dst`.
tt_status tt_ctx_share_scene(tt_ctx* dst, tt_ctx* src) {
    if (!dst || !src) return TT_ERR_INVALID_ARG;
    const tt_status st = share_begin(dst, src);
    if (st != TT_OK) return st;
    dst->tlas.borrow(src->tlas);
    dst->mesh_raw.borrow(src->mesh_raw);
    dst->mesh.borrow(src->mesh);
    dst->leaf.borrow(src->leaf);
    copy_host_light(dst->host, src->host);
    share_link(dst, src);
    return TT_OK;
}

// A frame slot's own TLAS over `src`'s BLASes (include/truetrace_hip.h). The TLAS nodes [0, n_tlas_nodes) are
// copied from src's device array into a free overlay region behind the scene's nodes, TLASBVH8Indices and
// _MeshData (+ MeshGpu, LeafMesh) into buffers of dst's own; the kernels address the copy through
// TraceArgs::tlas_base (the TLAS-level NodeOffset), so the BLAS nodes and triangles stay one shared copy.
tt_status tt_ctx_share_blas(tt_ctx* dst, tt_ctx* src, uint32_t n_tlas_nodes) {
    if (!dst || !src) return TT_ERR_INVALID_ARG;
    if (dst == src) return fail(dst, TT_ERR_INVALID_ARG, "a context cannot share its own scene");
    if (!src->has_scene) return fail(dst, TT_ERR_NO_SCENE, "the source context has no scene");
    if (src->lender) return fail(dst, TT_ERR_INVALID_ARG, "the source context shares another context's scene");
    if (dst->borrowers > 0) return fail(dst, TT_ERR_INVALID_ARG, "other contexts share this context's scene");
    if (dst->device != src->device) return fail(dst, TT_ERR_INVALID_ARG, "the contexts are on different devices");
    if (src->tlas_res == 0)
        return fail(dst, TT_ERR_UNSUPPORTED, "the source scene has no overlay regions (TT_NODE_STRIDE != 80, or a node "
                                             "array near the 32-bit offset limit)");
    if (n_tlas_nodes == 0 || n_tlas_nodes > src->tlas_res)
        return fail(dst, TT_ERR_INVALID_ARG, "tt_ctx_share_blas: n_tlas_nodes %u outside (0, %u] (the TLAS region)",
                    n_tlas_nodes, src->tlas_res);
    // Everything that can fail on src's side -- the TLAS read-back and walk, the overlay buffers -- happens
    // before dst is touched, so a refused call leaves dst as it was. The TLAS-side state is taken
    // as the device holds it now (a device TLAS refit leaves src's host copy stale).
    TT_HIP(dst, hipSetDevice(dst->device));
    TT_HIP(dst, hipStreamSynchronize(src->stream));
    SceneHost h;
    {
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        copy_host_light(h, src->host);
        h.tlas = src->host.tlas;
        h.mesh = src->host.mesh;
        h.blas_ok = src->host.blas_ok;
    }
    h.nodes.resize(n_tlas_nodes);
    TT_HIP(dst, hipMemcpy(h.nodes.data(), src->nodes.p, sizeof(tt_cwbvh_node) * n_tlas_nodes, hipMemcpyDeviceToHost));
    {
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        Validator v(h, src->host);
        if (!v.walk(0, 0, 0, true))
            return fail(dst, TT_ERR_INVALID_ARG, "tt_ctx_share_blas: the TLAS leaves [0, %u): %s", n_tlas_nodes, v.why.c_str());
        h.is_tlas_node.assign(n_tlas_nodes, 0u);
        h.tlas_nodes = v.tlas_visit;
        for (uint32_t n : h.tlas_nodes) h.is_tlas_node[n] = 1u;
    }
    const uint32_t n_tlas = (uint32_t)h.tlas.size(), n_mesh = (uint32_t)h.mesh.size();
    struct Fresh {  // dst's own TLAS-side buffers, adopted once nothing can fail any more
        DevBuf<int32_t> tlas;
        DevBuf<tt_mesh_data> mesh_raw;
        DevBuf<MeshGpu> mesh;
        DevBuf<LeafMesh> leaf;
        ~Fresh() {
            tlas.release();
            mesh_raw.release();
            mesh.release();
            leaf.release();
        }
    } fr;
    hipError_t e;
    if ((e = fr.tlas.alloc(n_tlas)) != hipSuccess || (e = fr.mesh_raw.alloc(n_mesh)) != hipSuccess ||
        (e = fr.mesh.alloc(n_mesh)) != hipSuccess || (e = fr.leaf.alloc(src->leaf.n)) != hipSuccess)
        return hip_fail(dst, e, "overlay TLAS-side buffers");
    // the overlay region: picked and reserved in one locked section (two frame slots made concurrently
    // over one lender never get the same region); a re-share over the same lender keeps its region
    uint32_t slot = TT_TLAS_SLOTS;
    const bool same_slot = dst->ovl && dst->lender == src;
    {
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        if (same_slot) {
            slot = dst->ovl_slot;
        } else {
            for (uint32_t k = 0; k < TT_TLAS_SLOTS; k++)
                if (!((src->ovl_used >> k) & 1u)) {
                    slot = k;
                    break;
                }
            if (slot == TT_TLAS_SLOTS)
                return fail(dst, TT_ERR_UNSUPPORTED, "all %u overlay regions of the source scene are in use", TT_TLAS_SLOTS);
            src->ovl_used |= 1u << slot;
        }
    }
    auto release_slot = [&] {
        if (same_slot) return;
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        src->ovl_used &= ~(1u << slot);
    };
    if (same_slot) {
        // unlink_borrower (in share_begin) frees the region bit: keep it reserved across the re-share
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        dst->ovl = false;
    }
    const tt_status st = share_begin(dst, src);
    if (st != TT_OK) {
        if (same_slot) {
            std::lock_guard<std::recursive_mutex> lk(src->mu);
            if (dst->lender == src)
                dst->ovl = true;  // failed before unlinking: dst keeps its frame slot as it was
            else
                src->ovl_used &= ~(1u << slot);  // unlinked, then failed: the region goes with it
        } else {
            release_slot();
        }
        return st;
    }
    auto adopt = [](auto& to, auto& from) {
        to.release();
        to.p = from.p;
        to.n = from.n;
        to.own = true;
        from.p = nullptr;
        from.n = 0;
    };
    adopt(dst->tlas, fr.tlas);
    adopt(dst->mesh_raw, fr.mesh_raw);
    adopt(dst->mesh, fr.mesh);
    adopt(dst->leaf, fr.leaf);
    dst->host = std::move(h);
    dst->ovl = true;
    dst->ovl_slot = slot;
    dst->n_tlas_own = n_tlas_nodes;
    dst->tlas_base = src->n_nodes_scene + slot * src->tlas_res;
    // device copies: a failure here leaves dst with no scene at all (never a half-linked one)
    auto abort_share = [&](hipError_t err, const char* what) {
        (void)hipStreamSynchronize(dst->stream);
        dst->has_scene = false;
        dst->ovl = false;
        dst->tlas_base = 0;
        dst->n_tlas_own = 0;
        dst->root_known = false;
        dst->host = SceneHost{};
        dst->nodes.release();
        dst->nodes_k.release();
        dst->tris_raw.release();
        dst->tris.release();
        dst->mat_tag.release();
        dst->mat_cut.release();
        dst->mat_glass.release();
        dst->tex.release();
        dst->atlas.release();
        dst->tlas.release();
        dst->mesh_raw.release();
        dst->mesh.release();
        dst->leaf.release();
        release_slot();
        return hip_fail(dst, err, what);
    };
    if ((e = hipMemcpyAsync(dst->nodes.p + dst->tlas_base, src->nodes.p, sizeof(tt_cwbvh_node) * n_tlas_nodes,
                            hipMemcpyDeviceToDevice, dst->stream)) != hipSuccess ||
        (e = refresh_node_copy(dst, dst->tlas_base, n_tlas_nodes)) != hipSuccess ||
        (e = hipMemcpyAsync(dst->tlas.p, src->tlas.p, sizeof(int32_t) * n_tlas, hipMemcpyDeviceToDevice, dst->stream)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(dst->mesh_raw.p, src->mesh_raw.p, sizeof(tt_mesh_data) * n_mesh, hipMemcpyDeviceToDevice,
                            dst->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(dst->mesh.p, src->mesh.p, sizeof(MeshGpu) * n_mesh, hipMemcpyDeviceToDevice, dst->stream)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(dst->leaf.p, src->leaf.p, sizeof(LeafMesh) * src->leaf.n, hipMemcpyDeviceToDevice,
                            dst->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(dst->stream)) != hipSuccess)
        return abort_share(e, "tt_ctx_share_blas: overlay copies");
    dst->root_known = true;  // its host TLAS copy is what the device holds
    share_link(dst, src);
    return TT_OK;
}

tt_status tt_tlas_refit(tt_ctx* c, uint32_t n_tlas_nodes, const float* mesh_aabbs, uint32_t n_mesh, uint32_t flags) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_REFUSE_BORROWER_TLAS(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    // (an overlay borrower's host.nodes are its own TLAS nodes: it refits those, in its overlay region)
    if (!mesh_aabbs || n_tlas_nodes == 0 || n_tlas_nodes > c->host.nodes.size())
        return fail(c, TT_ERR_INVALID_ARG, "tt_tlas_refit: null boxes or n_tlas_nodes out of range");
    if (n_mesh < c->host.mesh.size())
        return fail(c, TT_ERR_INVALID_ARG, "tt_tlas_refit: need one AABB per _MeshData record (%zu)", c->host.mesh.size());
    TT_HIP(c, hipSetDevice(c->device));
    if (c->refit_gen != c->scene_gen || c->refit_n_tlas != n_tlas_nodes) {
        RefitPlan plan;
        if (!tt_refit_build_plan(c->host.nodes.data(), n_tlas_nodes, plan))
            return fail(c, TT_ERR_INVALID_ARG, "tt_tlas_refit: a TLAS child index leaves [0, n_tlas_nodes)");
        TT_HIP(c, hipStreamSynchronize(c->stream));  // the old plan's buffers may be in use
        TT_HIP(c, tt_refit_prepare(plan, c->host.nodes.data(), n_tlas_nodes, c->refit));
        c->refit_gen = c->scene_gen;
        c->refit_n_tlas = n_tlas_nodes;
    }
    const float* d_boxes = mesh_aabbs;
    if (flags & TT_TRACE_DEVICE_PTRS) {
        if (!is_device_ptr(mesh_aabbs)) return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_DEVICE_PTRS set but boxes are not device memory");
    } else {
        if (c->st_boxes.n < (size_t)6 * n_mesh) TT_HIP(c, c->st_boxes.alloc((size_t)6 * n_mesh));
        TT_HIP(c, hipMemcpyAsync(c->st_boxes.p, mesh_aabbs, sizeof(float) * 6 * n_mesh, hipMemcpyHostToDevice, c->stream));
        d_boxes = c->st_boxes.p;
    }
    uint32_t slot;
    SceneWrite sw(c, false, !c->ovl);  // (an overlay's TLAS is read by nobody else)
    TT_HIP(c, sw.err);
    TT_HIP(c, ring_open(c, slot));
    TT_HIP(c, tt_refit_run(c->refit, d_boxes, c->tlas.p, c->nodes.p + c->tlas_base, c->stream));
    TT_HIP(c, refresh_node_copy(c, c->tlas_base, n_tlas_nodes));
    {
        std::lock_guard<std::recursive_mutex> lk(c->mu);
        c->root_known = false;  // node 0 was rewritten on the device
    }
    TT_HIP(c, ring_close(c, slot));
    TT_HIP(c, sw.end());
    if (!(flags & TT_TRACE_ASYNC) || !(flags & TT_TRACE_DEVICE_PTRS)) TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

tt_status tt_blas_refit(tt_ctx* c, const tt_blas_refit_params* p, const float* vertices, const int32_t* indices,
                        const int32_t* leaf_of_triangle) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_REFUSE_BORROWER(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!p || !vertices || !indices || !leaf_of_triangle || !p->n_tris || !p->n_vertices || p->vertex_stride < 6)
        return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: null array, empty mesh or vertex_stride < 6");
    if (p->mesh_index >= c->host.mesh.size())
        return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: mesh_index %u out of range", p->mesh_index);
    const tt_mesh_data& md = c->host.mesh[p->mesh_index];
    const uint32_t node_base = (uint32_t)md.NodeOffset, tri_base = (uint32_t)md.TriOffset;
    if ((uint32_t)(md.mesh_data_bvh_offsets & 0x7fffffff) != node_base || node_base >= c->host.nodes.size())
        return fail(c, TT_ERR_UNSUPPORTED, "tt_blas_refit: the mesh's BLAS root is not its first node");
    if ((uint64_t)tri_base + p->n_tris > c->host.n_tris)
        return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: TriOffset + n_tris exceeds the scene's triangles");
    const bool dev = (p->flags & TT_TRACE_DEVICE_PTRS) != 0;
    if (dev && !(is_device_ptr(vertices) && is_device_ptr(indices) && is_device_ptr(leaf_of_triangle)))
        return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_DEVICE_PTRS set but an array is not device memory");
    if (!dev) {
        for (uint64_t i = 0; i < 3ull * p->n_tris; i++)
            if (indices[i] < 0 || (uint32_t)indices[i] >= p->n_vertices)
                return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: index %d out of range", indices[i]);
        for (uint32_t i = 0; i < p->n_tris; i++)
            if (leaf_of_triangle[i] < 0 || (uint32_t)leaf_of_triangle[i] >= p->n_tris)
                return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: leaf_of_triangle[%u] out of range", i);
    }
    TT_HIP(c, hipSetDevice(c->device));
    tt_ctx::BlasRefit& R = c->blas_refit[p->mesh_index];
    if (R.gen != c->scene_gen || R.node_base != node_base || R.boxes.n < (size_t)6 * p->n_tris) {
        RefitPlan plan;
        const tt_cwbvh_node* base = c->host.nodes.data() + node_base;
        if (!tt_refit_build_plan(base, (uint32_t)(c->host.nodes.size() - node_base), plan))
            return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: a BLAS child index leaves the node array");
        if ((uint32_t)plan.leaf_end > p->n_tris)
            return fail(c, TT_ERR_INVALID_ARG, "tt_blas_refit: the BLAS references triangle %d beyond n_tris", plan.leaf_end - 1);
        uint32_t n_used = 0;
        for (int32_t b : plan.pair_bvh) n_used = std::max(n_used, (uint32_t)b + 1u);
        TT_HIP(c, hipStreamSynchronize(c->stream));  // the old plan's buffers may be in use
        TT_HIP(c, tt_refit_prepare(plan, base, n_used, R.dev));
        R.n_nodes = n_used;
        if (R.boxes.n < (size_t)6 * p->n_tris) TT_HIP(c, R.boxes.alloc((size_t)6 * p->n_tris));
        R.gen = c->scene_gen;
        R.node_base = node_base;
    }
    BlasConstructArgs a{};
    a.vertices = vertices;
    a.indices = indices;
    a.leaf_of = leaf_of_triangle;
    if (!dev) {
        const size_t nv = (size_t)p->n_vertices * p->vertex_stride;
        if (c->st_vtx.n < nv) TT_HIP(c, c->st_vtx.alloc(nv));
        if (c->st_idx.n < 3ull * p->n_tris) TT_HIP(c, c->st_idx.alloc(3ull * p->n_tris));
        if (c->st_leaf.n < p->n_tris) TT_HIP(c, c->st_leaf.alloc(p->n_tris));
        TT_HIP(c, hipMemcpyAsync(c->st_vtx.p, vertices, sizeof(float) * nv, hipMemcpyHostToDevice, c->stream));
        TT_HIP(c, hipMemcpyAsync(c->st_idx.p, indices, sizeof(int32_t) * 3 * p->n_tris, hipMemcpyHostToDevice, c->stream));
        TT_HIP(c, hipMemcpyAsync(c->st_leaf.p, leaf_of_triangle, sizeof(int32_t) * p->n_tris, hipMemcpyHostToDevice, c->stream));
        a.vertices = c->st_vtx.p;
        a.indices = c->st_idx.p;
        a.leaf_of = c->st_leaf.p;
    }
    a.n_tris = p->n_tris;
    a.n_vertices = p->n_vertices;
    a.vertex_stride = p->vertex_stride;
    std::memcpy(a.m, p->transform, sizeof(a.m));
    a.boxes = R.boxes.p;
    a.tris88 = c->tris_raw.p + tri_base;
    a.tripos = c->tris.p + tri_base;
    uint32_t slot;
    SceneWrite sw(c, true);
    TT_HIP(c, sw.err);
    TT_HIP(c, ring_open(c, slot));
    TT_HIP(c, tt_blas_construct(a, c->stream));
    TT_HIP(c, tt_refit_run(R.dev, R.boxes.p, nullptr, c->nodes.p + node_base, c->stream));
    TT_HIP(c, refresh_node_copy(c, node_base, R.n_nodes));
    TT_HIP(c, ring_close(c, slot));
    TT_HIP(c, sw.end());
    if (!(p->flags & TT_TRACE_ASYNC) || !dev) TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

tt_status tt_scene_read_tris(tt_ctx* c, uint32_t first, uint32_t count, tt_cuda_triangle* out) {
    if (!c) return TT_ERR_INVALID_ARG;
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!out || (uint64_t)first + count > c->host.n_tris)
        return fail(c, TT_ERR_INVALID_ARG, "tt_scene_read_tris: range out of bounds");
    TT_HIP(c, hipSetDevice(c->device));
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    TT_HIP(c, hipMemcpyAsync(out, c->tris_raw.p + first, sizeof(tt_cuda_triangle) * count, hipMemcpyDeviceToHost, c->stream));
    sr.end();
    TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

tt_status tt_scene_read_nodes(tt_ctx* c, uint32_t first, uint32_t count, tt_cwbvh_node* out) {
    if (!c) return TT_ERR_INVALID_ARG;
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!out || (uint64_t)first + count > c->n_nodes_scene)
        return fail(c, TT_ERR_INVALID_ARG, "tt_scene_read_nodes: range out of bounds");
    TT_HIP(c, hipSetDevice(c->device));
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    // the scene as this context traces it: an overlay borrower's TLAS nodes [0, n_tlas_own) from its region
    const uint32_t own_end = c->ovl ? std::max(first, std::min(first + count, c->n_tlas_own)) : first;
    if (own_end > first)
        TT_HIP(c, hipMemcpyAsync(out, c->nodes.p + c->tlas_base + first, sizeof(tt_cwbvh_node) * (own_end - first),
                                 hipMemcpyDeviceToHost, c->stream));
    if (first + count > own_end)
        TT_HIP(c, hipMemcpyAsync(out + (own_end - first), c->nodes.p + own_end,
                                 sizeof(tt_cwbvh_node) * (first + count - own_end), hipMemcpyDeviceToHost, c->stream));
    sr.end();
    TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

tt_status tt_scene_validate(const tt_cwbvh_node* nodes, uint32_t n_nodes, const tt_cuda_triangle* tris, uint32_t n_tris,
                            const int32_t* tlas, uint32_t n_tlas, const tt_mesh_data* md, uint32_t n_mesh,
                            const tt_material* mats, uint32_t n_mat, char* why, uint32_t why_len) {
    SceneHost h;
    std::vector<uint32_t> tags;
    bool any_invisible = false;
    std::string w;
    const tt_status st = check_scene(nodes, n_nodes, tris, n_tris, tlas, n_tlas, md, n_mesh, mats, n_mat, h, tags,
                                     any_invisible, w);
    if (why && why_len) {
        std::strncpy(why, w.c_str(), why_len - 1);
        why[why_len - 1] = 0;
    }
    return st;
}

namespace {
// Copies `bytes` of caller memory into the next pinned staging slot (waiting, if needed, until the
// copy last enqueued from that slot has completed), so the H2D copy can be asynchronous and the
// caller may reuse its buffer as soon as the call returns. stage_end() marks the slot in use by the
// copies enqueued since.
hipError_t stage_begin(tt_ctx* c, const void* src, size_t bytes, void*& out) {
    tt_ctx::Pinned& pn = c->pin[c->pin_cur];
    hipError_t e;
    if (!pn.ev && (e = hipEventCreateWithFlags(&pn.ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (pn.pending) {
        if ((e = hipEventSynchronize(pn.ev)) != hipSuccess) return e;
        pn.pending = false;
    }
    if (pn.n < bytes) {
        if (pn.p) (void)hipHostFree(pn.p);
        pn.p = nullptr;
        pn.n = 0;
        if ((e = hipHostMalloc(&pn.p, bytes, hipHostMallocDefault)) != hipSuccess) return e;
        pn.n = bytes;
    }
    std::memcpy(pn.p, src, bytes);
    out = pn.p;
    return hipSuccess;
}
hipError_t stage_end(tt_ctx* c) {
    tt_ctx::Pinned& pn = c->pin[c->pin_cur];
    c->pin_cur ^= 1u;
    const hipError_t e = hipEventRecord(pn.ev, c->stream);
    pn.pending = e == hipSuccess;
    return e;
}

// Rebuilds the TLAS leaf records from the host mirror (on upload) and uploads them on the stream.
tt_status refresh_leaves(tt_ctx* c) {
    std::vector<LeafMesh> lv = derive_leaves(c->host.tlas, c->host.mesh);
    if (c->leaf.n < lv.size()) {
        c->leaf.release();
        const hipError_t e = c->leaf.alloc(lv.size());
        if (e != hipSuccess) return hip_fail(c, e, "TLAS leaf records");
    }
    TT_HIP(c, hipMemcpyAsync(c->leaf.p, lv.data(), sizeof(LeafMesh) * lv.size(), hipMemcpyHostToDevice, c->stream));
    TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}
}  // namespace

tt_status tt_scene_update_nodes(tt_ctx* c, uint32_t first, uint32_t count, const tt_cwbvh_node* nodes) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_REFUSE_BORROWER_TLAS(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!nodes || (uint64_t)first + count > c->host.nodes.size())
        return fail(c, TT_ERR_INVALID_ARG, c->ovl ? "node update range out of bounds: a frame-slot TLAS (tt_ctx_share_blas) "
                                                    "rewrites only its own TLAS nodes"
                                                  : "node update range out of bounds");
    if (count == 0) return TT_OK;
    SceneHost& h = c->host;
    tt_ctx* L = c->ovl ? c->lender : nullptr;
    bool tlas_only = true, blas_side = false;
    {
        std::lock_guard<std::recursive_mutex> lk(L ? L->mu : c->mu);  // the nodes the walks read; node 0 (TT_ROOT_LEAF)
        std::vector<tt_cwbvh_node> saved(h.nodes.begin() + first, h.nodes.begin() + first + count);
        std::copy(nodes, nodes + count, h.nodes.begin() + first);
        // A rewrite of TLAS-level nodes only (the per-frame case: BVH8AggregatedBuffer.SetData of the
        // TLAS region) re-walks the TLAS level; the BLASes were validated at upload and are unchanged.
        // Any other rewrite re-validates the whole scene.
        // (a node that a validated BLAS also reaches -- a TLAS rewrite may have re-pointed a child into one
        // -- takes the full check: its triangle indices matter at BLAS level)
        // blas_side: the rewrite touches what frame-slot TLASes read too (a BLAS node, or a node outside the
        // TLAS region); on a frame slot every node of its range is its own TLAS region's
        const std::vector<uint8_t>& blas_nodes = L ? L->host.is_blas_node : h.is_blas_node;
        for (uint32_t i = first; i < first + count; i++) {
            tlas_only = tlas_only && (L || h.is_tlas_node[i] != 0) && blas_nodes[i] == 0;
            blas_side = blas_side || blas_nodes[i] != 0 || (!L && i >= c->tlas_res);
        }
        const char* refuse = nullptr;
        if (!tlas_only && L) refuse = "a frame-slot TLAS (tt_ctx_share_blas) rewrites TLAS nodes only";
        if (blas_side && !L && c->ovl_used)
            refuse = "a BLAS-side node rewrite while frame-slot TLASes (tt_ctx_share_blas) share this scene";
        if (refuse) {
            std::copy(saved.begin(), saved.end(), h.nodes.begin() + first);
            return fail(c, L ? TT_ERR_INVALID_ARG : TT_ERR_UNSUPPORTED, "%s", refuse);
        }
        Validator v = L ? Validator(h, L->host) : Validator(h);
        const bool ok = tlas_only ? v.walk(0, 0, 0, true) : v.run();
        if (!ok) {
            std::copy(saved.begin(), saved.end(), h.nodes.begin() + first);
            return fail(c, TT_ERR_INVALID_ARG, "scene validation failed after node update: %s", v.why.c_str());
        }
        if (tlas_only) {
            for (uint32_t n : h.tlas_nodes) h.is_tlas_node[n] = 0u;
            h.tlas_nodes = v.tlas_visit;
            for (uint32_t n : h.tlas_nodes) h.is_tlas_node[n] = 1u;
        } else {
            remember_validation(h, v);
        }
        if (first == 0) c->root_known = true;  // node 0 is the host's again
    }
    TT_HIP(c, hipSetDevice(c->device));
    void* pinned = nullptr;
    TT_HIP(c, stage_begin(c, nodes, sizeof(tt_cwbvh_node) * count, pinned));
    SceneWrite sw(c, blas_side, !c->ovl);
    TT_HIP(c, sw.err);
    TT_HIP(c, hipMemcpyAsync(c->nodes.p + c->tlas_base + first, pinned, sizeof(tt_cwbvh_node) * count,
                             hipMemcpyHostToDevice, c->stream));
    TT_HIP(c, stage_end(c));
    TT_HIP(c, refresh_node_copy(c, c->tlas_base + first, count));
    TT_HIP(c, sw.end());
    c->scene_gen++;  // a rewritten TLAS may have a new topology: the refit plan is rebuilt
    return TT_OK;
}

tt_status tt_scene_update_meshdata(tt_ctx* c, uint32_t first, uint32_t count, const tt_mesh_data* md) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    TT_REFUSE_BORROWER_TLAS(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!md || (uint64_t)first + count > c->host.mesh.size())
        return fail(c, TT_ERR_INVALID_ARG, "meshdata update range out of bounds");
    if (count == 0) return TT_OK;
    SceneHost& h = c->host;
    tt_ctx* L = c->ovl ? c->lender : nullptr;  // a frame-slot TLAS: its records, the lender's BLASes
    // Only records whose BLAS reference (root, NodeOffset, TriOffset) changed need a check, and only
    // against the BLASes validated so far; a BLAS never seen is walked once and remembered. The
    // per-frame transform update (MeshDataBuffer.SetData, AssetManager.cs:1825) changes none.
    std::vector<SceneHost::BlasKey> added;
    for (uint32_t i = 0; i < count; i++) {
        const tt_mesh_data& r = md[i];
        const tt_mesh_data& o = h.mesh[first + i];
        if (r.NodeOffset == o.NodeOffset && r.TriOffset == o.TriOffset &&
            ((r.mesh_data_bvh_offsets ^ o.mesh_data_bvh_offsets) & 0x7fffffff) == 0)
            continue;
        if (r.NodeOffset < 0 || r.TriOffset < 0)
            return fail(c, TT_ERR_INVALID_ARG, "scene validation failed after meshdata update: negative mesh offsets");
        const SceneHost::BlasKey k{(uint32_t)(r.mesh_data_bvh_offsets & 0x7fffffff), (uint32_t)r.NodeOffset,
                                   (uint32_t)r.TriOffset};
        if (std::binary_search(h.blas_ok.begin(), h.blas_ok.end(), k) ||
            std::find(added.begin(), added.end(), k) != added.end())
            continue;
        std::lock_guard<std::recursive_mutex> lk(L ? L->mu : c->mu);
        Validator v = L ? Validator(h, L->host) : Validator(h);
        if (!v.walk_mesh(r))
            return fail(c, TT_ERR_INVALID_ARG, "scene validation failed after meshdata update: %s", v.why.c_str());
        added.push_back(k);
        // (kept even if a later record fails: conservative; an overlay's BLASes are marked in the lender's
        // bookkeeping, so a later lender rewrite of those nodes is refused while overlays exist)
        std::vector<uint8_t>& blas_nodes = L ? L->host.is_blas_node : h.is_blas_node;
        for (uint32_t n : v.blas_visit) blas_nodes[n] = 1u;
    }
    if (!added.empty()) {
        h.blas_ok.insert(h.blas_ok.end(), added.begin(), added.end());
        std::sort(h.blas_ok.begin(), h.blas_ok.end());
    }
    std::memcpy(h.mesh.data() + first, md, sizeof(tt_mesh_data) * count);
    TT_HIP(c, hipSetDevice(c->device));
    // one small kernel on the stream reads the records in place from the pinned staging slot, stores them
    // to _MeshData in HBM, derives the traversal records (MeshGpu) and patches the TLAS leaf records that
    // name an updated mesh (no copy operation: each one waits for a free CU slot beside the trace grids)
    void* pinned = nullptr;
    TT_HIP(c, stage_begin(c, md, sizeof(tt_mesh_data) * count, pinned));
    SceneWrite sw(c, false, !c->ovl);  // (an overlay's records are read by nobody else)
    TT_HIP(c, sw.err);
    void* src = nullptr;
    TT_HIP(c, hipHostGetDevicePointer(&src, pinned, 0));
    const uint32_t n_tlas = (uint32_t)h.tlas.size();
    const uint32_t n = std::max(count, n_tlas);
    hipLaunchKernelGGL(tt_update_mesh_kernel, dim3((n + 255u) / 256u), dim3(256), 0, c->stream,
                       static_cast<const tt_mesh_data*>(src), c->mesh_raw.p, c->mesh.p, c->leaf.p, c->tlas.p, n_tlas, first,
                       count);
    TT_HIP(c, hipGetLastError());
    TT_HIP(c, stage_end(c));  // (after the kernel: it reads the staging slot)
    TT_HIP(c, sw.end());
    return TT_OK;
}

tt_status tt_scene_bytes(const tt_ctx* c, uint64_t* bytes) {
    if (!c || !bytes) return TT_ERR_INVALID_ARG;
    *bytes = c->nodes.n * sizeof(tt_cwbvh_node) + c->nodes_k.n + c->tris_raw.n * sizeof(tt_cuda_triangle) + c->tris.n * sizeof(TriPos) +
             c->tlas.n * 4 + c->mesh_raw.n * sizeof(tt_mesh_data) + c->mesh.n * sizeof(MeshGpu) + c->mat_tag.n * 4;
    return TT_OK;
}

namespace {
MatView mat_view(const tt_ctx* c) {
    MatView m;
    m.word = c->mat_tag.p;
    m.cut = c->mat_cut.p;
    m.raw = c->tris_raw.p;
    m.atlas = c->atlas.p;
    m.n_mat = c->host.n_mat;
    m.atlas_w = c->atlas_w;
    m.atlas_h = c->atlas_h;
    m.glass = c->mat_glass.p;
    m.tex = c->tex.p;
    m.tex_w = c->tex_w;
    m.tex_h = c->tex_h;
    return m;
}
}  // namespace

hipStream_t tt_ctx_stream_of(tt_ctx* c) { return c->stream; }  // tt_build.hip
hipError_t tt_ctx_bind_device(tt_ctx* c) { return hipSetDevice(c->device); }  // tt_build.hip
void tt_ctx_set_error(tt_ctx* c, const char* msg) {                // tt_build.hip
    if (c) c->err = msg ? msg : "";
}

}  // extern "C"

// n_dev (nullable): the device-resident ray count (tt_trace_closest_indirect); p->n_rays is then the
// capacity the launch covers, and the call is asynchronous with device pointers.
static tt_status trace_closest_call(tt_ctx* c, const tt_trace_params* p, const uint32_t* n_dev, tt_ray_data* rays,
                                    uint32_t* info, const tt_col_data* colors, tt_stats* stats,
                                    uint32_t* hits_out = nullptr) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!p || !rays) return fail(c, TT_ERR_INVALID_ARG, "null params or rays");
    if (p->screen_width == 0 || p->screen_height == 0) return fail(c, TT_ERR_INVALID_ARG, "zero screen size");
    if (p->bounce < 0) return fail(c, TT_ERR_INVALID_ARG, "negative bounce");
    // FarPlane (camera.farClipPlane) seeds best.t, the node test's t_max; the kernel's t_max clamp
    // assumes it is not a NaN (tt_traverse.h)
    if (p->far_plane != p->far_plane) return fail(c, TT_ERR_INVALID_ARG, "far_plane is NaN");
    if (info && p->bounce > 0 && !colors)
        return fail(c, TT_ERR_INVALID_ARG, "GlobalColors required for _PrimaryTriangleInfo at bounce > 0");
    if (c->any_cutout && !c->atlas.p)
        return fail(c, TT_ERR_UNSUPPORTED,
                    "scene has Cutout materials but no alpha atlas was uploaded (tt_scene_upload_alpha_atlas)");
    const uint64_t wh = (uint64_t)p->screen_width * p->screen_height;
    if (wh > 0x7fffffffull) return fail(c, TT_ERR_INVALID_ARG, "screen too large");
    const uint32_t off = (p->bounce % 2 == 1) ? (uint32_t)wh : 0u;
    if ((uint64_t)off + p->n_rays > 0xffffffffull) return fail(c, TT_ERR_INVALID_ARG, "ray range overflows");
    const bool dev = (p->flags & TT_TRACE_DEVICE_PTRS) != 0;
    const bool async = dev && ((p->flags & TT_TRACE_ASYNC) || n_dev);
    const bool want_stats = (p->flags & TT_TRACE_STATS) != 0;
    const int info_mode = info ? (p->bounce == 0 ? 1 : 2) : 0;
    const bool adaptive = (p->flags & TT_TRACE_ADAPTIVE_ORDER) && !want_stats && !n_dev;
    if (n_dev) {
        if (!dev) return fail(c, TT_ERR_INVALID_ARG, "a device-resident ray count needs TT_TRACE_DEVICE_PTRS");
        if (want_stats) return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_STATS needs a host ray count");
        if (!is_device_ptr(n_dev)) return fail(c, TT_ERR_INVALID_ARG, "the ray count pointer is not device memory");
    }
    if (hits_out) {
        if (!dev) return fail(c, TT_ERR_INVALID_ARG, "a hit-record stream needs TT_TRACE_DEVICE_PTRS");
        if (!is_device_ptr(hits_out)) return fail(c, TT_ERR_INVALID_ARG, "hits_out is not device memory");
        if (reinterpret_cast<uintptr_t>(hits_out) % 16) return fail(c, TT_ERR_INVALID_ARG, "hits_out must be 16-byte aligned");
        // the kernel stores record i at the 32-bit byte offset 16 i of a 2 GiB buffer descriptor
        if (p->n_rays > (1u << 27)) return fail(c, TT_ERR_INVALID_ARG, "a hit-record stream holds at most 2^27 rays per call");
    }
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if (p->n_rays == 0) return TT_OK;
    if (reinterpret_cast<uintptr_t>(rays) % 16 || (info && reinterpret_cast<uintptr_t>(info) % 16))
        return fail(c, TT_ERR_INVALID_ARG, "GlobalRays / _PrimaryTriangleInfo must be 16-byte aligned");
    TT_HIP(c, hipSetDevice(c->device));

    tt_ray_data* d_rays = rays;
    uint32_t* d_info = info;
    const tt_col_data* d_colors = colors;
    const size_t ray_end = (size_t)off + p->n_rays;
    if (dev) {
        if (!is_device_ptr(rays)) return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_DEVICE_PTRS set but rays is not device memory");
    } else {
        if (c->st_rays.n < ray_end) TT_HIP(c, c->st_rays.alloc(ray_end));
        d_rays = c->st_rays.p;
        TT_HIP(c, hipMemcpyAsync(d_rays + off, rays + off, sizeof(tt_ray_data) * p->n_rays, hipMemcpyHostToDevice, c->stream));
        if (info) {
            if (c->st_info.n < wh * 4) TT_HIP(c, c->st_info.alloc(wh * 4));
            d_info = c->st_info.p;
            TT_HIP(c, hipMemcpyAsync(d_info, info, sizeof(uint32_t) * 4 * wh, hipMemcpyHostToDevice, c->stream));
        }
        if (info && p->bounce > 0) {
            if (c->st_colors.n < wh) TT_HIP(c, c->st_colors.alloc(wh));
            TT_HIP(c, hipMemcpyAsync(c->st_colors.p, colors, sizeof(tt_col_data) * wh, hipMemcpyHostToDevice, c->stream));
            d_colors = c->st_colors.p;
        }
    }
    TraceArgs a;
    std::memset(&a, 0, sizeof(a));
    a.nodes = kernel_nodes(c);
    a.n_nodes = c->n_nodes_dev;  // (the overlay regions included: a frame-slot TLAS lives there)
    a.tlas_base = c->tlas_base;
    a.tris = c->tris.p;
    a.n_tris = c->host.n_tris;
    a.tlas = c->tlas.p;
    a.mesh = c->mesh.p;
    a.leaf = c->leaf.p;
    a.mat_tag = c->mat_tag.p;
    a.n_mat = c->host.n_mat;
    a.mat = mat_view(c);
    a.rays = d_rays;
    a.info = d_info;
    a.colors = d_colors;
    const uint32_t ci = c->ctl_cur;
    a.ctl = c->ctl + ci;
    a.ctl_next = c->ctl + (ci ^ 1u);
    a.sticky_overflow = c->sticky;
    a.spill = c->spill.p;
    a.n_rays = p->n_rays;
    a.n_rays_dev = n_dev;
    a.ray_offset = off;
    a.width = p->screen_width;
    a.height = p->screen_height;
    a.n_pixels = (uint32_t)wh;
    a.far_plane = p->far_plane;
    a.bounce = p->bounce;
    a.flags = p->flags;
    // (the kernel also requires its actual count to be W*H: a device count decides at run time)
    a.tile_swizzle = ((n_dev ? p->n_rays >= wh : p->n_rays == wh) && p->screen_width % 8 == 0 &&
                      p->screen_height % 8 == 0) ? 1u : 0u;
    a.div_width = fastdiv_make(std::max(1u, p->screen_width));
    a.div_tiles = fastdiv_make(std::max(1u, p->screen_width >> 3));
    a.hits_out = reinterpret_cast<uint4*>(hits_out);
    {  // TT_ROOT_LEAF: node 0 as a one-leaf TLAS root, when the host knows the device's node 0 (the lender's,
       // or a frame-slot TLAS's own)
        tt_ctx* owner = (c->lender && !c->ovl) ? c->lender : c;
        std::lock_guard<std::recursive_mutex> lk(owner->mu);
        if (owner->root_known && !owner->host.nodes.empty()) {
            a.root = root_leaf_of(reinterpret_cast<const uint32_t*>(owner->host.nodes.data()));
            a.root.base_child += c->tlas_base;
        }
    }
#ifdef TT_DIAG_BLOCKS  // diagnostic builds only: the block counters' device buffer (tools/diag_blocks.py)
    if (const char* dp = std::getenv("TT_DIAG_PTR"))
        a.diag_times = reinterpret_cast<unsigned long long*>(std::strtoull(dp, nullptr, 0));
#endif
    const bool matcheck = (c->any_invisible && p->bounce == 0) || c->any_cutout ||
                          ((p->flags & TT_TRACE_IGNORE_GLASS) && c->host.any_atlas_shadow) ||
                          ((p->flags & TT_TRACE_IGNORE_BACKFACING) && p->bounce == 0);
    // one dequeue chunk per wave: a launch smaller than the resident grid spreads over as many
    // waves as it has chunks (r02: sizing this for 256-ray chunks left a 260k-ray launch -- one
    // rank's shard at 8 GPUs -- on ~1 wave per SIMD, 4 chunks each)
    static const uint32_t chunks_per_wave = [] {  // TT_CHUNKS_PER_WAVE: experiment knob (default 1)
        const char* e = std::getenv("TT_CHUNKS_PER_WAVE");
        const int v = e ? std::atoi(e) : 1;
        return (uint32_t)std::max(1, std::min(v, 64));
    }();
    const uint32_t chunks_needed = (p->n_rays + tt_trace_chunk_rays() - 1u) / tt_trace_chunk_rays();
    const uint32_t waves_needed = (chunks_needed + chunks_per_wave - 1u) / chunks_per_wave;
    const uint32_t wpb = std::max(1u, tt_trace_block_size() / 64u);  // waves per block
    const uint32_t blocks_needed = (waves_needed + wpb - 1u) / wpb;
    const uint32_t grid = std::max(
        1u, std::min(c->grid_of[(adaptive ? 12 : want_stats ? 6 : 0) + (matcheck ? 3 : 0) + info_mode], blocks_needed));
    // TT_TRACE_ADAPTIVE_ORDER: this launch fills cost[cur ^ 1] (per 64-ray chunk); with the previous
    // launch's costs in cost[cur] the order kernel (inside the timed entry) sorts this launch's chunks
    tt_ctx::OrderSlot* os = nullptr;
    const uint32_t n_chunks = (p->n_rays + 63u) / 64u;
    if (adaptive) {
        os = &c->ord[std::min(p->bounce, 7)];
        if (os->w != p->screen_width || os->h != p->screen_height) {  // (costs outlive scene updates: a hint)
            os->valid = false;
            os->w = p->screen_width;
            os->h = p->screen_height;
        }
        if (os->order.n < n_chunks) {  // (a fresh map pair starts from zero costs)
            TT_HIP(c, os->order.alloc(n_chunks));
            TT_HIP(c, os->cost[0].alloc(n_chunks));
            TT_HIP(c, os->cost[1].alloc(n_chunks));
            TT_HIP(c, hipMemsetAsync(os->cost[0].p, 0, sizeof(uint32_t) * n_chunks, c->stream));
            os->valid = false;
        }
        if (!os->valid) TT_HIP(c, hipMemsetAsync(os->cost[os->cur ^ 1u].p, 0, sizeof(uint32_t) * n_chunks, c->stream));
        a.chunk_cost = os->cost[os->cur ^ 1u].p;
    }
    // Control blocks: every trace kernel zeroes the OTHER block at its start (block 0, plain stores;
    // the previous launch on the stream, which used it, has finished), so back-to-back async
    // launches need no fill kernel in between. Synchronous / stats launches, and the first launch
    // after an any-hit launch, still zero their block here. (A reset by the last wave to exit instead
    // needs a device-scope fence per wave, which writes back L2 under the draining waves: measured
    // 15% slower, profiles/r01_exp_ctl_reset.txt.)
    static const bool always_reset = std::getenv("TT_CTL_ALWAYS_RESET") != nullptr;  // A/B knob
    if (!async || want_stats || !c->ctl_zero[ci] || always_reset)
        TT_HIP(c, hipMemsetAsync(c->ctl + ci, 0, sizeof(TraceControl), c->stream));
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    const uint32_t slot = c->ring_n % TT_RING;
    const bool ring = c->timing || !async;  // (a synchronous call reports its kernel time)
    if (ring) TT_HIP(c, hipEventRecord(c->ring0[slot], c->stream));
    c->ctl_zero[0] = c->ctl_zero[1] = false;
    static const bool record_only = std::getenv("TT_ORDER_RECORD_ONLY") != nullptr;  // A/B knob: costs, no order
    if (os && os->valid && record_only)  // the order kernel (which clears the map this launch fills) is skipped
        TT_HIP(c, hipMemsetAsync(os->cost[os->cur ^ 1u].p, 0, sizeof(uint32_t) * n_chunks, c->stream));
    if (os && os->valid && !record_only) {
        OrderArgs o;
        o.cost = os->cost[os->cur].p;
        o.cost_clear = os->cost[os->cur ^ 1u].p;
        o.n_rays = p->n_rays;
        o.n_chunks = n_chunks;
        static const uint32_t hot = [] {  // A/B knob: hoist only the chunks of long rays
            const char* e = std::getenv("TT_ORDER_HOT");
            return e ? (uint32_t)std::atoi(e) : 0u;
        }();
        o.hot = hot;
        o.order = os->order.p;
        TT_HIP(c, tt_launch_order(o, c->stream));
        a.order = os->order.p;
    }
    TT_HIP(c, tt_launch_trace(a, want_stats, matcheck, info_mode, grid, c->stream));
    note_stream_launch(c->stream);
    if (os) {
        os->cur ^= 1u;
        os->valid = true;
        os->n_chunks = n_chunks;
    }
    c->ctl_zero[ci ^ 1u] = true;
    c->ctl_cur = ci ^ 1u;
    if (ring) TT_HIP(c, hipEventRecord(c->ring1[slot], c->stream));
    sr.end();
    if (ring) {
        c->ring_n++;
        c->ev0 = c->ring0[slot];
        c->ev1 = c->ring1[slot];
    }
    if (async) return TT_OK;
    TraceControl ctl;
    TT_HIP(c, hipMemcpyAsync(&ctl, c->ctl + ci, sizeof(ctl), hipMemcpyDeviceToHost, c->stream));
    if (!dev) {
        TT_HIP(c, hipMemcpyAsync(rays + off, d_rays + off, sizeof(tt_ray_data) * p->n_rays, hipMemcpyDeviceToHost, c->stream));
        if (info) TT_HIP(c, hipMemcpyAsync(info, d_info, sizeof(uint32_t) * 4 * wh, hipMemcpyDeviceToHost, c->stream));
    }
    TT_HIP(c, hipStreamSynchronize(c->stream));
    float ms = 0.0f;
    TT_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (stats) {
        stats->kernel_ms = ms;
        if (want_stats) {
            stats->rays = ctl.stats[0];
            stats->node_visits = ctl.stats[1];
            stats->tri_tests = ctl.stats[2];
            stats->blas_entries = ctl.stats[3];
            stats->hits = ctl.stats[4];
            stats->reps_exhausted = ctl.stats[5];
            stats->stack_overflows = ctl.stats[6];
            stats->accepts = ctl.stats[7];
            for (int k = 0; k < 8; k++) c->last_diag[k] = ctl.diag[k];
        }
        stats->stack_overflows = std::max<uint64_t>(stats->stack_overflows, ctl.err_overflow);
    }
    if (ctl.err_overflow)
        return fail(c, TT_ERR_STACK_OVERFLOW, "%u rays needed more than %d traversal stack entries", ctl.err_overflow,
                    TT_STACK_SIZE);
    return TT_OK;
}

extern "C" {

tt_status tt_trace_chunk_costs(tt_ctx* c, int32_t bounce, uint32_t* costs, uint32_t max, uint32_t* n) {
    if (!c || !n || (max && !costs) || bounce < 0) return TT_ERR_INVALID_ARG;
    *n = 0;
    const tt_ctx::OrderSlot& os = c->ord[std::min(bounce, 7)];
    if (!os.valid) return TT_OK;
    TT_HIP(c, hipSetDevice(c->device));
    const uint32_t k = std::min(os.n_chunks, max);
    if (k) TT_HIP(c, hipMemcpyAsync(costs, os.cost[os.cur].p, sizeof(uint32_t) * k, hipMemcpyDeviceToHost, c->stream));
    TT_HIP(c, hipStreamSynchronize(c->stream));
    *n = k;
    return TT_OK;
}

tt_status tt_trace_closest(tt_ctx* c, const tt_trace_params* p, tt_ray_data* rays, uint32_t* info,
                           const tt_col_data* colors, tt_stats* stats) {
    return trace_closest_call(c, p, nullptr, rays, info, colors, stats);
}

tt_status tt_trace_closest_hits(tt_ctx* c, const tt_trace_params* p, tt_ray_data* rays, uint32_t* info,
                                const tt_col_data* colors, uint32_t* hits_out) {
    if (!hits_out) return c ? fail(c, TT_ERR_INVALID_ARG, "null hits_out") : TT_ERR_INVALID_ARG;
    return trace_closest_call(c, p, nullptr, rays, info, colors, nullptr, hits_out);
}

tt_status tt_trace_closest_indirect(tt_ctx* c, const tt_trace_params* p, const uint32_t* n_rays_dev, tt_ray_data* rays,
                                    uint32_t* info, const tt_col_data* colors) {
    if (!n_rays_dev) return c ? fail(c, TT_ERR_INVALID_ARG, "null device ray count") : TT_ERR_INVALID_ARG;
    return trace_closest_call(c, p, n_rays_dev, rays, info, colors, nullptr);
}

}  // extern "C"

// full = false: tt_trace_shadow's contract (Direct at bounce 0 + NEEPosA only, the caller does the
// rest); full = true: tt_trace_shadow_ex's (plus CacheBuffer / Indirect / PrimaryNEERay)
static tt_status shadow_call(tt_ctx* c, const tt_shadow_params* p, tt_shadow_ray* rays, float* visibility,
                             tt_col_data* colors, float* nee_pos, tt_cache_data* cache, tt_stats* stats, bool full,
                             const uint32_t* n_dev = nullptr) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!p || !rays) return fail(c, TT_ERR_INVALID_ARG, "null params or shadow rays");
    if (p->screen_width == 0 || p->screen_height == 0) return fail(c, TT_ERR_INVALID_ARG, "zero screen size");
    if (p->bounce < 0) return fail(c, TT_ERR_INVALID_ARG, "negative bounce");
    if (c->any_atlas_shadow && !c->tex.p)
        return fail(c, TT_ERR_UNSUPPORTED,
                    "scene has glass (specTrans == 1) materials but no texture atlas was uploaded "
                    "(tt_scene_upload_texture_atlas; the shadow tint samples it, CommonData.cginc:618-625)");
    if (c->any_cutout && !c->atlas.p)
        return fail(c, TT_ERR_UNSUPPORTED,
                    "scene has Cutout materials but no alpha atlas was uploaded (tt_scene_upload_alpha_atlas)");
    const uint64_t wh = (uint64_t)p->screen_width * p->screen_height;
    if (wh > 0x7fffffffull) return fail(c, TT_ERR_INVALID_ARG, "screen too large");
    const bool dev = (p->flags & TT_TRACE_DEVICE_PTRS) != 0;
    const bool async = dev && ((p->flags & TT_TRACE_ASYNC) || n_dev);
    const bool want_stats = (p->flags & TT_TRACE_STATS) != 0;
    if (n_dev) {
        if (!dev) return fail(c, TT_ERR_INVALID_ARG, "a device-resident ray count needs TT_TRACE_DEVICE_PTRS");
        if (want_stats) return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_STATS needs a host ray count");
        if (!is_device_ptr(n_dev)) return fail(c, TT_ERR_INVALID_ARG, "the ray count pointer is not device memory");
    }
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if (p->n_rays == 0) return TT_OK;
    if (reinterpret_cast<uintptr_t>(rays) % 16 || (visibility && reinterpret_cast<uintptr_t>(visibility) % 16) ||
        (nee_pos && reinterpret_cast<uintptr_t>(nee_pos) % 16))
        return fail(c, TT_ERR_INVALID_ARG, "shadow rays / visibility / NEEPosA must be 16-byte aligned");
    TT_HIP(c, hipSetDevice(c->device));
    tt_shadow_ray* d_rays = rays;
    float4* d_vis = reinterpret_cast<float4*>(visibility);
    tt_col_data* d_col = colors;
    float4* d_nee = reinterpret_cast<float4*>(nee_pos);
    tt_cache_data* d_cache = cache;
    if (dev) {
        if (!is_device_ptr(rays)) return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_DEVICE_PTRS set but rays is not device memory");
    } else {
        if (cache) {
            if (c->st_cache.n < wh) TT_HIP(c, c->st_cache.alloc(wh));
            d_cache = c->st_cache.p;
            TT_HIP(c, hipMemcpyAsync(d_cache, cache, sizeof(tt_cache_data) * wh, hipMemcpyHostToDevice, c->stream));
        }
        if (c->st_shadow.n < p->n_rays) TT_HIP(c, c->st_shadow.alloc(p->n_rays));
        d_rays = c->st_shadow.p;
        TT_HIP(c, hipMemcpyAsync(d_rays, rays, sizeof(tt_shadow_ray) * p->n_rays, hipMemcpyHostToDevice, c->stream));
        if (visibility) {
            if (c->st_vis.n < p->n_rays) TT_HIP(c, c->st_vis.alloc(p->n_rays));
            d_vis = c->st_vis.p;
        }
        if (colors) {
            if (c->st_colors.n < wh) TT_HIP(c, c->st_colors.alloc(wh));
            d_col = c->st_colors.p;
            TT_HIP(c, hipMemcpyAsync(d_col, colors, sizeof(tt_col_data) * wh, hipMemcpyHostToDevice, c->stream));
        }
        if (nee_pos) {
            if (c->st_nee.n < wh) TT_HIP(c, c->st_nee.alloc(wh));
            d_nee = c->st_nee.p;
            TT_HIP(c, hipMemcpyAsync(d_nee, nee_pos, sizeof(float4) * wh, hipMemcpyHostToDevice, c->stream));
        }
    }
    // the accumulations beyond Direct / NEEPosA run in a second pass that reads the visibility
    // records: give the traversal one when the caller passed none
    const bool vis_check = (p->flags & TT_SHADOW_VISIBILITY_CHECK) != 0;
    const bool accumulate = full && !vis_check && (d_col || d_cache);
    if (accumulate && !d_vis) {
        if (c->st_vis.n < p->n_rays) TT_HIP(c, c->st_vis.alloc(p->n_rays));
        d_vis = c->st_vis.p;
    }
    ShadowArgs a;
    std::memset(&a, 0, sizeof(a));
    a.nodes = kernel_nodes(c);
    a.n_nodes = c->n_nodes_dev;  // (the overlay regions included: a frame-slot TLAS lives there)
    a.tlas_base = c->tlas_base;
    a.tris = c->tris.p;
    a.n_tris = c->host.n_tris;
    a.tlas = c->tlas.p;
    a.mesh = c->mesh.p;
    a.leaf = c->leaf.p;
    a.mat_tag = c->mat_tag.p;
    a.n_mat = c->host.n_mat;
    a.mat = mat_view(c);
    a.rays = d_rays;
    a.visibility = d_vis;
    a.colors = d_col;
    a.nee_pos = d_nee;
    a.cache = d_cache;
    a.ctl = c->ctl + c->ctl_cur;
    a.sticky_overflow = c->sticky;
    a.spill = c->spill.p;
    a.n_rays = p->n_rays;
    a.n_rays_dev = n_dev;
    a.width = p->screen_width;
    a.height = p->screen_height;
    a.bounce = p->bounce;
    a.flags = p->flags;
    const bool matcheck = c->any_shadow_skip || c->any_cutout || c->any_atlas_shadow;
    const uint32_t wpb = std::max(1u, tt_trace_block_size() / 64u);  // waves per block
    const uint32_t blocks_needed = ((p->n_rays + tt_trace_chunk_rays() - 1u) / tt_trace_chunk_rays() + wpb - 1u) / wpb;
    const uint32_t grid =
        std::max(1u, std::min(c->shadow_grid_of[(want_stats ? 2 : 0) + (matcheck ? 1 : 0)], blocks_needed));
    TT_HIP(c, hipMemsetAsync(c->ctl + c->ctl_cur, 0, sizeof(TraceControl), c->stream));
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    const uint32_t slot = c->ring_n % TT_RING;
    const bool ring = c->timing || !async;  // (a synchronous call reports its kernel time)
    if (ring) TT_HIP(c, hipEventRecord(c->ring0[slot], c->stream));
    c->ctl_zero[0] = c->ctl_zero[1] = false;  // the any-hit kernel zeroes nothing
    TT_HIP(c, tt_launch_shadow(&a, grid, c->stream, want_stats ? 1 : 0, matcheck ? 1 : 0));
    note_stream_launch(c->stream);
    if (ring) TT_HIP(c, hipEventRecord(c->ring1[slot], c->stream));
    if (accumulate) TT_HIP(c, tt_launch_shadow_accumulate(&a, d_vis, c->stream));
    sr.end();
    if (ring) {
        c->ring_n++;
        c->ev0 = c->ring0[slot];
        c->ev1 = c->ring1[slot];
    }
    if (async) return TT_OK;
    TraceControl ctl;
    TT_HIP(c, hipMemcpyAsync(&ctl, c->ctl + c->ctl_cur, sizeof(ctl), hipMemcpyDeviceToHost, c->stream));
    if (!dev) {
        TT_HIP(c, hipMemcpyAsync(rays, d_rays, sizeof(tt_shadow_ray) * p->n_rays, hipMemcpyDeviceToHost, c->stream));
        if (visibility)
            TT_HIP(c, hipMemcpyAsync(visibility, d_vis, sizeof(float4) * p->n_rays, hipMemcpyDeviceToHost, c->stream));
        if (colors) TT_HIP(c, hipMemcpyAsync(colors, d_col, sizeof(tt_col_data) * wh, hipMemcpyDeviceToHost, c->stream));
        if (nee_pos) TT_HIP(c, hipMemcpyAsync(nee_pos, d_nee, sizeof(float4) * wh, hipMemcpyDeviceToHost, c->stream));
        if (cache) TT_HIP(c, hipMemcpyAsync(cache, d_cache, sizeof(tt_cache_data) * wh, hipMemcpyDeviceToHost, c->stream));
    }
    TT_HIP(c, hipStreamSynchronize(c->stream));
    float ms = 0.0f;
    TT_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (stats) {
        stats->kernel_ms = ms;
        if (want_stats) {  // hits = occluded rays, accepts = rays that reached |t|
            stats->rays = ctl.stats[0];
            stats->node_visits = ctl.stats[1];
            stats->tri_tests = ctl.stats[2];
            stats->blas_entries = ctl.stats[3];
            stats->hits = ctl.stats[4];
            stats->reps_exhausted = ctl.stats[5];
            stats->stack_overflows = ctl.stats[6];
            stats->accepts = ctl.stats[7];
        }
        stats->stack_overflows = std::max<uint64_t>(stats->stack_overflows, ctl.err_overflow);
    }
    if (ctl.err_overflow)
        return fail(c, TT_ERR_STACK_OVERFLOW, "%u shadow rays needed more than %d traversal stack entries",
                    ctl.err_overflow, TT_STACK_SIZE);
    return TT_OK;
}

extern "C" {

tt_status tt_trace_shadow(tt_ctx* c, const tt_shadow_params* p, tt_shadow_ray* rays, float* visibility,
                          tt_col_data* colors, float* nee_pos, tt_stats* stats) {
    return shadow_call(c, p, rays, visibility, colors, nee_pos, nullptr, stats, false);
}

tt_status tt_trace_shadow_ex(tt_ctx* c, const tt_shadow_params* p, tt_shadow_ray* rays, float* visibility,
                             tt_col_data* colors, float* nee_pos, tt_cache_data* cache, tt_stats* stats) {
    return shadow_call(c, p, rays, visibility, colors, nee_pos, cache, stats, true);
}

tt_status tt_trace_shadow_ex_indirect(tt_ctx* c, const tt_shadow_params* p, const uint32_t* n_rays_dev,
                                      tt_shadow_ray* rays, float* visibility, tt_col_data* colors, float* nee_pos,
                                      tt_cache_data* cache) {
    if (!n_rays_dev) return c ? fail(c, TT_ERR_INVALID_ARG, "null device ray count") : TT_ERR_INVALID_ARG;
    return shadow_call(c, p, rays, visibility, colors, nee_pos, cache, nullptr, true, n_rays_dev);
}

tt_status tt_resolve_normals(tt_ctx* c, const tt_trace_params* p, const tt_ray_data* rays, float* normals6) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!p || !rays || !normals6) return fail(c, TT_ERR_INVALID_ARG, "null argument");
    const uint64_t wh = (uint64_t)p->screen_width * p->screen_height;
    const uint32_t off = (p->bounce % 2 == 1) ? (uint32_t)wh : 0u;
    if (p->n_rays == 0) return TT_OK;
    TT_HIP(c, hipSetDevice(c->device));
    const bool dev = (p->flags & TT_TRACE_DEVICE_PTRS) != 0;
    const tt_ray_data* d_rays = rays;
    float* d_out = normals6;
    if (!dev) {
        const size_t ray_end = (size_t)off + p->n_rays;
        if (c->st_rays.n < ray_end) TT_HIP(c, c->st_rays.alloc(ray_end));
        TT_HIP(c, hipMemcpyAsync(c->st_rays.p + off, rays + off, sizeof(tt_ray_data) * p->n_rays, hipMemcpyHostToDevice, c->stream));
        d_rays = c->st_rays.p;
        if (c->st_normals.n < (size_t)6 * p->n_rays) TT_HIP(c, c->st_normals.alloc((size_t)6 * p->n_rays));
        d_out = c->st_normals.p;
    }
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    TT_HIP(c, tt_launch_resolve(d_rays, off, p->n_rays, p->far_plane, c->tris_raw.p, (uint32_t)c->tris_raw.n,
                                c->mesh_raw.p, (uint32_t)c->mesh_raw.n, d_out, c->stream));
    sr.end();
    if (!dev) TT_HIP(c, hipMemcpyAsync(normals6, d_out, sizeof(float) * 6 * p->n_rays, hipMemcpyDeviceToHost, c->stream));
    TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

tt_status tt_generate_primary(tt_ctx* c, const tt_camera* cam, tt_ray_data* rays) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    if (!cam || !rays || !cam->width || !cam->height) return fail(c, TT_ERR_INVALID_ARG, "bad camera or rays");
    const uint64_t wh = (uint64_t)cam->width * cam->height;
    if (wh > 0x7fffffffull) return fail(c, TT_ERR_INVALID_ARG, "screen too large");
    TT_HIP(c, hipSetDevice(c->device));
    const bool dev = (cam->flags & TT_TRACE_DEVICE_PTRS) != 0;
    // TT_TRACE_ASYNC with device rays: nothing waits (the camera goes in the kernel arguments)
    const bool async = dev && (cam->flags & TT_TRACE_ASYNC);
    tt_ray_data* d = rays;
    if (!dev) {
        if (c->st_rays.n < wh) TT_HIP(c, c->st_rays.alloc(wh));
        d = c->st_rays.p;
    } else if (!is_device_ptr(rays)) {
        return fail(c, TT_ERR_INVALID_ARG, "TT_TRACE_DEVICE_PTRS set but rays is not device memory");
    }
    uint32_t slot;
    TT_HIP(c, ring_open(c, slot));
    TT_HIP(c, tt_launch_generate(cam->cam_to_world, cam->cam_inv_proj, cam->width, cam->height, cam->near_plane, cam->far_plane,
                                 cam->jitter, cam->frames_accumulated, cam->max_bounce, d, c->stream));
    note_stream_launch(c->stream);
    TT_HIP(c, ring_close(c, slot));
    if (!dev) TT_HIP(c, hipMemcpyAsync(rays, d, sizeof(tt_ray_data) * wh, hipMemcpyDeviceToHost, c->stream));
    if (!async) TT_HIP(c, hipStreamSynchronize(c->stream));
    return TT_OK;
}

}  // extern "C"

// n_dev (nullable): device-resident count of the rays traced at p->bounce (p->n_rays = capacity);
// n_next_dev (nullable): the survivor count is written there on the device and the call returns
// without synchronizing (n_next may then be null).
static tt_status enqueue_call(tt_ctx* c, const tt_trace_params* p, const uint32_t* n_dev, tt_ray_data* rays,
                              int32_t frames, int32_t max_bounce, uint32_t* n_next, uint32_t* n_next_dev) {
    if (!c) return TT_ERR_INVALID_ARG;
    TT_REFUSE_DEAD_STREAM(c);
    if (!c->has_scene) return fail(c, TT_ERR_NO_SCENE, "no scene uploaded");
    if (!p || !rays || (!n_next && !n_next_dev)) return fail(c, TT_ERR_INVALID_ARG, "null argument");
    const uint64_t wh = (uint64_t)p->screen_width * p->screen_height;
    if (!wh || wh > 0x7fffffffull || p->n_rays > wh) return fail(c, TT_ERR_INVALID_ARG, "bad ray count / screen");
    const uint32_t src = (p->bounce % 2 == 1) ? (uint32_t)wh : 0u, dst = (p->bounce % 2 == 1) ? 0u : (uint32_t)wh;
    const bool dev = (p->flags & TT_TRACE_DEVICE_PTRS) != 0;
    if (n_dev || n_next_dev) {
        if (!dev) return fail(c, TT_ERR_INVALID_ARG, "device-resident ray counts need TT_TRACE_DEVICE_PTRS");
        if ((n_dev && !is_device_ptr(n_dev)) || (n_next_dev && !is_device_ptr(n_next_dev)))
            return fail(c, TT_ERR_INVALID_ARG, "a ray count pointer is not device memory");
    }
    TT_HIP(c, hipSetDevice(c->device));
    // [0] survivor count, [1] tile ticket, [2..3] pad, then one 64-bit look-back word per tile
    // two counter blocks, used in turn: each enqueue zeroes the other block for the next one (no fill
    // between enqueues); a larger capacity reallocates and fills both
    const size_t ctl_words = 4 + 2 * (size_t)tt_bounce_tiles(p->n_rays);
    if (c->counter_words < ctl_words) {
        TT_HIP(c, hipStreamSynchronize(c->stream));  // (the old blocks may be in use)
        c->counter.release();
        TT_HIP(c, c->counter.alloc(2 * ctl_words));
        TT_HIP(c, hipMemsetAsync(c->counter.p, 0, 2 * 4 * ctl_words, c->stream));
        c->counter_words = (uint32_t)ctl_words;
        c->counter_cur = 0;
    }
    uint32_t* const ctl_cur = c->counter.p + (size_t)c->counter_cur * c->counter_words;
    uint32_t* const ctl_next = c->counter.p + (size_t)(c->counter_cur ^ 1u) * c->counter_words;
    tt_ray_data* d = rays;
    if (!dev) {
        if (c->st_rays.n < 2 * wh) {
            // keep nothing: the host copy is the source of truth for host-pointer calls
            TT_HIP(c, c->st_rays.alloc(2 * wh));
        }
        d = c->st_rays.p;
        TT_HIP(c, hipMemcpyAsync(d + src, rays + src, sizeof(tt_ray_data) * p->n_rays, hipMemcpyHostToDevice, c->stream));
    }
    uint32_t slot;
    SceneRead sr(c);
    TT_HIP(c, sr.err);
    TT_HIP(c, ring_open(c, slot));
    TT_HIP(c, tt_launch_bounce(d, src, dst, p->n_rays, p->far_plane, p->bounce, frames, max_bounce, c->tris_raw.p,
                               c->mesh_raw.p, ctl_cur, c->stream, n_dev, n_next_dev, ctl_next, c->counter_words,
                               c->frame_pixels));
    c->counter_cur ^= 1u;
    TT_HIP(c, ring_close(c, slot));
    sr.end();
    if (n_next_dev) {  // BufferSizes[CurBounce + 1].tracerays stays on the GPU: no host round trip
        if (n_next) *n_next = 0;
        return TT_OK;
    }
    uint32_t cnt = 0;
    TT_HIP(c, hipMemcpyAsync(&cnt, ctl_cur, 4, hipMemcpyDeviceToHost, c->stream));
    TT_HIP(c, hipStreamSynchronize(c->stream));
    if (!dev && cnt) {
        TT_HIP(c, hipMemcpy(rays + dst, d + dst, sizeof(tt_ray_data) * cnt, hipMemcpyDeviceToHost));
    }
    *n_next = cnt;
    return TT_OK;
}

extern "C" {

tt_status tt_enqueue_diffuse_bounce(tt_ctx* c, const tt_trace_params* p, tt_ray_data* rays, int32_t frames,
                                    int32_t max_bounce, uint32_t* n_next) {
    if (c && !n_next) return fail(c, TT_ERR_INVALID_ARG, "null argument");
    return enqueue_call(c, p, nullptr, rays, frames, max_bounce, n_next, nullptr);
}

tt_status tt_enqueue_diffuse_bounce_indirect(tt_ctx* c, const tt_trace_params* p, const uint32_t* n_rays_dev,
                                             tt_ray_data* rays, int32_t frames, int32_t max_bounce,
                                             uint32_t* n_next_dev) {
    if (!n_next_dev) return c ? fail(c, TT_ERR_INVALID_ARG, "null device survivor count") : TT_ERR_INVALID_ARG;
    return enqueue_call(c, p, n_rays_dev, rays, frames, max_bounce, nullptr, n_next_dev);
}

}  // extern "C"
