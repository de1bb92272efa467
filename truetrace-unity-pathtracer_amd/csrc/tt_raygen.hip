// tt_raygen.hip — the producers either side of the trace dispatch:
//  * tt_generate_kernel: Generate + CreateCameraRay (RayGenKernels.compute:40-57,
//    CommonData.cginc:511-567, UseDoF off) writing RayData into GlobalRays[pixel];
//  * tt_bounce_kernel: the diffuse-lobe subset of kernel_shade's next-ray enqueue
//    (RayTracingShader.compute:52-84, 99-122, 293, 498-506): hit point, unsmoothed normal
//    offset, cosine-hemisphere direction in GetTangentSpace(norm), then compaction of the
//    survivors into the other half of the ping-pong buffer. The reference appends with one
//    InterlockedAdd per ray on one counter (RayTracingShader.compute:500), so its order is
//    whatever the atomics serialise to; one atomic per wave on one word still serialised at
//    ~88 per microsecond (375 us for a 1080p frame, profiles/r02/r02a_kernel_stats.csv). Here
//    the compaction is a STABLE single-pass scan: 4096-ray tiles taken in ticket order, a block
//    ballot/LDS prefix inside the tile and a decoupled look-back over the preceding tiles'
//    published counts (one 64-bit status word per tile, flag and value together), so the
//    survivors land in source order -- deterministic, and the oracle restates the same order.
//  * sincos in the cosine-lobe sample is pinned (sincos_pinned): HLSL leaves its precision to
//    the driver, so both sides evaluate the same float polynomials with explicit FMAs.
#include "tt_device.h"

namespace {

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

__device__ __forceinline__ float3 normalize3(float3 v) {
    const float inv = 1.0f / sqrtf(fma_(v.z, v.z, fma_(v.y, v.y, v.x * v.x)));
    return make_float3(v.x * inv, v.y * inv, v.z * inv);
}
__device__ __forceinline__ float3 cross3(float3 a, float3 b) {
    return make_float3(fma_(a.y, b.z, -(a.z * b.y)), fma_(a.z, b.x, -(a.x * b.z)), fma_(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float dot3(float3 a, float3 b) { return fma_(a.z, b.z, fma_(a.y, b.y, a.x * b.x)); }

// pcg_hash / hash_with / random() (non-ASVGF branch) — CommonData.cginc:374-389, :413-426
__device__ __forceinline__ uint32_t pcg_hash(uint32_t seed) {
    const uint32_t state = seed * 747796405u + 2891336453u;
    const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
__device__ __forceinline__ uint32_t hash_with(uint32_t seed, uint32_t hash) {
    seed = (seed ^ 61u) ^ hash;
    seed += seed << 3;
    seed ^= seed >> 4;
    seed *= 0x27d4eb2du;
    return seed;
}
__device__ __forceinline__ float2 random2(uint32_t samdim, uint32_t pixel_index, int32_t frames, int32_t max_bounce,
                                          int32_t cur_bounce) {
    const uint32_t hash = pcg_hash((pixel_index * 258u + samdim) * (uint32_t)(max_bounce + 1) + (uint32_t)cur_bounce);
    const float k = __uint_as_float(0x2f7fffffu);
    return make_float2((float)hash_with((uint32_t)frames, hash) * k, (float)hash_with((uint32_t)frames + 0xdeadbeefu, hash) * k);
}

__device__ __forceinline__ float3 i_octahedral_32(uint32_t data) {
    const uint32_t ix = data & 65535u, iy = (data >> 16) & 65535u;
    const float vx = (float)ix / 32767.5f - 1.0f, vy = (float)iy / 32767.5f - 1.0f;
    float3 nor = make_float3(vx, vy, 1.0f - fabsf(vx) - fabsf(vy));
    const float t = fmaxf(-nor.z, 0.0f);
    nor.x += (nor.x > 0.0f) ? -t : t;
    nor.y += (nor.y > 0.0f) ? -t : t;
    return normalize3(nor);
}
// octahedral_32 — CommonData.cginc:840-846 (round = round-half-even, DXIL Round_ne)
__device__ __forceinline__ uint32_t octahedral_32(float3 nor) {
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

__device__ __forceinline__ float3 mul_inv(const float* W, float3 x) {
    auto M = [&](int r, int c) { return W[c * 4 + r]; };
    return make_float3(fma_(M(2, 0), x.z, fma_(M(1, 0), x.y, M(0, 0) * x.x)),
                       fma_(M(2, 1), x.z, fma_(M(1, 1), x.y, M(0, 1) * x.x)),
                       fma_(M(2, 2), x.z, fma_(M(1, 2), x.y, M(0, 2) * x.x)));
}

// the camera travels in the kernel arguments (no staging copy per frame: a copy is one more small
// operation on the stream that waits for a free CU slot beside the persistent trace grids)
struct CamArgs {
    float c2w[16], ip[16];
};
// one camera ray of pixel (x, y) into *o (RayData, hits = (0, 0, asuint(FarPlane), 0))
__device__ __forceinline__ void generate_one(const CamArgs& cam, uint32_t x, uint32_t y, uint32_t width, uint32_t height,
                                             float near_plane, float far_plane, int32_t jitter, int32_t frames,
                                             int32_t max_bounce, uint4* o) {
    const uint32_t pixel_index = y * width + x;
    float jx = 0.0f, jy = 0.0f;
    if (jitter) {
        const float2 r = random2(0, pixel_index, frames, max_bounce, 0);
        jx = r.x - 0.5f;
        jy = r.y - 0.5f;
    }
    auto C = [&](int r, int c) { return cam.c2w[c * 4 + r]; };
    auto P = [&](int r, int c) { return cam.ip[c * 4 + r]; };
    const float uvx = ((float)x + jx) / (float)width * 2.0f - 1.0f;
    const float uvy = ((float)y + jy) / (float)height * 2.0f - 1.0f;
    const float3 origin = make_float3(C(0, 3), C(1, 3), C(2, 3));
    float3 d = make_float3(fma_(P(0, 1), uvy, P(0, 0) * uvx) + P(0, 3), fma_(P(1, 1), uvy, P(1, 0) * uvx) + P(1, 3),
                           fma_(P(2, 1), uvy, P(2, 0) * uvx) + P(2, 3));
    d = make_float3(fma_(C(0, 2), d.z, fma_(C(0, 1), d.y, C(0, 0) * d.x)),
                    fma_(C(1, 2), d.z, fma_(C(1, 1), d.y, C(1, 0) * d.x)),
                    fma_(C(2, 2), d.z, fma_(C(2, 1), d.y, C(2, 0) * d.x)));
    d = normalize3(d);
    o[0] = make_uint4(__float_as_uint(origin.x + near_plane * d.x), __float_as_uint(origin.y + near_plane * d.y),
                      __float_as_uint(origin.z + near_plane * d.z), pixel_index);
    o[1] = make_uint4(__float_as_uint(d.x), __float_as_uint(d.y), __float_as_uint(d.z), 0u);
    o[2] = make_uint4(0u, 0u, __float_as_uint(far_plane), 0u);
}

__global__ __launch_bounds__(256) void tt_generate_kernel(const CamArgs cam,
                                                          uint32_t width, uint32_t height, float near_plane,
                                                          float far_plane, int32_t jitter, int32_t frames,
                                                          int32_t max_bounce, tt_ray_data* __restrict__ rays) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= width || y >= height) return;
    generate_one(cam, x, y, width, height, near_plane, far_plane, jitter, frames, max_bounce,
                 reinterpret_cast<uint4*>(rays + y * width + x));
}

// The rays of a pixel list (a multi-GPU group member's screen tiles, tt_group_trace_frame) for `batch` frames:
// ray b n + i is pixel pixels[i]'s camera ray of frame b (frames_accumulated = frames + b), bit for bit the one
// tt_generate_kernel writes at GlobalRays[pixel] for that frame, with PixelIndex + b W H (frame b of a screen
// `batch` frames tall, tt_ctx_set_frame_pixels).
__global__ __launch_bounds__(256) void tt_generate_list_kernel(const CamArgs cam, const uint32_t* __restrict__ pixels,
                                                               uint32_t n, uint32_t batch, uint32_t width,
                                                               uint32_t height, float near_plane, float far_plane,
                                                               int32_t jitter, int32_t frames, int32_t max_bounce,
                                                               tt_ray_data* __restrict__ rays) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n * batch) return;
    const uint32_t b = r / n, p = pixels[r - b * n];
    uint4* o = reinterpret_cast<uint4*>(rays + r);
    generate_one(cam, p % width, p / width, width, height, near_plane, far_plane, jitter, frames + (int32_t)b,
                 max_bounce, o);
    if (b) o[0].w = p + b * width * height;
}

// sin/cos of the disc-sample angle phi in [-3pi/4, 3pi/4] (sample_disc's two branches give
// [-pi/4, pi/4] and [pi/4, 3pi/4]): cephes single-precision minimax polynomials on
// [-pi/4, pi/4] evaluated with explicit FMAs; |phi| > pi/4 is reduced by pi/2 (two-constant
// Cody-Waite). Pinned: oracle/tt_oracle.c sincos_pinned is the same sequence of operations.
__device__ __forceinline__ void sincos_pinned(float phi, float* s, float* c) {
    const bool big = fabsf(phi) > 0.785398185253143310546875f;
    const float q = phi > 0.0f ? 1.0f : -1.0f;
    const float r = big ? fma_(-q, -4.37113882867379e-8f, fma_(-q, 1.57079637050628662109375f, phi)) : phi;
    const float z = r * r;
    const float sp = fma_(fma_(fma_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
    const float cp = fma_(fma_(fma_(fma_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f), z,
                               -0.5f), z, 1.0f);
    // phi = q pi/2 + r: sin(phi) = q cos(r), cos(phi) = -q sin(r)
    *s = big ? q * cp : sp;
    *c = big ? -q * sp : cp;
}

// pdf > 0 decision and omega_o of sample(): cosine-weighted hemisphere from random(1, pixel)
// (RayTracingShader.compute:52-84)
__device__ __forceinline__ float3 cosine_sample(uint32_t pixel, int32_t frames, int32_t max_bounce, int32_t cur_bounce,
                                                float* pdf) {
    const float2 rnd = random2(1, pixel, frames, max_bounce, cur_bounce);
    float a = 2.0f * rnd.x - 1.0f, b = 2.0f * rnd.y - 1.0f;
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
    sincos_pinned(phi, &sp, &cp);
    const float dx = rr * cp, dz = rr * sp;
    const float3 om = make_float3(dx, sqrtf(fabsf(1.0f - (dx * dx + dz * dz))), dz);
    *pdf = om.y * 0.318309886548f;
    return om;
}

// The new ray of a surviving hit (kernel_shade's diffuse path, RayTracingShader.compute:99-122,
// 284, 293, 503).
// RayData as three 16-B words: (origin, PixelIndex), (direction, last_pdf), hits
struct Ray3 {
    uint4 a, b, h;
};
__device__ __forceinline__ void bounce_ray(const Ray3& R, float3 om, float pdf, const tt_cuda_triangle* tris,
                                           const tt_mesh_data* md, uint4* o) {
    const float t = __uint_as_float(R.h.z);
    const int32_t mesh_id = (int32_t)R.h.x, tri = (int32_t)R.h.y;
    const float u = (float)(R.h.w & 0xffffu) / 65535.0f, v = (float)(R.h.w >> 16) / 65535.0f;
    const float* W = md[mesh_id].W2L;
    const tt_cuda_triangle& T = tris[tri];
    const float3 dir = make_float3(__uint_as_float(R.b.x), __uint_as_float(R.b.y), __uint_as_float(R.b.z));
    const float3 org = make_float3(__uint_as_float(R.a.x), __uint_as_float(R.a.y), __uint_as_float(R.a.z));
    const float3 pos = make_float3(dir.x * t + org.x, dir.y * t + org.y, dir.z * t + org.z);
    // Geomnorm (GetTriangleNormal) and USGNorm (RayTracingShader.compute:111-118)
    const float3 n0 = i_octahedral_32(T.norms[0]), n1 = i_octahedral_32(T.norms[1]), n2 = i_octahedral_32(T.norms[2]);
    const float w0 = 1.0f - u - v;
    float3 g = mul_inv(W, make_float3(n0.x * w0 + u * n1.x + v * n2.x, n0.y * w0 + u * n1.y + v * n2.y,
                                      n0.z * w0 + u * n1.z + v * n2.z));
    g = normalize3(g);
    float3 us = mul_inv(W, cross3(normalize3(make_float3(T.posedge1[0], T.posedge1[1], T.posedge1[2])),
                                  normalize3(make_float3(T.posedge2[0], T.posedge2[1], T.posedge2[2]))));
    us = normalize3(us);
    us = make_float3(-us.x, -us.y, -us.z);
    if (dot3(us, g) < 0) us = make_float3(-us.x, -us.y, -us.z);
    if (dot3(dir, us) > 0.0f) {  // GotFlipped: backfacing
        us = make_float3(-us.x, -us.y, -us.z);
        g = make_float3(-g.x, -g.y, -g.z);
    }
    const float3 norm = i_octahedral_32(octahedral_32(g));
    // GetTangentSpace(norm) — CommonData.cginc:332-343 (helper (1,0,0), or (0,0,1) if |n.x| > 0.99)
    const float3 helper = fabsf(norm.x) > 0.99f ? make_float3(0, 0, 1) : make_float3(1, 0, 0);
    const float3 tangent = normalize3(cross3(norm, helper));
    const float3 binormal = cross3(norm, tangent);
    float3 nd = make_float3(om.x * tangent.x + om.y * norm.x + om.z * binormal.x,
                            om.x * tangent.y + om.y * norm.y + om.z * binormal.y,
                            om.x * tangent.z + om.y * norm.z + om.z * binormal.z);
    nd = normalize3(nd);
    o[0] = make_uint4(__float_as_uint(us.x * 0.0001f + pos.x), __float_as_uint(us.y * 0.0001f + pos.y),
                      __float_as_uint(us.z * 0.0001f + pos.z), R.a.w);
    o[1] = make_uint4(__float_as_uint(nd.x), __float_as_uint(nd.y), __float_as_uint(nd.z), __float_as_uint(pdf));
    o[2] = R.h;
}

// Decoupled look-back status word of a tile: bits 0-31 the count, bit 32 "aggregate" (this
// tile's own survivors), bit 33 "inclusive" (survivors of tiles [0, tile]); 0 = not yet published.
// Flag and value travel in one 64-bit word, so relaxed device-scope atomics suffice (no fences).
constexpr uint64_t TT_LB_AGG = 1ull << 32, TT_LB_INC = 2ull << 32;
__device__ __forceinline__ void lb_publish(unsigned long long* st, uint32_t tile, uint64_t flag, uint32_t v) {
    __hip_atomic_store(st + tile, (unsigned long long)(flag | v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Exclusive prefix of tile `tile` (> 0): one wave reads the 64 preceding status words at once
// (lane k reads tile - 1 - k), waits until all are published, sums up to and including the
// nearest inclusive one, and slides the window back when there is none.
__device__ __forceinline__ uint32_t lb_lookback(unsigned long long* st, uint32_t tile, uint32_t lane) {
    uint32_t prefix = 0;
    int32_t j = (int32_t)tile - 1;
    while (true) {
        const int32_t idx = j - (int32_t)lane;
        uint64_t w = TT_LB_INC;  // before tile 0: an inclusive zero
        if (idx >= 0) {
            do {
                w = __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((w >> 32) == 0u);
        }
        const uint64_t inc = __ballot((w & TT_LB_INC) != 0u);
        // lanes [0, first inclusive lane] contribute; none inclusive -> all 64, then slide
        const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 63u;
        uint32_t v = lane <= stop ? (uint32_t)w : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        prefix += v;
        if (inc) return prefix;
        j -= 64;
    }
}

constexpr uint32_t TT_BOUNCE_K = 4;                          // rays per thread
constexpr uint32_t TT_BOUNCE_BLOCK = 1024;                   // threads per tile (16 waves)
constexpr uint32_t TT_BOUNCE_WAVES = TT_BOUNCE_BLOCK / 64;
constexpr uint32_t TT_BOUNCE_TILE = TT_BOUNCE_BLOCK * TT_BOUNCE_K;  // 4096 rays per tile: few tickets, short look-backs

__global__ __launch_bounds__(TT_BOUNCE_BLOCK) void tt_bounce_kernel(tt_ray_data* __restrict__ rays, uint32_t src_off, uint32_t dst_off,
                                                        uint32_t n, float far_plane, int32_t cur_bounce, int32_t frames,
                                                        int32_t max_bounce, const tt_cuda_triangle* __restrict__ tris,
                                                        const tt_mesh_data* __restrict__ md, uint32_t* __restrict__ ctl,
                                                        unsigned long long* __restrict__ lb, uint32_t n_tiles,
                                                        const uint32_t* __restrict__ n_dev, uint32_t* __restrict__ n_next_dev,
                                                        uint32_t* __restrict__ ctl_next, uint32_t ctl_next_words,
                                                        uint32_t frame_pixels) {
    __shared__ uint32_t s_tile, s_prefix;
    __shared__ uint32_t s_cnt[TT_BOUNCE_K][TT_BOUNCE_WAVES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    // the next enqueue on this stream uses the other counter block: zero it now (plain vector stores; it
    // starts after this launch completes), so no fill kernel runs between enqueues
    if (ctl_next)
        for (uint32_t w = blockIdx.x * TT_BOUNCE_BLOCK + tid; w < ctl_next_words; w += gridDim.x * TT_BOUNCE_BLOCK)
            ctl_next[w] = 0u;
    if (tid == 0) s_tile = atomicAdd(&ctl[1], 1u);  // tiles in ticket order: look-back never waits on an unstarted block
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * TT_BOUNCE_TILE;
    // device-resident count (the reference's BufferSizes[CurBounce].tracerays): tiles past it find no
    // rays, publish 0 and keep the look-back chain complete up to the grid's last tile
    if (n_dev) n = min(*n_dev, n);
    // pass 1: which rays survive (hit, and the cosine sample's pdf > 0); keep the ray and omega_o
    Ray3 R[TT_BOUNCE_K];
    float3 om[TT_BOUNCE_K];
    float pdf[TT_BOUNCE_K];
    uint64_t live[TT_BOUNCE_K];
#pragma unroll
    for (uint32_t k = 0; k < TT_BOUNCE_K; k++) {
        const uint32_t i = base + k * TT_BOUNCE_BLOCK + tid;
        bool ok = false;
        if (i < n) {
            const uint4* rp = reinterpret_cast<const uint4*>(rays + src_off + i);
            R[k].a = rp[0];
            R[k].b = rp[1];
            R[k].h = rp[2];
            const float t = __uint_as_float(R[k].h.z);
            if (t < far_plane && (int32_t)R[k].h.y >= 0) {
                // batched frames (tt_ctx_set_frame_pixels): PixelIndex p is pixel p mod n of frame p / n, whose
                // random numbers are that pixel's at frames + p / n; 0: PixelIndex as-is (the reference's form)
                uint32_t px = R[k].a.w;
                int32_t fr = frames;
                if (frame_pixels) {
                    const uint32_t j = px / frame_pixels;
                    px -= j * frame_pixels;
                    fr += (int32_t)j;
                }
                om[k] = cosine_sample(px, fr, max_bounce, cur_bounce, &pdf[k]);
                ok = pdf[k] > 0.0f;
            }
        }
        live[k] = __ballot(ok);
        if (lane == 0) s_cnt[k][wave] = (uint32_t)__popcll(live[k]);
    }
    __syncthreads();
    // tile count, published before the look-back so successors can sum past this tile
    if (wave == 0) {
        uint32_t total = 0;
#pragma unroll
        for (uint32_t k = 0; k < TT_BOUNCE_K; k++)
            for (uint32_t w = 0; w < TT_BOUNCE_WAVES; w++) total += s_cnt[k][w];
        uint32_t prefix = 0;
        if (tile == 0) {
            if (lane == 0) lb_publish(lb, 0, TT_LB_INC, total);
        } else {
            if (lane == 0) lb_publish(lb, tile, TT_LB_AGG, total);
            prefix = lb_lookback(lb, tile, lane);
            if (lane == 0) lb_publish(lb, tile, TT_LB_INC, prefix + total);
        }
        if (lane == 0) {
            s_prefix = prefix;
            if (tile == n_tiles - 1u) {
                ctl[0] = prefix + total;  // the survivor count tt_enqueue returns
                if (n_next_dev) *n_next_dev = prefix + total;  // BufferSizes[CurBounce + 1].tracerays
            }
        }
    }
    __syncthreads();
    // pass 2: survivors in source order (k-major, then thread) at prefix + rank
    uint32_t slot = s_prefix;
#pragma unroll
    for (uint32_t k = 0; k < TT_BOUNCE_K; k++) {
        uint32_t before = 0, all = 0;
        for (uint32_t w = 0; w < TT_BOUNCE_WAVES; w++) {
            before += w < wave ? s_cnt[k][w] : 0u;
            all += s_cnt[k][w];
        }
        if ((live[k] >> lane) & 1ull) {
            const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(live[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live[k], 0u));
            bounce_ray(R[k], om[k], pdf[k], tris, md, reinterpret_cast<uint4*>(rays + dst_off + slot + before + pre));
        }
        slot += all;
    }
}

}  // namespace

// c2w, ip: HOST arrays (column-major 4x4 each), copied into the kernel arguments
hipError_t tt_launch_generate(const float* c2w, const float* ip, uint32_t w, uint32_t h, float near_plane, float far_plane,
                              int32_t jitter, int32_t frames, int32_t max_bounce, tt_ray_data* rays, hipStream_t st) {
    CamArgs cam;
    for (int i = 0; i < 16; i++) {
        cam.c2w[i] = c2w[i];
        cam.ip[i] = ip[i];
    }
    hipLaunchKernelGGL(tt_generate_kernel, dim3((w + 255u) / 256u, h), dim3(256), 0, st, cam, w, h, near_plane, far_plane,
                       jitter, frames, max_bounce, rays);
    return hipGetLastError();
}

// pixels: DEVICE array of n pixel indices < w * h (the caller checked them)
hipError_t tt_launch_generate_list(const float* c2w, const float* ip, const uint32_t* pixels, uint32_t n,
                                   uint32_t batch, uint32_t w, uint32_t h, float near_plane, float far_plane,
                                   int32_t jitter, int32_t frames, int32_t max_bounce, tt_ray_data* rays,
                                   hipStream_t st) {
    if (n == 0 || batch == 0) return hipSuccess;
    CamArgs cam;
    for (int i = 0; i < 16; i++) {
        cam.c2w[i] = c2w[i];
        cam.ip[i] = ip[i];
    }
    hipLaunchKernelGGL(tt_generate_list_kernel, dim3((n * batch + 255u) / 256u), dim3(256), 0, st, cam, pixels, n,
                       batch, w, h, near_plane, far_plane, jitter, frames, max_bounce, rays);
    return hipGetLastError();
}

uint32_t tt_bounce_tiles(uint32_t n) { return (n + TT_BOUNCE_TILE - 1u) / TT_BOUNCE_TILE; }

// counter: [0] survivor count, [1] tile ticket, then tt_bounce_tiles(n) 64-bit status words; all
// zero at the launch (the caller's fill, or the previous launch's ctl_next). ctl_next (nullable): the
// ctl_next_words words this launch zeroes for the next one.
// n_dev (nullable): device-resident ray count, clamped to n (then n is the capacity the grid covers);
// n_next_dev (nullable): receives the survivor count on the device.
hipError_t tt_launch_bounce(tt_ray_data* rays, uint32_t src_off, uint32_t dst_off, uint32_t n, float far_plane,
                            int32_t cur_bounce, int32_t frames, int32_t max_bounce, const tt_cuda_triangle* tris,
                            const tt_mesh_data* md, uint32_t* counter, hipStream_t st, const uint32_t* n_dev,
                            uint32_t* n_next_dev, uint32_t* ctl_next, uint32_t ctl_next_words,
                            uint32_t frame_pixels) {
    if (n == 0) {
        if (ctl_next) {  // (this block stays zero: the next launch's block is the caller's to fill)
            const hipError_t e = hipMemsetAsync(ctl_next, 0, 4 * (size_t)ctl_next_words, st);
            if (e != hipSuccess) return e;
        }
        if (n_next_dev) return hipMemsetAsync(n_next_dev, 0, 4, st);
        return hipSuccess;
    }
    const uint32_t tiles = tt_bounce_tiles(n);
    hipLaunchKernelGGL(tt_bounce_kernel, dim3(tiles), dim3(TT_BOUNCE_BLOCK), 0, st, rays, src_off, dst_off, n, far_plane,
                       cur_bounce, frames, max_bounce, tris, md, counter,
                       reinterpret_cast<unsigned long long*>(counter + 4), tiles, n_dev, n_next_dev, ctl_next,
                       ctl_next_words, frame_pixels);
    return hipGetLastError();
}
