// tt_raygen.hip — the producers either side of the trace dispatch:
//  * tt_generate_kernel: Generate + CreateCameraRay (RayGenKernels.compute:40-57,
//    CommonData.cginc:511-567, UseDoF off) writing RayData into GlobalRays[pixel];
//  * tt_bounce_kernel: the diffuse-lobe subset of kernel_shade's next-ray enqueue
//    (RayTracingShader.compute:52-84, 99-122, 293, 498-506): hit point, unsmoothed normal
//    offset, cosine-hemisphere direction in GetTangentSpace(norm), then compaction of the
//    survivors into the other half of the ping-pong buffer. The reference appends with one
//    InterlockedAdd per ray; here a wave ballots its survivors, one lane reserves popcount
//    slots and every survivor writes at base + mbcnt prefix (one atomic per wave).
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

__global__ __launch_bounds__(256) void tt_generate_kernel(const float* __restrict__ c2w, const float* __restrict__ ip,
                                                          uint32_t width, uint32_t height, float near_plane,
                                                          float far_plane, int32_t jitter, int32_t frames,
                                                          int32_t max_bounce, tt_ray_data* __restrict__ rays) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= width || y >= height) return;
    const uint32_t pixel_index = y * width + x;
    float jx = 0.0f, jy = 0.0f;
    if (jitter) {
        const float2 r = random2(0, pixel_index, frames, max_bounce, 0);
        jx = r.x - 0.5f;
        jy = r.y - 0.5f;
    }
    auto C = [&](int r, int c) { return c2w[c * 4 + r]; };
    auto P = [&](int r, int c) { return ip[c * 4 + r]; };
    const float uvx = ((float)x + jx) / (float)width * 2.0f - 1.0f;
    const float uvy = ((float)y + jy) / (float)height * 2.0f - 1.0f;
    const float3 origin = make_float3(C(0, 3), C(1, 3), C(2, 3));
    float3 d = make_float3(fma_(P(0, 1), uvy, P(0, 0) * uvx) + P(0, 3), fma_(P(1, 1), uvy, P(1, 0) * uvx) + P(1, 3),
                           fma_(P(2, 1), uvy, P(2, 0) * uvx) + P(2, 3));
    d = make_float3(fma_(C(0, 2), d.z, fma_(C(0, 1), d.y, C(0, 0) * d.x)),
                    fma_(C(1, 2), d.z, fma_(C(1, 1), d.y, C(1, 0) * d.x)),
                    fma_(C(2, 2), d.z, fma_(C(2, 1), d.y, C(2, 0) * d.x)));
    d = normalize3(d);
    uint4* o = reinterpret_cast<uint4*>(rays + pixel_index);
    o[0] = make_uint4(__float_as_uint(origin.x + near_plane * d.x), __float_as_uint(origin.y + near_plane * d.y),
                      __float_as_uint(origin.z + near_plane * d.z), pixel_index);
    o[1] = make_uint4(__float_as_uint(d.x), __float_as_uint(d.y), __float_as_uint(d.z), 0u);
    o[2] = make_uint4(0u, 0u, __float_as_uint(far_plane), 0u);
}

__global__ __launch_bounds__(256) void tt_bounce_kernel(tt_ray_data* __restrict__ rays, uint32_t src_off, uint32_t dst_off,
                                                        uint32_t n, float far_plane, int32_t cur_bounce, int32_t frames,
                                                        int32_t max_bounce, const tt_cuda_triangle* __restrict__ tris,
                                                        const tt_mesh_data* __restrict__ md, uint32_t* __restrict__ counter) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool live = false;
    tt_ray_data nr;
    if (i < n) {
        const tt_ray_data R = rays[src_off + i];
        const float t = __uint_as_float(R.hits[2]);
        if (t < far_plane && (int32_t)R.hits[1] >= 0) {
            const int32_t mesh_id = (int32_t)R.hits[0], tri = (int32_t)R.hits[1];
            const float u = (float)(R.hits[3] & 0xffffu) / 65535.0f, v = (float)(R.hits[3] >> 16) / 65535.0f;
            const float* W = md[mesh_id].W2L;
            const tt_cuda_triangle& T = tris[tri];
            const float3 dir = make_float3(R.direction[0], R.direction[1], R.direction[2]);
            const float3 org = make_float3(R.origin[0], R.origin[1], R.origin[2]);
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
            // sample(): cosine-weighted hemisphere, random(1, pixel) — RayTracingShader.compute:52-84
            const float2 rnd = random2(1, R.PixelIndex, frames, max_bounce, cur_bounce);
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
            sincosf(phi, &sp, &cp);
            const float dx = rr * cp, dz = rr * sp;
            const float3 om = make_float3(dx, sqrtf(fabsf(1.0f - (dx * dx + dz * dz))), dz);
            const float pdf = om.y * 0.318309886548f;
            // GetTangentSpace(norm) — CommonData.cginc (helper (1,0,0), or (0,0,1) if |n.x| > 0.99)
            const float3 helper = fabsf(norm.x) > 0.99f ? make_float3(0, 0, 1) : make_float3(1, 0, 0);
            const float3 tangent = normalize3(cross3(norm, helper));
            const float3 binormal = cross3(norm, tangent);
            float3 nd = make_float3(om.x * tangent.x + om.y * norm.x + om.z * binormal.x,
                                    om.x * tangent.y + om.y * norm.y + om.z * binormal.y,
                                    om.x * tangent.z + om.y * norm.z + om.z * binormal.z);
            nd = normalize3(nd);
            if (pdf > 0.0f) {
                live = true;
                nr.origin[0] = us.x * 0.0001f + pos.x;
                nr.origin[1] = us.y * 0.0001f + pos.y;
                nr.origin[2] = us.z * 0.0001f + pos.z;
                nr.PixelIndex = R.PixelIndex;
                nr.direction[0] = nd.x;
                nr.direction[1] = nd.y;
                nr.direction[2] = nd.z;
                nr.last_pdf = pdf;
                nr.hits[0] = R.hits[0];
                nr.hits[1] = R.hits[1];
                nr.hits[2] = R.hits[2];
                nr.hits[3] = R.hits[3];
            }
        }
    }
    // wave-ballot compaction: one atomic per wave (vs one InterlockedAdd per ray, :500)
    const uint64_t m = __ballot(live);
    if (m == 0) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    if (live) {
        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        uint4* o = reinterpret_cast<uint4*>(rays + dst_off + base + pre);
        o[0] = make_uint4(__float_as_uint(nr.origin[0]), __float_as_uint(nr.origin[1]), __float_as_uint(nr.origin[2]),
                          nr.PixelIndex);
        o[1] = make_uint4(__float_as_uint(nr.direction[0]), __float_as_uint(nr.direction[1]),
                          __float_as_uint(nr.direction[2]), __float_as_uint(nr.last_pdf));
        o[2] = make_uint4(nr.hits[0], nr.hits[1], nr.hits[2], nr.hits[3]);
    }
}

}  // namespace

hipError_t tt_launch_generate(const float* c2w, const float* ip, uint32_t w, uint32_t h, float near_plane, float far_plane,
                              int32_t jitter, int32_t frames, int32_t max_bounce, tt_ray_data* rays, hipStream_t st) {
    hipLaunchKernelGGL(tt_generate_kernel, dim3((w + 255u) / 256u, h), dim3(256), 0, st, c2w, ip, w, h, near_plane, far_plane,
                       jitter, frames, max_bounce, rays);
    return hipGetLastError();
}

hipError_t tt_launch_bounce(tt_ray_data* rays, uint32_t src_off, uint32_t dst_off, uint32_t n, float far_plane,
                            int32_t cur_bounce, int32_t frames, int32_t max_bounce, const tt_cuda_triangle* tris,
                            const tt_mesh_data* md, uint32_t* counter, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tt_bounce_kernel, dim3((n + 255u) / 256u), dim3(256), 0, st, rays, src_off, dst_off, n, far_plane,
                       cur_bounce, frames, max_bounce, tris, md, counter);
    return hipGetLastError();
}
