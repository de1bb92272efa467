// tt_resolve.hip — attribute resolve for the hits in GlobalRays: interpolated shading normal
// (GetTriangleNormal, CommonData.cginc:904-911) and the unsmoothed geometric normal
// (RayTracingShader.compute:111-118), both through Inverse = transpose((float3x3)W2L).
// Not part of the trace hot loop; it exists so "normals within 1e-5" is checkable at the
// boundary. One ray per lane, HBM-bound (48 B ray + 88 B triangle + 64 B W2L in, 24 B out).
#include "tt_device.h"

namespace {

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

__device__ __forceinline__ float3 normalize3(float3 v) {
    const float inv = 1.0f / sqrtf(fma_(v.z, v.z, fma_(v.y, v.y, v.x * v.x)));
    return make_float3(v.x * inv, v.y * inv, v.z * inv);
}

// i_octahedral_32 — CommonData.cginc:849-857
__device__ __forceinline__ float3 i_octahedral_32(uint32_t data) {
    const uint32_t ix = data & 65535u, iy = (data >> 16) & 65535u;
    const float vx = (float)ix / 32767.5f - 1.0f, vy = (float)iy / 32767.5f - 1.0f;
    float3 nor = make_float3(vx, vy, 1.0f - fabsf(vx) - fabsf(vy));
    const float t = fmaxf(-nor.z, 0.0f);
    nor.x += (nor.x > 0.0f) ? -t : t;
    nor.y += (nor.y > 0.0f) ? -t : t;
    return normalize3(nor);
}

// mul(Inverse, x) with Inverse = transpose(W2L 3x3): row r = sum_c W2L(c, r) * x_c
__device__ __forceinline__ float3 mul_inv(const float* W, float3 x) {
    auto M = [&](int r, int c) { return W[c * 4 + r]; };
    return make_float3(fma_(M(2, 0), x.z, fma_(M(1, 0), x.y, M(0, 0) * x.x)),
                       fma_(M(2, 1), x.z, fma_(M(1, 1), x.y, M(0, 1) * x.x)),
                       fma_(M(2, 2), x.z, fma_(M(1, 2), x.y, M(0, 2) * x.x)));
}

__global__ __launch_bounds__(256) void tt_resolve_kernel(const tt_ray_data* __restrict__ rays, uint32_t off, uint32_t n,
                                                         float far_plane, const tt_cuda_triangle* __restrict__ tris,
                                                         uint32_t n_tris, const tt_mesh_data* __restrict__ md,
                                                         uint32_t n_mesh, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tt_ray_data* r = rays + off + i;
    float* o = out + (size_t)6 * i;
    const uint4 h = reinterpret_cast<const uint4*>(r)[2];
    const float t = __uint_as_float(h.z);
    const int32_t mesh_id = (int32_t)h.x, tri = (int32_t)h.y;
    if (!(t < far_plane) || tri < 0 || (uint32_t)tri >= n_tris || (uint32_t)mesh_id >= n_mesh) {
        for (int k = 0; k < 6; k++) o[k] = 0.0f;
        return;
    }
    // get() — CommonData.cginc:441-455
    const float u = (float)(h.w & 0xffffu) / 65535.0f;
    const float v = (float)(h.w >> 16) / 65535.0f;
    const float* W = md[mesh_id].W2L;
    const tt_cuda_triangle& T = tris[tri];
    const float3 n0 = i_octahedral_32(T.norms[0]), n1 = i_octahedral_32(T.norms[1]), n2 = i_octahedral_32(T.norms[2]);
    const float w0 = 1.0f - u - v;
    const float3 ni = make_float3(n0.x * w0 + u * n1.x + v * n2.x, n0.y * w0 + u * n1.y + v * n2.y,
                                  n0.z * w0 + u * n1.z + v * n2.z);
    float3 g = mul_inv(W, ni);
    const float gs = 1.0f / sqrtf(fma_(g.z, g.z, fma_(g.y, g.y, g.x * g.x)));
    g = make_float3(gs * g.x, gs * g.y, gs * g.z);
    const float3 e1 = normalize3(make_float3(T.posedge1[0], T.posedge1[1], T.posedge1[2]));
    const float3 e2 = normalize3(make_float3(T.posedge2[0], T.posedge2[1], T.posedge2[2]));
    const float3 c = make_float3(fma_(e1.y, e2.z, -(e1.z * e2.y)), fma_(e1.z, e2.x, -(e1.x * e2.z)),
                                 fma_(e1.x, e2.y, -(e1.y * e2.x)));
    float3 us = mul_inv(W, c);
    const float uss = 1.0f / sqrtf(fma_(us.z, us.z, fma_(us.y, us.y, us.x * us.x)));
    us = make_float3(-(uss * us.x), -(uss * us.y), -(uss * us.z));
    if (fma_(us.z, g.z, fma_(us.y, g.y, us.x * g.x)) < 0) us = make_float3(-us.x, -us.y, -us.z);
    o[0] = g.x;
    o[1] = g.y;
    o[2] = g.z;
    o[3] = us.x;
    o[4] = us.y;
    o[5] = us.z;
}

}  // namespace

hipError_t tt_launch_resolve(const tt_ray_data* rays, uint32_t ray_offset, uint32_t n, float far_plane,
                             const tt_cuda_triangle* tris, uint32_t n_tris, const tt_mesh_data* md, uint32_t n_mesh,
                             float* out, hipStream_t st) {
    const uint32_t grid = (n + 255u) / 256u;
    hipLaunchKernelGGL(tt_resolve_kernel, dim3(grid), dim3(256), 0, st, rays, ray_offset, n, far_plane, tris, n_tris, md,
                       n_mesh, out);
    return hipGetLastError();
}
