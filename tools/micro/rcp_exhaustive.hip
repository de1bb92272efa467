// Exhaustive check over all 2^32 fp32 inputs: is v_rcp_f32 + one FMA Newton step
// (e = fma(-a, r, 1), r' = fma(e, r, r)) bitwise equal to the correctly rounded 1.0f / a?
// Prints mismatch counts per input class (by biased exponent) and a few examples.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void k(uint32_t hi, unsigned long long* bad_by_exp, uint32_t* examples, uint32_t* n_ex) {
    const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float a = __uint_as_float(bits);
    const float ref = 1.0f / a;
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = __builtin_fmaf(-a, r, 1.0f);
    const float r2 = __builtin_fmaf(e, r, r);
    const bool same = (__float_as_uint(ref) == __float_as_uint(r2)) || (ref != ref && r2 != r2);
    if (!same) {
        atomicAdd(&bad_by_exp[(bits >> 23) & 0xff], 1ull);
        const uint32_t i = atomicAdd(n_ex, 1u);
        if (i < 64) { examples[2 * i] = bits; examples[2 * i + 1] = __float_as_uint(r2); }
    }
}

int main() {
    unsigned long long* d_bad; uint32_t *d_ex, *d_n;
    hipMalloc(&d_bad, 256 * 8); hipMalloc(&d_ex, 128 * 4); hipMalloc(&d_n, 4);
    hipMemset(d_bad, 0, 256 * 8); hipMemset(d_n, 0, 4);
    for (uint32_t hi = 0; hi < 256; hi++) hipLaunchKernelGGL(k, dim3(1 << 16), dim3(256), 0, 0, hi, d_bad, d_ex, d_n);
    hipDeviceSynchronize();
    unsigned long long bad[256]; uint32_t ex[128], n;
    hipMemcpy(bad, d_bad, sizeof bad, hipMemcpyDeviceToHost);
    hipMemcpy(ex, d_ex, sizeof ex, hipMemcpyDeviceToHost);
    hipMemcpy(&n, d_n, 4, hipMemcpyDeviceToHost);
    unsigned long long total = 0;
    for (int e = 0; e < 256; e++) { total += bad[e]; if (bad[e]) printf("exp %3d (2^%d): %llu mismatches\n", e, e - 127, bad[e]); }
    printf("total mismatches %llu of 2^32\n", total);
    for (uint32_t i = 0; i < (n < 16 ? n : 16); i++) {
        float a, r; uint32_t b = ex[2 * i], rb = ex[2 * i + 1];
        memcpy(&a, &b, 4); memcpy(&r, &rb, 4);
        printf("  a=%08x (%g) newton=%08x (%g) exact=%g\n", b, a, rb, r, 1.0f / a);
    }
    return 0;
}
