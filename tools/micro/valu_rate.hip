// Microbenchmark: VALU wave-instruction throughput on gfx950 for (a) independent v_fma_f32,
// (b) v_cvt_f32_ubyte + fma + min/max mixes like the CWBVH node test. Prints cycles per
// wave-instruction per SIMD at 4 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void fma_loop(float* out, int iters, float a) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            x0 = __builtin_fmaf(x0, a, 1.0f); x1 = __builtin_fmaf(x1, a, 1.0f); x2 = __builtin_fmaf(x2, a, 1.0f);
            x3 = __builtin_fmaf(x3, a, 1.0f); x4 = __builtin_fmaf(x4, a, 1.0f); x5 = __builtin_fmaf(x5, a, 1.0f);
            x6 = __builtin_fmaf(x6, a, 1.0f); x7 = __builtin_fmaf(x7, a, 1.0f);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

__global__ __launch_bounds__(256) void cvt_loop(float* out, int iters, unsigned q) {
    float acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
    unsigned v = q ^ threadIdx.x;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            acc0 = fmaxf(acc0, __builtin_fmaf((float)(v & 0xff), 1.5f, acc1));
            acc1 = fminf(acc1, __builtin_fmaf((float)((v >> 8) & 0xff), 1.5f, acc2));
            acc2 = fmaxf(acc2, __builtin_fmaf((float)((v >> 16) & 0xff), 1.5f, acc3));
            acc3 = fminf(acc3, __builtin_fmaf((float)(v >> 24), 1.5f, acc0));
            v = v * 1664525u + 1013904223u;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc0 + acc1 + acc2 + acc3;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * cus * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;  // 256-thread blocks: 4 waves each -> wps waves per SIMD
        hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0001f);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double instr_per_simd = (double)iters * 16 * 8 * wps;  // wave-instructions per SIMD
        printf("fma  waves/SIMD=%d  %.3f ms  %.2f ns/wave-instr/SIMD  (%.2f cycles @2.4GHz)\n", wps, ms,
               ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
        hipLaunchKernelGGL(cvt_loop, dim3(blocks), dim3(256), 0, 0, out, 10, 12345u);
        hipEventRecord(e0);
        hipLaunchKernelGGL(cvt_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 12345u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("cvt  waves/SIMD=%d  %.3f ms  (per 16-step unroll: see ISA count)\n", wps, ms);
    }
    return 0;
}
