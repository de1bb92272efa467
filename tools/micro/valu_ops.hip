// Microbenchmark: wave64 issue cost (cycles per wave-instruction per SIMD, 8 waves/SIMD) of the
// VALU ops the CWBVH node test is made of. 16 independent chains per lane, inline asm.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    float r[16];
    unsigned u[16];
    double d[16];
    unsigned long long sm[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) { r[i] = threadIdx.x + i; u[i] = threadIdx.x * 77 + i; d[i] = r[i]; }
    const float a = 1.0001f, b = 0.5f;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
            if (OP == 1) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(r[i]) : "v"(u[i]));
            if (OP == 2) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 15]), "v"(0x0c0c0c01u));
            if (OP == 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[i]) : "v"(d[(i + 1) & 15]), "v"(d[(i + 2) & 15]));
            if (OP == 4) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
            if (OP == 5) asm volatile("v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a) : "vcc");
            if (OP == 6) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 7) asm volatile("v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[0,1,0]" : "+v"(r[i]) : "v"(u[i]), "v"(b));
            if (OP == 8) asm volatile("v_rcp_f32 %0, %0" : "+v"(r[i]));
            if (OP == 9) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(u[i]));
            if (OP == 10) asm volatile("v_max_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
            if (OP == 11) asm volatile("v_min_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
            if (OP == 12) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
            if (OP == 13) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
            if (OP == 14) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
            if (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a));
            if (OP == 16) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(r[i]), "v"(a) : "vcc");
            if (OP == 17) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 18) asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 19) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 20) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(r[i]) : "v"(u[i]));
            if (OP == 21) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
            if (OP == 22) asm volatile("v_mov_b32 %0, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 15]));
            if (OP == 23) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 24) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 15]));
            if (OP == 25) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 15]));
            if (OP == 26) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(sm[i & 3]) : "v"(r[i]), "v"(a));
            if (OP == 27) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(r[i]) : "v"(a));
            if (OP == 28) asm volatile("v_max_i32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
            if (OP == 29) asm volatile("v_cvt_pk_f32_fp8 %0, %1" : "=v"(d[i]) : "v"(u[i]));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) s += r[i] + (float)u[i] + (float)d[i];
    out[blockIdx.x * 256 + threadIdx.x] = s + (float)(sm[0] ^ sm[1] ^ sm[2] ^ sm[3]);
}

template <int OP>
void run(const char* name, float* out, int cus, double instr_per_iter) {
    const int blocks = cus * 8, iters = 4000;  // 8 blocks x 4 waves = 8 waves per SIMD
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 10);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = (double)iters * 16 * instr_per_iter * 8;  // wave-instructions per SIMD
    printf("%-22s %.3f ms  %.2f ns/wave-instr/SIMD  (%.2f cycles @2.1GHz)\n", name, ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.1);
}

int main() {
    hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
    float* out; (void)hipMalloc(&out, sizeof(float) * 256 * p.multiProcessorCount * 8);
    run<0>("v_fma_f32", out, p.multiProcessorCount, 1);
    run<1>("v_cvt_f32_ubyte1", out, p.multiProcessorCount, 1);
    run<2>("v_perm_b32", out, p.multiProcessorCount, 1);
    run<3>("v_pk_fma_f32", out, p.multiProcessorCount, 1);
    run<4>("v_max3_f32", out, p.multiProcessorCount, 1);
    run<5>("v_cmp+v_cndmask", out, p.multiProcessorCount, 2);
    run<6>("v_lshlrev_b32", out, p.multiProcessorCount, 1);
    run<7>("v_fma_mix_f32", out, p.multiProcessorCount, 1);
    run<8>("v_rcp_f32", out, p.multiProcessorCount, 1);
    run<9>("v_bfe_u32", out, p.multiProcessorCount, 1);
    run<10>("v_max_f32", out, p.multiProcessorCount, 1);
    run<11>("v_min_f32", out, p.multiProcessorCount, 1);
    run<12>("v_mul_f32", out, p.multiProcessorCount, 1);
    run<13>("v_add_f32", out, p.multiProcessorCount, 1);
    run<14>("v_fmac_f32", out, p.multiProcessorCount, 1);
    run<15>("v_cndmask_b32", out, p.multiProcessorCount, 1);
    run<16>("v_cmp_lt_f32 (vcc)", out, p.multiProcessorCount, 1);
    run<17>("v_and_b32", out, p.multiProcessorCount, 1);
    run<18>("v_or_b32", out, p.multiProcessorCount, 1);
    run<19>("v_add_u32", out, p.multiProcessorCount, 1);
    run<20>("v_cvt_f32_u32", out, p.multiProcessorCount, 1);
    run<21>("v_med3_f32", out, p.multiProcessorCount, 1);
    run<22>("v_mov_b32", out, p.multiProcessorCount, 1);
    run<23>("v_lshl_or_b32", out, p.multiProcessorCount, 1);
    run<24>("v_pk_mul_f32", out, p.multiProcessorCount, 1);
    run<25>("v_pk_add_f32", out, p.multiProcessorCount, 1);
    run<26>("v_cmp_lt_f32_e64 (sgpr)", out, p.multiProcessorCount, 1);
    run<27>("v_sub_f32", out, p.multiProcessorCount, 1);
    run<28>("v_max_i32", out, p.multiProcessorCount, 1);
    run<29>("v_cvt_pk_f32_fp8", out, p.multiProcessorCount, 1);
    return 0;
}
