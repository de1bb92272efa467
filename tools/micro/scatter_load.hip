// Microbenchmark: vector-memory throughput per CU for the access shapes of the CWBVH node fetch.
// Modes: 0 coalesced 16 B/lane; 1 one random 64-B line per lane (dwordx4); 2 four lanes per line;
// 3 the node fetch itself: 5 x dwordx4 of a random 80-B node per lane from a 2.5 MB array;
// 4 same as 3 but nodes padded to 128 B; 5 node fetch with 8 lanes sharing a node.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hsh(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }

template <int MODE>
__global__ __launch_bounds__(256) void k(const uint4* __restrict__ buf, uint32_t n16, int iters, uint4* out) {
    const uint32_t lane = threadIdx.x & 63, w = (blockIdx.x * 256 + threadIdx.x) >> 6;
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint32_t s = hsh(w * 977 + 13);
    for (int i = 0; i < iters; i++) {
        s = hsh(s + i);
        const uint32_t r = hsh(s ^ lane * 0x9e3779b9u);
        if (MODE == 0) {
            const uint4 v = buf[(s % (n16 / 64)) * 64 + lane];
            acc.x += v.x; acc.y ^= v.y;
        } else if (MODE == 1) {
            const uint4 v = buf[(r % (n16 / 4)) * 4];
            acc.x += v.x; acc.y ^= v.y;
        } else if (MODE == 2) {
            const uint32_t line = hsh(s ^ (lane >> 2) * 0x9e3779b9u) % (n16 / 4);
            const uint4 v = buf[line * 4 + (lane & 3)];
            acc.x += v.x; acc.y ^= v.y;
        } else if (MODE == 3 || MODE == 4 || MODE == 5) {
            const uint32_t stride = MODE == 4 ? 8 : 5;
            const uint32_t nn = n16 / stride;
            const uint32_t node = (MODE == 5 ? hsh(s ^ (lane >> 3) * 0x9e3779b9u) : r) % nn;
            const uint4* p = buf + (size_t)node * stride;
            const uint4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
            acc.x += a.x + b.y + c.z + d.w + e.x; acc.y ^= a.y ^ e.w;
        }
    }
    if (acc.x == 0x12345678u) out[w] = acc;
}

template <int MODE>
float run(const uint4* buf, uint32_t n16, int blocks, int iters, uint4* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, buf, n16, 4, out);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const size_t bytes = 2560 * 1024;  // 2.5 MB, like the C2 node array
    uint4* buf; uint4* out;
    (void)hipMalloc(&buf, bytes); (void)hipMalloc(&out, sizeof(uint4) * 65536);
    (void)hipMemset(buf, 1, bytes);
    const uint32_t n16 = bytes / 16;
    const int iters = 4000;
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
        const int blocks = cus * bpc;
        const double wave_instr_per_cu = (double)iters * 4 * bpc;  // waves per CU = 4*bpc
        const char* names[6] = {"coalesced16", "line/lane", "4lanes/line", "node80", "node128", "node80/8lanes"};
        float ms[6] = {run<0>(buf, n16, blocks, iters, out), run<1>(buf, n16, blocks, iters, out), run<2>(buf, n16, blocks, iters, out),
                       run<3>(buf, n16, blocks, iters, out), run<4>(buf, n16, blocks, iters, out), run<5>(buf, n16, blocks, iters, out)};
        for (int m = 0; m < 6; m++) {
            const double loads = wave_instr_per_cu * (m >= 3 ? 5 : 1);
            printf("waves/CU=%2d %-14s %8.3f ms  %.1f cycles per wave-load-instr per CU (2.4GHz)\n", 4 * bpc, names[m], ms[m],
                   ms[m] * 1e-3 * 2.4e9 / loads);
        }
    }
    return 0;
}
