// Which XCD does block b of a dispatch run on? Records XCC_ID (hardware register 20) per block for
// (1) a launch alone and (2) two launches overlapping on two streams, and prints how often it equals
// blockIdx % 8 -- the placement the trace kernels' segment scheduler assumes (csrc/tt_traverse.h).
// Build: hipcc --offload-arch=gfx950 -O2 tools/xcc_map.hip -o tools/xcc_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void record(unsigned* out, unsigned spin) {
    if (threadIdx.x == 0) {
        out[blockIdx.x] = (unsigned)__builtin_amdgcn_s_getreg(20 | (3 << 11));
        // hold the CU slot for a while so the other stream's blocks interleave
        const long long t0 = clock64();
        while (clock64() - t0 < (long long)spin) {
        }
    }
}

static void report(const char* what, const std::vector<unsigned>& v) {
    size_t same = 0, hist[8] = {};
    for (size_t b = 0; b < v.size(); b++) {
        same += (v[b] & 7u) == (b & 7u);
        hist[v[b] & 7u]++;
    }
    printf("%-28s blocks %zu  xcc == blockIdx %% 8: %.3f  per-xcc:", what, v.size(), (double)same / v.size());
    for (int k = 0; k < 8; k++) printf(" %zu", hist[k]);
    printf("\n");
    // the XCC each blockIdx % 8 class ran on (a fixed bijection keeps the segment scheduler XCD-local)
    size_t m[8][8] = {};
    for (size_t b = 0; b < v.size(); b++) m[b & 7u][v[b] & 7u]++;
    for (int c = 0; c < 8; c++) {
        printf("    blockIdx %% 8 = %d ->", c);
        for (int k = 0; k < 8; k++) printf(" %4zu", m[c][k]);
        printf("\n");
    }
}

int main() {
    const unsigned nb = 4096;
    unsigned *a, *b;
    if (hipMalloc(&a, nb * 4) != hipSuccess || hipMalloc(&b, nb * 4) != hipSuccess) return 1;
    hipStream_t s0, s1;
    if (hipStreamCreate(&s0) != hipSuccess || hipStreamCreate(&s1) != hipSuccess) return 1;
    int nxcc = -1;
    (void)hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, 0);
    printf("hipDeviceAttributeNumberOfXccs = %d\n", nxcc);
    std::vector<unsigned> ha(nb), hb(nb);
    record<<<nb, 64, 0, s0>>>(a, 20000);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipMemcpy(ha.data(), a, nb * 4, hipMemcpyDeviceToHost);
    report("alone", ha);
    for (int rep = 0; rep < 3; rep++) {
        record<<<nb, 64, 0, s0>>>(a, 200000);
        record<<<nb - 3 * rep - 1, 64, 0, s1>>>(b, 200000);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        (void)hipMemcpy(ha.data(), a, nb * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(hb.data(), b, nb * 4, hipMemcpyDeviceToHost);
        hb.resize(nb - 3 * rep - 1);
        report("overlapped, stream 0", ha);
        report("overlapped, stream 1", hb);
        hb.resize(nb);
        // a third launch after an odd-sized one on the same stream
        record<<<nb - 5, 64, 0, s0>>>(a, 1000);
        record<<<nb, 64, 0, s0>>>(a, 1000);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        (void)hipMemcpy(ha.data(), a, nb * 4, hipMemcpyDeviceToHost);
        report("after an odd-sized launch", ha);
    }
    return 0;
}
