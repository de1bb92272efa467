// coop_fetch.hip -- micro: how much texture-path time the closest-hit kernel's scattered node loads cost, and
// what a cooperative fetch would save ("what TD's 0.88 is made of").
//
// Every lane of every wave needs one 80-B node per iteration (nodes at random 128-B-aligned slots of a table
// sized like the C2 scene's node working set). Three ways to get the 80 B into the lane's registers:
//   scatter  the kernel's way: five 16-B buffer loads at the lane's own node (each wave instruction touches
//            ~64 different lines);
//   coop     five 16-B loads in which five consecutive lanes read one node's five chunks (each instruction
//            touches ~13 lines), chunks handed to their owners through a 5-KiB LDS block per wave
//            (ds_write_b128 x 5, ds_read_b128 x 5; the node indices go through LDS first);
//   coop4    as coop, but the fifth chunk is loaded by its owner directly (four cooperative loads covering 64 B
//            of each node + one scattered load; 4 KiB LDS per wave).
// The XOR of everything loaded is written per lane, so no load is dead. One wave per block, BLOCKS_PER_CU
// blocks per CU, like the trace kernel. Prints ns per node per CU for each form.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/coop_fetch.hip -o tools/micro/bin/coop_fetch
// Run:   tools/micro/bin/coop_fetch [table_MiB=40] [iters=256] [blocks_per_cu=20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <int MODE>  // 0 scatter, 1 coop, 2 coop4
__global__ __launch_bounds__(64) void fetch(const uint8_t* __restrict__ table, uint32_t n_nodes, uint32_t iters,
                                            uint32_t* __restrict__ out) {
    __shared__ u32x4 stage[64 * 5];
    __shared__ uint32_t s_idx[64];
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(table), 0,
                                                                       (int)(n_nodes * 128u), 0x00020000);
    const uint32_t lane = threadIdx.x;
    uint32_t acc = 0;
    uint32_t seed = blockIdx.x * 64u + lane;
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t mine = hash(seed ^ (it * 0x9e3779b9u)) % n_nodes;  // the node this lane needs
        u32x4 c0, c1, c2, c3, c4;
        if (MODE == 0) {
            const uint32_t no = mine * 128u;
            c0 = ld16(r, no);
            c1 = ld16(r, no + 16u);
            c2 = ld16(r, no + 32u);
            c3 = ld16(r, no + 48u);
            c4 = ld16(r, no + 64u);
        } else {
            constexpr uint32_t K = MODE == 1 ? 5u : 4u;  // cooperative chunks per node
            s_idx[lane] = mine;
            __syncthreads();  // (one wave per block: orders the LDS hand-off across lanes)
#pragma unroll
            for (uint32_t i = 0; i < K; i++) {
                const uint32_t s = i * 64u + lane, j = s / K, c = s % K;  // slot -> (node owner, chunk)
                const u32x4 v = ld16(r, s_idx[j] * 128u + c * 16u);
                stage[j * 5u + c] = v;
            }
            if (MODE == 2) c4 = ld16(r, mine * 128u + 64u);
            __syncthreads();
            c0 = stage[lane * 5u + 0u];
            c1 = stage[lane * 5u + 1u];
            c2 = stage[lane * 5u + 2u];
            c3 = stage[lane * 5u + 3u];
            if (MODE == 1) c4 = stage[lane * 5u + 4u];
            __syncthreads();  // (the next iteration rewrites the block)
        }
        acc ^= c0.x ^ c1.y ^ c2.z ^ c3.w ^ c4.x ^ c0.w ^ c4.w;
    }
    out[blockIdx.x * 64u + lane] = acc;
}

int main(int argc, char** argv) {
    const uint32_t mib = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 40u;
    const uint32_t iters = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 256u;
    const uint32_t bpc = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 20u;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const uint32_t cus = (uint32_t)prop.multiProcessorCount;
    const uint32_t n_nodes = mib * 1024u * 1024u / 128u;
    uint8_t* table = nullptr;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&table, (size_t)n_nodes * 128u));
    std::vector<uint8_t> h((size_t)n_nodes * 128u);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
    CHECK(hipMemcpy(table, h.data(), h.size(), hipMemcpyHostToDevice));
    const uint32_t blocks = cus * bpc;
    CHECK(hipMalloc(&out, (size_t)blocks * 64u * 4u));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[3] = {"scatter (5 x 16-B per lane)", "coop (5 chunks via LDS)", "coop4 (4 via LDS + 1 own)"};
    std::printf("table %u MiB (%u nodes of 128 B), %u CUs x %u one-wave blocks, %u iterations\n", mib, n_nodes, cus, bpc,
                iters);
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 3; mode++) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(fetch<0>, dim3(blocks), dim3(64), 0, 0, table, n_nodes, iters, out);
                if (mode == 1) hipLaunchKernelGGL(fetch<1>, dim3(blocks), dim3(64), 0, 0, table, n_nodes, iters, out);
                if (mode == 2) hipLaunchKernelGGL(fetch<2>, dim3(blocks), dim3(64), 0, 0, table, n_nodes, iters, out);
            };
            launch();  // warm
            CHECK(hipEventRecord(e0, 0));
            for (int k = 0; k < 5; k++) launch();
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double nodes = 5.0 * blocks * 64.0 * iters;
            std::printf("rep %d  %-30s %8.3f ms  %7.3f ns/node/CU  %7.1f Gnodes/s\n", rep, names[mode], ms / 5.0,
                        ms * 1e6 / nodes * cus, nodes / (ms * 1e-3) / 1e9);
        }
    CHECK(hipFree(table));
    CHECK(hipFree(out));
    return 0;
}
