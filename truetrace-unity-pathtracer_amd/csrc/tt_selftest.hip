// tt_selftest.hip — on-device self-test of the kernels' fast reciprocal (rcp_rn, tt_device.h)
// against the correctly rounded IEEE division over every fp32 bit pattern.
#include "tt_device.h"

namespace {
__global__ void tt_rcp_check_kernel(uint32_t hi, unsigned long long* bad) {
    const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float a = __uint_as_float(bits);
    const float fast = rcp_rn(a), ref = 1.0f / a;
    const bool same = __float_as_uint(fast) == __float_as_uint(ref) || (fast != fast && ref != ref);
    const uint64_t m = __ballot(!same);
    if ((threadIdx.x & 63u) == 0u && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}
}  // namespace

hipError_t tt_launch_rcp_selftest(unsigned long long* d_bad, hipStream_t st) {
    for (uint32_t hi = 0; hi < 256u; hi++) {
        hipLaunchKernelGGL(tt_rcp_check_kernel, dim3(1u << 16), dim3(256), 0, st, hi, d_bad);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
