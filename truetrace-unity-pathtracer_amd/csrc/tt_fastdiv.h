// tt_fastdiv.h — exact unsigned division by a launch-constant divisor (round-up multiplier, valid
// for every 32-bit n and d >= 1): q = (t + ((n - t) >> s1)) >> s2 with t = umulhi(m, n). The host
// fills it (fastdiv_make); it replaces the ~40-instruction VALU udiv in the refill and pixel decode.
// Plain C++ apart from the device entry point, so tests/native/test_fastdiv.cpp checks the host
// construction with g++ against '/' (fastdiv_eval is the same arithmetic on the host).
#ifndef TT_FASTDIV_H
#define TT_FASTDIV_H
#include <stdint.h>

struct FastDiv {
    uint32_t m, s1, s2;
};
inline FastDiv fastdiv_make(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) l++;
    const unsigned __int128 m = (((unsigned __int128)1 << 32) * (((unsigned __int128)1 << l) - d)) / d + 1u;
    return FastDiv{(uint32_t)m, l < 1 ? l : 1u, l > 1 ? l - 1 : 0u};
}
inline uint32_t fastdiv_eval(uint32_t n, const FastDiv& d) {  // host mirror of fastdiv()
    const uint32_t t = (uint32_t)(((uint64_t)d.m * n) >> 32);
    return (t + ((n - t) >> d.s1)) >> d.s2;
}
#ifdef __HIPCC__
__device__ __forceinline__ uint32_t fastdiv(uint32_t n, const FastDiv& d) {
    const uint32_t t = __umulhi(d.m, n);
    return (t + ((n - t) >> d.s1)) >> d.s2;
}
#endif
#endif  // TT_FASTDIV_H
