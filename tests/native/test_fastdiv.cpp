// FastDiv (truetrace-unity-pathtracer_amd/csrc/tt_fastdiv.h) against '/': every divisor 1..4096,
// 2^k - 1 / 2^k / 2^k + 1 and divisors near 2^32, each over edge numerators (0, 1, d - 1, d, d + 1,
// multiples +-1, near 2^32) and seeded random ones. Exit status = number of mismatches (capped).
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "../../truetrace-unity-pathtracer_amd/csrc/tt_fastdiv.h"

static uint64_t bad = 0, checked = 0;
static void check(uint32_t n, uint32_t d, const FastDiv& f) {
    checked++;
    if (fastdiv_eval(n, f) != n / d) {
        if (bad < 10) std::printf("mismatch n=%u d=%u got %u want %u\n", n, d, fastdiv_eval(n, f), n / d);
        bad++;
    }
}
static void divisor(uint32_t d, std::mt19937_64& rng) {
    const FastDiv f = fastdiv_make(d);
    const uint64_t edges[] = {0, 1, 2, d - 1ull, d, d + 1ull, 2ull * d - 1, 2ull * d, 2ull * d + 1, 0xffffffffull,
                              0xfffffffeull, 0x80000000ull, 0x7fffffffull, (0xffffffffull / d) * d,
                              (0xffffffffull / d) * d - 1, 1920ull * 1080 - 1, 3840ull * 2160 - 1};
    for (uint64_t n : edges)
        if (n <= 0xffffffffull) check((uint32_t)n, d, f);
    for (int k = 0; k < 2000; k++) check((uint32_t)rng(), d, f);
    for (int k = 0; k < 200; k++) check((uint32_t)(rng() % (16ull * d + 1)), d, f);
}
int main() {
    std::mt19937_64 rng(0x5EEDull);
    for (uint32_t d = 1; d <= 4096; d++) divisor(d, rng);
    for (int k = 1; k < 32; k++) {
        const uint64_t p = 1ull << k;
        divisor((uint32_t)(p - 1), rng);
        divisor((uint32_t)p, rng);
        if (p + 1 <= 0xffffffffull) divisor((uint32_t)(p + 1), rng);
    }
    for (uint64_t d = 0xffffffffull; d > 0xffffffffull - 64; d--) divisor((uint32_t)d, rng);
    for (int k = 0; k < 2000; k++) divisor((uint32_t)(rng() | 1u), rng);
    std::printf("checked %llu, mismatches %llu\n", (unsigned long long)checked, (unsigned long long)bad);
    return bad > 100 ? 100 : (int)bad;
}
