// fastdiv.h -- unsigned 32-bit division by a runtime-invariant divisor
// (host + device; no HIP dependency so the CPU tests can check it).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define RT_HOST_DEVICE __host__ __device__
#else
#define RT_HOST_DEVICE
#endif

namespace rtamd {

// Unsigned division by a runtime-invariant divisor d (Granlund-Montgomery,
// round-up variant): q = (t + ((n - t) >> 1)) >> s with t = mulhi(n, m);
// exact for every 32-bit n.  d == 1 is flagged (one != 0).
struct FastDiv {
    uint32_t m, s, one, d;
};
RT_HOST_DEVICE inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{0, 0, d <= 1u ? 1u : 0u, d ? d : 1u};
    if (d > 1) {
        uint32_t l = 0;
        while ((1ull << l) < d) ++l;  // ceil(log2 d), >= 1
        f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
        f.s = l - 1;
    }
    return f;
}
RT_HOST_DEVICE inline uint32_t fastdiv_apply(uint32_t n, const FastDiv &f) {
    if (f.one) return n;
    const uint32_t t = (uint32_t)(((uint64_t)n * f.m) >> 32);  // v_mul_hi_u32 on device
    return (t + ((n - t) >> 1)) >> f.s;
}

}  // namespace rtamd
