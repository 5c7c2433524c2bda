// exactdiv.h -- correctly rounded f32 division and reciprocal for gfx950
// without HIP's general divide expansion (v_div_scale x2, v_rcp, 5 fma,
// v_div_fmas, v_div_fixup per quotient).
//
// The reference divides with plain Rust f32 `/` (IEEE, correctly rounded):
// NVec3::new's three divisions by the length (maths.rs:111-118), the normal's
// `/ radius` (common.rs:95) and the camera's `/ (W-1)`, `/ (H-1)`
// (common.rs:335-336).  A quotient a/b computed here is the same bits:
//
//   y  = RN(1/b)            v_rcp_f32 (<= 1 ulp) + one Newton step with fma
//   q  = RN(a*y)            within 1 ulp of a/b
//   r  = RN(q*b - a)        exact (fma; the remainder is representable)
//   q' = RN(q - r*y)        Markstein's theorem: q' == RN(a/b)
//
// Markstein (IBM J. R&D 34(1), 1990; Muller et al., Handbook of
// Floating-Point Arithmetic, 2nd ed., Thm 4.10): if y is 1/b correctly
// rounded and q is within one ulp of a/b, the corrected quotient is a/b
// correctly rounded, provided no step under- or overflows.  The guards below
// keep every operand in that range (denominator in [2^-40, 2^40], numerator
// 0 or of magnitude in [2^-60, 2^60]: then |q| >= 2^-100 and the remainder's
// quantum is >= 2^-149) and callers fall back to the HIP divide otherwise.
// The one step rcp -> RN(1/b) is not covered by the theorem for every
// hardware rcp result, so it is checked exhaustively on the device for every
// b in the guarded range (tools/exactdiv_check.hip, tests/test_gpu_exactdiv.py).
//
// Signed zeros: with r = q*b - a and q' = q - r*y (rather than r = a - q*b,
// q' = q + r*y) a zero numerator keeps its sign for b > 0, as IEEE division
// does; b > 0 is part of the denominator guard.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rtamd {

// b in [2^-40, 2^40] (so also b > 0, finite, not NaN): one unsigned compare.
__device__ __forceinline__ bool xdiv_den_ok(float b) {
    return (__float_as_uint(b) - 0x2B800000u) <= (0x53800000u - 0x2B800000u);
}

// a == 0 or |a| in [2^-60, 2^60) for three numerators (frexp exponent of 0 is 0;
// of inf/NaN it is 0 as well, which the magnitude test rejects: a sum, not a
// max, because fmaxf drops NaN operands).
__device__ __forceinline__ bool xdiv_num3_ok(float a, float b, float c) {
    const int e = min(min(__builtin_amdgcn_frexp_expf(a), __builtin_amdgcn_frexp_expf(b)),
                      __builtin_amdgcn_frexp_expf(c));
    const float m = (fabsf(a) + fabsf(b)) + fabsf(c);
    return (e >= -59) & (m < 0x1p60f);
}

// The same guard for numerators bounded by the denominator (|a| <= b (1 +
// 2^-22), as the components of a vector are by its computed length): with b
// <= 2^40 the upper bound holds by itself, so only the exponents are checked
// (0 and inf/NaN have frexp exponent 0; inf/NaN components make the length
// fail xdiv_den_ok).
__device__ __forceinline__ bool xdiv_num3_small_ok(float a, float b, float c) {
    const int e = min(min(__builtin_amdgcn_frexp_expf(a), __builtin_amdgcn_frexp_expf(b)),
                      __builtin_amdgcn_frexp_expf(c));
    return e >= -59;
}

// RN(1/b) for b in the guarded range (exhaustively checked, see above).
__device__ __forceinline__ float xdiv_rcp(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

// RN(a/b) given y = RN(1/b), b > 0, within the guards.
__device__ __forceinline__ float xdiv(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(q, b, -a);
    return __builtin_fmaf(-r, y, q);
}

// RN(sqrt(a)) -- the bits of IEEE sqrtf (maths.rs:107 `f32::sqrt`,
// common.rs:84) without the general expansion's denormal scaling and class
// fix-up.  gfx950's v_sqrt_f32 is within one ulp of the exact root for every
// positive normal input (tools/sqrt_probe.hip), so the correctly rounded root
// is s, s - ulp or s + ulp; the two residuals a - s'*s (one fma each, exact
// enough for a >= 2^-96) pick it, as in the general sequence.  Inputs below
// 2^-96 (and zero, negatives, NaN) take HIP's sqrtf.  Checked on the device
// against sqrtf for all 2^32 inputs (tools/exactdiv_check.hip).
__device__ __forceinline__ float xsqrt(float a) {
    const float s = __builtin_amdgcn_sqrtf(a);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, a);
    const float rp = __builtin_fmaf(-sp, s, a);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    if (__builtin_expect(!(a >= 0x1p-96f), 0)) r = __builtin_sqrtf(a);
    return r;
}

}  // namespace rtamd
