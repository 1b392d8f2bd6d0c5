// rt_jsnum.h — JS `number` semantics shared by the host builder and the gfx950 kernels.
//
// The reference computes in IEEE binary64 with one rounding per operation and never fuses a
// multiply with an add (V8).  Everything including this header is compiled with
// -ffp-contract=off and without fast-math so that `a*b + c` stays two rounded operations and
// `/`, sqrt stay correctly rounded on both the host and the device.
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD static inline
#endif

namespace rtjs {

// ToInt32 (ECMA-262 §7.1.6): the conversion behind `x << k`, `x | y`, `x << 0`.
RT_HD int32_t toint32(double x)
{
    if (!(fabs(x) < 2147483648.0)) {                 // rare: huge or non-finite
        if (!isfinite(x)) return 0;
        double m = fmod(trunc(x), 4294967296.0);
        if (m < 0) m += 4294967296.0;
        return (int32_t)(uint32_t)m;
    }
    return (int32_t)x;                               // truncation toward zero
}

// isNegative (src/math/mathutils.ts:45-47): x < 0 || Object.is(x, -0)
RT_HD bool is_negative(double x) { return x < 0 || (x == 0 && signbit(x)); }

// Math.sign: NaN stays NaN, ±0 keep their sign.
RT_HD double sign(double x)
{
    if (x > 0) return 1.0;
    if (x < 0) return -1.0;
    return x;
}

// Math.min / Math.max (NaN-propagating, -0 < +0).
RT_HD double jmin(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b;
}
RT_HD double jmax(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a;
}

// vector.dot (src/math/vector.ts:78-86): accumulator starts at +0, left to right.  The explicit
// `0.0 +` matters: it turns a -0 first product into +0 exactly as the JS loop does.
RT_HD double dot3(double a0, double a1, double a2, double b0, double b1, double b2)
{
    double s = 0.0;
    s += a0 * b0;
    s += a1 * b1;
    s += a2 * b2;
    return s;
}

// RT_SCATTER_COUNTER draws (include/rt.h): the splitmix64 finaliser over (seed, pixel, draw).
RT_HD uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
RT_HD double counter_draw(uint64_t seed, uint64_t pixel, uint32_t n)
{
    const uint64_t x = mix64(seed + pixel * 0x9E3779B97F4A7C15ULL + ((uint64_t)n + 1) * 0xD1B54A32D192ED03ULL);
    return (double)(x >> 11) * 1.1102230246251565e-16;   // 2^-53
}

// (z << 2) + (y << 1) + (x << 0) on ToInt32 values (src/octree_space.ts:82,124).
RT_HD double octant_sum(int32_t x, int32_t y, int32_t z)
{
    return (double)(int32_t)((uint32_t)z << 2) + (double)(int32_t)((uint32_t)y << 1) + (double)x;
}

}  // namespace rtjs
