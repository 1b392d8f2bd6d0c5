// rt_jsnum.h — JS `number` semantics shared by the host builder and the gfx950 kernels.
//
// The reference computes in IEEE binary64 with one rounding per operation and never fuses a
// multiply with an add (V8).  Everything including this header is compiled with
// -ffp-contract=off and without fast-math so that `a*b + c` stays two rounded operations and
// `/`, sqrt stay correctly rounded on both the host and the device.
#pragma once

#include <math.h>
#include <stdint.h>
#include <string.h>

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

// ---- Math.atan / Math.atan2 as V8 computes them ---------------------------------------------------
// V8 implements Math.atan2 with the fdlibm algorithm (e_atan2.c / s_atan.c: argument reduction
// against atan(0.5), atan(1), atan(1.5), atan(inf), an 11-term odd polynomial, hi/lo constant
// pairs).  Restated here in plain binary64 (no contraction), so the texture coordinates of
// uv_map_sphere (src/math/uv_mapping.ts:19-25) match the reference bit for bit; pinned against
// node by tests/golden/gen_texture.js.
RT_HD uint32_t hi_word(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)(b >> 32); }
RT_HD uint32_t lo_word(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)b; }

RT_HD double js_atan(double x)
{
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                              9.82793723247329054082e-01, 1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                              1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                           1.42857142725034663711e-01, -1.11111104054623557880e-01,
                           9.09088713343650656196e-02, -7.69187620504482999495e-02,
                           6.66107313738753120669e-02, -5.83357013379057348645e-02,
                           4.97687799461593236017e-02, -3.65315727442169155270e-02,
                           1.62858201153657823623e-02};
    const int32_t hx = (int32_t)hi_word(x);
    const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
    int id;
    if (ix >= 0x44100000u) {                         // |x| >= 2^66
        if (ix > 0x7ff00000u || (ix == 0x7ff00000u && lo_word(x) != 0)) return x + x;   // NaN
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000u) {                          // |x| < 0.4375
        if (ix < 0x3e400000u) return x;              // |x| < 2^-27
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000u) {                      // |x| < 1.1875
            if (ix < 0x3fe60000u) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }   // 7/16 <= |x| < 11/16
            else                  { id = 1; x = (x - 1.0) / (x + 1.0); }         // 11/16 <= |x| < 19/16
        } else {
            if (ix < 0x40038000u) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }  // |x| < 2.4375
            else                  { id = 3; x = -1.0 / x; }                      // 2.4375 <= |x| < 2^66
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

RT_HD double js_atan2(double y, double x)
{
    const double tiny = 1.0e-300;
    const double pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00;
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const int32_t hx = (int32_t)hi_word(x), hy = (int32_t)hi_word(y);
    const uint32_t ix = (uint32_t)hx & 0x7fffffffu, iy = (uint32_t)hy & 0x7fffffffu;
    const uint32_t lx = lo_word(x), ly = lo_word(y);
    if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;                                // NaN
    if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return js_atan(y);   // x == 1.0
    int m = (int)(((uint32_t)hy >> 31) & 1u) | (int)(((uint32_t)hx >> 30) & 2u);   // 2*sign(x) + sign(y)
    if ((iy | ly) == 0) {                            // y = +-0
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   // x = +-0
    if (ix == 0x7ff00000u) {                         // x = +-inf
        if (iy == 0x7ff00000u) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0 * pi_o_4 + tiny;
            default: return -3.0 * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0: return 0.0;
        case 1: return -0.0;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (iy == 0x7ff00000u) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   // y = +-inf
    const int k = ((int32_t)iy - (int32_t)ix) >> 20;
    double z;
    if (k > 60) {                                    // |y/x| > 2^60
        z = pi_o_2 + 0.5 * pi_lo;
        m &= 1;
    } else if (hx < 0 && k < -60) {
        z = 0.0;                                     // 0 > |y|/x > -2^-60
    } else {
        z = js_atan(fabs(y / x));
    }
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

// uv_map_sphere (src/math/uv_mapping.ts:19-25) of a direction / offset vector
RT_HD void uv_map_sphere(double d0, double d1, double d2, double &u, double &v)
{
    const double JS_PI = 3.141592653589793, JS_EPS = 2.220446049250313e-16;
    u = js_atan2(d1, d0) / JS_PI / 2.0 + 0.5 - JS_EPS;
    const double len = sqrt((0.0 + d0 * d0) + d1 * d1);   // vector.length(vector.reduce(dir, 2))
    v = js_atan2(d2, len) / JS_PI + 0.5 - JS_EPS;
}

// ImageTexture.get_color (src/texture/texture_image.ts:40-63): the texel index (pixel, not byte),
// or -1 where the reference throws 'Texture coordinates out of bounds'.
RT_HD int64_t texel_index(double u, double v, int32_t width, int32_t height)
{
    const double JS_EPS = 2.220446049250313e-16;
    if (u < 0 - JS_EPS || u > 1 - JS_EPS || v < 0 - JS_EPS || v > 1 - JS_EPS) return -1;
    const int32_t ui = toint32(u * (double)width), vi = toint32(v * (double)height);
    return (int64_t)vi * width + ui;
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
