// rt_math.h -- deterministic binary32 primitives shared by the HIP kernels and
// the host-side constant builder (compiled __host__ __device__).
//
// The reference is HLSL (fxc, cs_5_0), whose pow/exp/log/sin/cos/div/rsq are
// implementation-defined hardware approximations.  This framework fixes one
// definition (rules R1-R9) so the GPU frame is bit-exact
// against the CPU oracle:
//   * a*b+c forms of the HLSL source are single fused multiply-adds (fxc `mad`);
//   * a/b is a * rcp(b) with a correctly rounded rcp (D3D `div` = rcp+mul);
//   * sqrt is correctly rounded; normalize(v) = v * rcp(sqrt(dot(v,v)));
//   * exp2/log2/sin/cos are the fixed polynomials below (1-2 ulp), pow(x,y) =
//     exp2(y*log2(x)), exp(x) = exp2(x*log2(e));
//   * max/min are IEEE-754-2019 maximumNumber/minimumNumber (v_max_f32).
// Build every translation unit that includes this with -ffp-contract=off.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define RT_HD static inline
#endif

namespace rtm {

RT_HD float fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

RT_HD uint32_t bits(float f)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(uint32_t, f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}
RT_HD float fbits(uint32_t u)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(float, u);
#else
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}

RT_HD bool isnan_(float x) { return x != x; }

// IEEE 754-2019 maximumNumber / minimumNumber (R6).
RT_HD float max(float a, float b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmaximum_numf(a, b);
#else
    if (a != a) return b;
    if (b != b) return a;
    if (a > b) return a;
    if (b > a) return b;
    return (bits(a) >> 31) ? b : a;
#endif
}
RT_HD float min(float a, float b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fminimum_numf(a, b);
#else
    if (a != a) return b;
    if (b != b) return a;
    if (a < b) return a;
    if (b < a) return b;
    return (bits(a) >> 31) ? a : b;
#endif
}
RT_HD float sat(float x) { return min(max(x, 0.0f), 1.0f); }
RT_HD float rcp(float x) { return 1.0f / x; }           // correctly rounded
RT_HD float sqrt(float x) { return __builtin_sqrtf(x); } // correctly rounded
RT_HD float floor(float x) { return __builtin_floorf(x); }
RT_HD float abs(float x) { return __builtin_fabsf(x); }
RT_HD float rint(float x) { return __builtin_rintf(x); }
RT_HD float lerp(float a, float b, float t) { return fma(t, b - a, a); }

RT_HD float exp2(float x)
{
    if (isnan_(x)) return x;
    if (x >= 128.0f) return __builtin_inff();
    if (x < -150.0f) return 0.0f;
    float n = rint(x);
    float f = x - n;
    float p = 0x1.41a6fep-13f;
    p = fma(p, f, 0x1.5f44f0p-10f);
    p = fma(p, f, 0x1.3b2dfep-7f);
    p = fma(p, f, 0x1.c6aed6p-5f);
    p = fma(p, f, 0x1.ebfbdap-3f);
    p = fma(p, f, 0x1.62e430p-1f);
    p = fma(p, f, 1.0f);
    return __builtin_ldexpf(p, (int)n);
}

// log2 for x > 0 finite (callers: pow of non-negative bases); full special-case
// handling kept for the primitive-parity tests.
RT_HD float log2(float x)
{
    if (isnan_(x)) return x;
    if (x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -__builtin_inff();
    if (x == __builtin_inff()) return x;
    uint32_t ix = bits(x);
    int e = 0;
    if (ix < 0x00800000u) {
        x = x * 8388608.0f;
        ix = bits(x);
        e = -23;
    }
    e += (int)(ix >> 23) - 127;
    uint32_t mb = (ix & 0x007fffffu) | 0x3f800000u;
    if (mb > 0x3fb504f3u) {
        mb -= 0x00800000u;
        e += 1;
    }
    float f = fbits(mb) - 1.0f;
    float p = -0x1.c362c0p-4f;
    p = fma(p, f, 0x1.7d9132p-3f);
    p = fma(p, f, -0x1.87381ap-3f);
    p = fma(p, f, 0x1.a2f85ep-3f);
    p = fma(p, f, -0x1.eabd64p-3f);
    p = fma(p, f, 0x1.277e9ap-2f);
    p = fma(p, f, -0x1.715a76p-2f);
    p = fma(p, f, 0x1.ec7094p-2f);
    p = fma(p, f, -0x1.715470p-1f);
    p = fma(p, f, 0x1.715476p+0f);
    return fma(f, p, (float)e);
}

// log2 restricted to finite x >= 0 (no NaN/negative/inf branches): the hot
// path only takes pow of abs()/saturate()/distance values.
RT_HD float log2_nonneg(float x)
{
    if (x == 0.0f) return -__builtin_inff();
#if defined(__HIP_DEVICE_COMPILE__)
    int e;
    float m = __builtin_frexpf(x, &e); // m in [0.5,1), handles subnormals
    // frexp mantissa m in [0.5,1): our m' = 2m in [1,2), e' = e-1
    uint32_t mb = bits(m) + 0x00800000u;
    e -= 1;
#else
    uint32_t ix = bits(x);
    int e = 0;
    if (ix < 0x00800000u) {
        x = x * 8388608.0f;
        ix = bits(x);
        e = -23;
    }
    e += (int)(ix >> 23) - 127;
    uint32_t mb = (ix & 0x007fffffu) | 0x3f800000u;
#endif
    if (mb > 0x3fb504f3u) {
        mb -= 0x00800000u;
        e += 1;
    }
    float f = fbits(mb) - 1.0f;
    float p = -0x1.c362c0p-4f;
    p = fma(p, f, 0x1.7d9132p-3f);
    p = fma(p, f, -0x1.87381ap-3f);
    p = fma(p, f, 0x1.a2f85ep-3f);
    p = fma(p, f, -0x1.eabd64p-3f);
    p = fma(p, f, 0x1.277e9ap-2f);
    p = fma(p, f, -0x1.715a76p-2f);
    p = fma(p, f, 0x1.ec7094p-2f);
    p = fma(p, f, -0x1.715470p-1f);
    p = fma(p, f, 0x1.715476p+0f);
    return fma(f, p, (float)e);
}

// exp2 for finite arguments in the ranges the hot path produces (y*log2(x)
// with x >= 0 yields -inf for x == 0: mapped to 0 like exp2 above).
RT_HD float exp2_fin(float x)
{
    if (x < -150.0f) return 0.0f;
    if (x >= 128.0f) return __builtin_inff();
    float n = rint(x);
    float f = x - n;
    float p = 0x1.41a6fep-13f;
    p = fma(p, f, 0x1.5f44f0p-10f);
    p = fma(p, f, 0x1.3b2dfep-7f);
    p = fma(p, f, 0x1.c6aed6p-5f);
    p = fma(p, f, 0x1.ebfbdap-3f);
    p = fma(p, f, 0x1.62e430p-1f);
    p = fma(p, f, 1.0f);
    return __builtin_ldexpf(p, (int)n);
}

// pow_nonneg without control flow, for latency-bound code where a single wave's
// dependency chain is the critical path: every lane runs both polynomials and the
// special cases are selected afterwards, so it is bit-identical to pow_nonneg for
// x >= 0 finite and finite y > 0 (x == 0 -> log2 -inf -> exp2 0; the clamped
// exp2 argument only ever replaces results that are then selected away).
RT_HD float pow_nonneg_flat(float x, float y)
{
#if !defined(__HIP_DEVICE_COMPILE__)
    return exp2_fin(y * log2_nonneg(x));
#else
    int e;
    float m = __builtin_frexpf(x, &e);
    uint32_t mb = bits(m) + 0x00800000u;
    e -= 1;
    const bool hi = mb > 0x3fb504f3u;
    mb = hi ? mb - 0x00800000u : mb;
    e = hi ? e + 1 : e;
    float f = fbits(mb) - 1.0f;
    float p = -0x1.c362c0p-4f;
    p = fma(p, f, 0x1.7d9132p-3f);
    p = fma(p, f, -0x1.87381ap-3f);
    p = fma(p, f, 0x1.a2f85ep-3f);
    p = fma(p, f, -0x1.eabd64p-3f);
    p = fma(p, f, 0x1.277e9ap-2f);
    p = fma(p, f, -0x1.715a76p-2f);
    p = fma(p, f, 0x1.ec7094p-2f);
    p = fma(p, f, -0x1.715470p-1f);
    p = fma(p, f, 0x1.715476p+0f);
    const float lg = x == 0.0f ? -__builtin_inff() : fma(f, p, (float)e);
    const float a = y * lg;
    const float ac = min(max(a, -150.0f), 128.0f);
    const float n = rint(ac);
    const float g = ac - n;
    float q = 0x1.41a6fep-13f;
    q = fma(q, g, 0x1.5f44f0p-10f);
    q = fma(q, g, 0x1.3b2dfep-7f);
    q = fma(q, g, 0x1.c6aed6p-5f);
    q = fma(q, g, 0x1.ebfbdap-3f);
    q = fma(q, g, 0x1.62e430p-1f);
    q = fma(q, g, 1.0f);
    float r = __builtin_ldexpf(q, (int)n);
    r = a >= 128.0f ? __builtin_inff() : r;
    return a < -150.0f ? 0.0f : r;
#endif
}

RT_HD float pow(float x, float y) { return exp2(y * log2(x)); }
// pow for x >= 0 (abs/saturate/length bases) and finite y > 0.
RT_HD float pow_nonneg(float x, float y) { return exp2_fin(y * log2_nonneg(x)); }
RT_HD float exp(float x) { return exp2(x * 0x1.715476p+0f); }
RT_HD float exp_fin(float x) { return exp2_fin(x * 0x1.715476p+0f); }

RT_HD void sincos(float x, float* s, float* c)
{
    float k = rint(x * 0x1.45f306p-1f);
    float r = fma(-k, 0x1.921fb6p+0f, x);
    r = fma(-k, -0x1.777a5cp-25f, r);
    r = fma(-k, -0x1.000000p-49f, r);
    float u = r * r;
    float ps = fma(fma(-0x1.99071ap-13f, u, 0x1.110630p-7f), u, -0x1.555540p-3f);
    float sv = fma(r * u, ps, r);
    float pc = fma(fma(fma(0x1.9906cap-16f, u, -0x1.6c0786p-10f), u, 0x1.55553ap-5f), u, -0.5f);
    float cv = fma(u, pc, 1.0f);
    // quadrant k mod 4 with exact float ops (no out-of-range float->int conversion)
    int q = (int)(k - 4.0f * floor(k * 0.25f));
    float so = (q & 1) ? cv : sv;
    float co = (q & 1) ? sv : cv;
    if (q == 2 || q == 3) so = -so;
    if (q == 1 || q == 2) co = -co;
    *s = so;
    *c = co;
}
RT_HD float sin(float x)
{
    if (isnan_(x) || abs(x) == __builtin_inff()) return __builtin_nanf("");
    float s, c;
    sincos(x, &s, &c);
    return s;
}
RT_HD float cos(float x)
{
    if (isnan_(x) || abs(x) == __builtin_inff()) return __builtin_nanf("");
    float s, c;
    sincos(x, &s, &c);
    return c;
}

struct f3 {
    float x, y, z;
};
RT_HD f3 mk(float x, float y, float z)
{
    f3 r;
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}
RT_HD float dot(f3 a, f3 b) { return fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)); }
RT_HD float length(f3 a) { return sqrt(dot(a, a)); }
RT_HD f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD f3 scale(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RT_HD f3 normalize(f3 a) { return scale(a, rcp(sqrt(dot(a, a)))); }

} // namespace rtm
