/*
 * rt_oracle.c -- TEST INFRASTRUCTURE, NOT PRODUCT CODE (see rt_oracle.h).
 *
 * Plain-C restatement of the reference HLSL hot path.  Every function cites the
 * reference file:line it follows (paths relative to /root/reference/gpuraytrace).
 * Compile with -ffp-contract=off: every fused multiply-add below is explicit.
 *
 * Evaluation rules (the reference is HLSL cs_5_0 compiled by fxc; D3D11 leaves
 * mad fusion and transcendental precision to the implementation, so the
 * restatement fixes them, and the HIP kernels follow the same rules):
 *  R1  every arithmetic operator is one IEEE binary32 round-to-nearest-even op;
 *  R2  a product that feeds an add/sub in the dataflow (a*b+c, c-a*b, and HLSL
 *      lerp / mad) is ONE fused multiply-add (fxc emits `mad`); where two
 *      products feed one add, the left one is fused.  One site departs from
 *      that default and is fixed here as written: tracing.hlsl:54
 *      `RAY_STEP*stepmod*dirLength - dist*(1-RAY_STEP_FACTOR)` fuses the
 *      subtrahend's product, fma(-dist, 1-F, (0.03*stepmod)*dirLength) (the
 *      minuend is itself a two-multiply chain, so it is the one kept rounded;
 *      trace_ray below, rt_shader.h march_begin);
 *  R3  a / b = a * rcp(b), rcp = correctly rounded 1/b (fxc/D3D `div`);
 *  R4  dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)); length = sqrt(dot(v,v));
 *      normalize(v) = v * rcp(sqrt(dot(v,v))); mul(v,M) = dp4 fma chain;
 *      sqrt correctly rounded;
 *  R5  exp2/log2/sin/cos are the fixed polynomial implementations below;
 *      pow(x,y) = exp2(y*log2(x)) (pow(x, 2.0) literal = x*x); exp(x) = exp2(x*log2e);
 *  R6  max/min: a NaN operand yields the other operand, -0 < +0 (IEEE
 *      maximumNumber/minimumNumber); saturate(x) = min(max(x,0),1);
 *  R7  compile-time constants (`const static`) are folded in double from the
 *      float literals and rounded once to float;
 *  R8  (noise) gradperm is HLSL dot() under R4 with the permGradients values
 *      as given (any gradient table, not only Noise.cpp's {-1,0,1} set);
 *  R9  output quantisation to R8G8B8A8_UNORM: rint(saturate(c) * 255).
 */
#include "rt_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;

static inline f3 v3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------------ */
/* R6                                                                        */
float ro_max(float a, float b)
{
    if (a != a) return b;
    if (b != b) return a;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a; /* equal: prefer +0 */
}
float ro_min(float a, float b)
{
    if (a != a) return b;
    if (b != b) return a;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b; /* equal: prefer -0 */
}
static inline float sat(float x) { return ro_min(ro_max(x, 0.0f), 1.0f); }
static inline float rcp(float x) { return 1.0f / x; }

/* Arithmetic conventions of the HLSL-level operations (rules R2, R3, R5).  The default build is
 * the restatement the GPU matches bit for bit.  Convention VARIANTS (RO_CONV_*, built only as
 * separate checker libraries by `make -C oracle variants`, never linked into the product) re-evaluate
 * the same HLSL with another equally valid reading of it, to bound how far the D3D path's
 * unknowable choices (fxc mad fusion, div, transcendental precision) can move a frame
 * (scripts/parity_sensitivity.py, profiles/r03/parity_sensitivity.md):
 *   RO_CONV_UNFUSED  every HLSL a*b+c (mad, lerp, dot, mul, tracing.hlsl:54) as a rounded product
 *                    and a rounded add;
 *   RO_CONV_IEEEDIV  a / b as an IEEE division (not a * rcp(b)); normalize(v) = v / length(v);
 *   RO_CONV_LIBM     pow / exp / exp2 / log2 / sin / cos from the C library (glibc, ~0.5-1 ulp)
 *                    instead of the R5 polynomials.
 * MAD(a,b,c) = a*b + c; DIVADD(a,b,c) = a/b + c; DIVR(a,b) = a/b. */
#ifdef RO_CONV_UNFUSED
#define MAD(a, b, c) ((a) * (b) + (c))
#else
#define MAD(a, b, c) fmaf((a), (b), (c))
#endif
#ifdef RO_CONV_IEEEDIV
#define DIVR(a, b) ((a) / (b))
#define DIVADD(a, b, c) ((a) / (b) + (c))
#else
#define DIVR(a, b) ((a) * rcp(b))
#define DIVADD(a, b, c) MAD((a), rcp(b), (c))
#endif
static inline float lerp(float a, float b, float t) { return MAD(t, b - a, a); }

/* ------------------------------------------------------------------------ */
/* R5: polynomial transcendentals.  Coefficients are near-minimax fits,
 * written as hex floats so the HIP path can use the identical constants. */
float ro_exp2(float x)
{
#ifdef RO_CONV_LIBM
    return exp2f(x);
#endif
    if (x != x) return x;
    if (x >= 128.0f) return INFINITY;
    if (x < -150.0f) return 0.0f;
    float n = rintf(x);
    float f = x - n; /* exact, |f| <= 0.5 */
    float p = 0x1.41a6fep-13f;
    p = fmaf(p, f, 0x1.5f44f0p-10f);
    p = fmaf(p, f, 0x1.3b2dfep-7f);
    p = fmaf(p, f, 0x1.c6aed6p-5f);
    p = fmaf(p, f, 0x1.ebfbdap-3f);
    p = fmaf(p, f, 0x1.62e430p-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)n); /* one rounding (only for subnormal results) */
}

float ro_log2(float x)
{
#ifdef RO_CONV_LIBM
    return log2f(x);
#endif
    if (x != x) return x;
    if (x < 0.0f) return NAN;
    if (x == 0.0f) return -INFINITY;
    if (isinf(x)) return x;
    uint32_t ix = fbits(x);
    int e = 0;
    if (ix < 0x00800000u) { x *= 8388608.0f; ix = fbits(x); e = -23; }
    e += (int)(ix >> 23) - 127;
    uint32_t mb = (ix & 0x007fffffu) | 0x3f800000u;
    if (mb > 0x3fb504f3u) { mb -= 0x00800000u; e += 1; } /* m in [sqrt(.5), sqrt(2)] */
    float f = bitsf(mb) - 1.0f;                            /* exact */
    float p = -0x1.c362c0p-4f;
    p = fmaf(p, f, 0x1.7d9132p-3f);
    p = fmaf(p, f, -0x1.87381ap-3f);
    p = fmaf(p, f, 0x1.a2f85ep-3f);
    p = fmaf(p, f, -0x1.eabd64p-3f);
    p = fmaf(p, f, 0x1.277e9ap-2f);
    p = fmaf(p, f, -0x1.715a76p-2f);
    p = fmaf(p, f, 0x1.ec7094p-2f);
    p = fmaf(p, f, -0x1.715470p-1f);
    p = fmaf(p, f, 0x1.715476p+0f);
    return fmaf(f, p, (float)e);
}

#ifdef RO_CONV_LIBM
float ro_pow(float x, float y) { return powf(x, y); }
float ro_exp(float x) { return expf(x); }
#else
float ro_pow(float x, float y) { return ro_exp2(y * ro_log2(x)); }
float ro_exp(float x) { return ro_exp2(x * 0x1.715476p+0f); }
#endif

static void sincos_red(float x, float* s, float* c)
{
    float k = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(-k, 0x1.921fb6p+0f, x);
    r = fmaf(-k, -0x1.777a5cp-25f, r);
    r = fmaf(-k, -0x1.000000p-49f, r);
    float u = r * r;
    float ps = fmaf(fmaf(-0x1.99071ap-13f, u, 0x1.110630p-7f), u, -0x1.555540p-3f);
    float sv = fmaf(r * u, ps, r);
    float pc = fmaf(fmaf(fmaf(0x1.9906cap-16f, u, -0x1.6c0786p-10f), u, 0x1.55553ap-5f), u, -0.5f);
    float cv = fmaf(u, pc, 1.0f);
    /* quadrant k mod 4 with exact float ops (no out-of-range float->int conversion) */
    int q = (int)(k - 4.0f * floorf(k * 0.25f));
    switch (q) {
    case 0: *s = sv; *c = cv; break;
    case 1: *s = cv; *c = -sv; break;
    case 2: *s = -sv; *c = -cv; break;
    default: *s = -cv; *c = sv; break;
    }
}
#ifdef RO_CONV_LIBM
float ro_sin(float x) { return sinf(x); }
float ro_cos(float x) { return cosf(x); }
#else
float ro_sin(float x) { float s, c; if (x != x || isinf(x)) return NAN; sincos_red(x, &s, &c); return s; }
float ro_cos(float x) { float s, c; if (x != x || isinf(x)) return NAN; sincos_red(x, &s, &c); return c; }
#endif

void ro_batch_unary(int op, const float* x, float* y, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        float v = x[i];
        switch (op) {
        case 0: y[i] = ro_exp2(v); break;
        case 1: y[i] = ro_log2(v); break;
        case 2: y[i] = ro_exp(v); break;
        case 3: y[i] = ro_sin(v); break;
        case 4: y[i] = ro_cos(v); break;
        case 5: y[i] = sqrtf(v); break;
        case 6: y[i] = rcp(v); break;
        default: y[i] = rcp(sqrtf(v)); break;
        }
    }
}
void ro_batch_binary(int op, const float* a, const float* b, float* y, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        switch (op) {
        case 0: y[i] = ro_pow(a[i], b[i]); break;
        case 1: y[i] = ro_max(a[i], b[i]); break;
        default: y[i] = ro_min(a[i], b[i]); break;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* R4 vector helpers */
static inline float dot3(f3 a, f3 b) { return MAD(a.z, b.z, MAD(a.y, b.y, a.x * b.x)); }
static inline float len3(f3 a) { return sqrtf(dot3(a, a)); }
static inline f3 sub3(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 scale3(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
#ifdef RO_CONV_IEEEDIV
static inline f3 norm3(f3 a) { float l = sqrtf(dot3(a, a)); return v3(a.x / l, a.y / l, a.z / l); }
#else
static inline f3 norm3(f3 a) { return scale3(a, rcp(sqrtf(dot3(a, a)))); }
#endif

/* ------------------------------------------------------------------------ */
/* Noise tables: Graphics/Noise.cpp:6-24 (g3), :39-56 (generate), :58-61,
 * :63-80 (perm2D), :82-94 (gradients).  `rand` is the CRT's: MSVC LCG (the
 * reference's shipping platform, vcredist) or glibc TYPE_3 random(). */
static const float g3[16][3] = {
    {1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1}, {1, 0, -1}, {-1, 0, -1},
    {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}, {1, 1, 0}, {0, -1, 1}, {-1, 1, 0}, {0, -1, -1}};

typedef struct { int kind; uint32_t lcg; int32_t r[34]; int idx; uint32_t ring[34]; } crt_rand;

static void crt_srand(crt_rand* g, uint32_t seed, int kind)
{
    g->kind = kind;
    if (kind == RO_RAND_MSVC) { g->lcg = seed; return; }
    /* glibc srandom_r, TYPE_3: r[i] = 16807*r[i-1] mod (2^31-1), then 310 discards */
    int32_t r[344];
    r[0] = (int32_t)(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; ++i) {
        int64_t w = (16807LL * r[i - 1]) % 2147483647LL;
        if (w < 0) w += 2147483647LL;
        r[i] = (int32_t)w;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    uint32_t s[344];
    for (int i = 0; i < 34; ++i) s[i] = (uint32_t)r[i];
    for (int i = 34; i < 344; ++i) s[i] = s[i - 31] + s[i - 3];
    for (int i = 0; i < 34; ++i) g->ring[i] = s[310 + i]; /* last 34 values */
    g->idx = 0;
}

static int crt_rand_next(crt_rand* g)
{
    if (g->kind == RO_RAND_MSVC) {
        g->lcg = g->lcg * 214013u + 2531011u;
        return (int)((g->lcg >> 16) & 0x7fffu);
    }
    /* ring holds s[n-34 .. n-1]; s[n] = s[n-31] + s[n-3] */
    uint32_t v = g->ring[(g->idx + 3) % 34] + g->ring[(g->idx + 31) % 34];
    g->ring[g->idx] = v;
    g->idx = (g->idx + 1) % 34;
    return (int)(v >> 1);
}

void ro_noise_generate(ro_noise* out, uint32_t seed, int rand_kind)
{
    crt_rand g;
    memset(&g, 0, sizeof(g));
    crt_srand(&g, seed, rand_kind);
    int32_t* p = out->perm;
    for (int x = 0; x < 128; ++x) p[x] = x;
    for (int x = 0; x < 128; ++x) {
        int j = crt_rand_next(&g) % 128;
        int32_t t = p[x]; p[x] = p[j]; p[j] = t;
    }
    for (int x = 0; x < 128; ++x) {
        for (int y = 0; y < 128; ++y) {
            uint8_t* c = out->perm2d + (x + y * 128) * 4;
            int A = p[x % 128] + y;
            int B = p[(x + 1) % 128] + y;
            c[0] = (uint8_t)p[A % 128];
            c[1] = (uint8_t)p[(A + 1) % 128];
            c[2] = (uint8_t)p[B % 128];
            c[3] = (uint8_t)p[(B + 1) % 128];
        }
    }
    for (int x = 0; x < 128; ++x) {
        const float* gr = g3[p[x] % 16];
        out->grad[x * 4 + 0] = gr[0];
        out->grad[x * 4 + 1] = gr[1];
        out->grad[x * 4 + 2] = gr[2];
        out->grad[x * 4 + 3] = 0.0f;
    }
}

/* ------------------------------------------------------------------------ */
/* Per-evaluation context (cbuffers + counters). */
typedef struct {
    const ro_noise* nz;
    const ro_frame* fr;
    f3 eye, sun;
    float density_factor, step_factor, one_minus_step_factor, min_limit;
    uint64_t noise_calls, density_calls;
    float pixel_secondary_steps; /* shadow + AO march iterations of the current pixel (parity study) */
#ifdef RO_STUDY /* scripts/skip_study.c: which pixel / ray the samples belong to */
    int64_t study_pixel;
#endif
} ctx;

#ifdef RO_STUDY
static void ro_study_sample(ctx* c, f3 p, float d, int calcfog, int skiprefine, int max_steps, int iters,
                            float dist, float enddist, float step, float lastStep);
#endif

static void ctx_init(ctx* c, const ro_noise* nz, const ro_frame* fr)
{
    c->nz = nz;
    c->fr = fr;
    c->eye = v3(fr->eye[0], fr->eye[1], fr->eye[2]);
    c->sun = v3(fr->sun[0], fr->sun[1], fr->sun[2]);
    /* tracing.hlsl:32-41 (R7 folding) */
    c->density_factor = fr->recording ? 0.15f : 0.35f;
    c->step_factor = fr->recording ? 1.001f : 1.009f;
    c->one_minus_step_factor = (float)(1.0 - (double)c->step_factor);
    c->min_limit = (float)((double)0.02f * (double)0.03f);
    c->noise_calls = 0;
    c->density_calls = 0;
    c->pixel_secondary_steps = 0.0f;
#ifdef RO_STUDY
    c->study_pixel = -1;
#endif
}

/* noise.hlsl:145-150 gradperm: dot(permGradients[x % 128].xyz, p) under R4 */
static inline float gradperm(const ctx* c, uint32_t i, float x, float y, float z)
{
    const float* g = c->nz->grad + (i % 128u) * 4;
    return MAD(g[2], z, MAD(g[1], y, g[0] * x));
}

/* noise.hlsl:139-142 */
static inline float fade(float t) { return ((t * t) * t) * MAD(t, MAD(t, 6.0f, -15.0f), 10.0f); }

/* noise.hlsl:153-179 (the live `#if 1` block) */
static float noise3d(ctx* c, float px, float py, float pz)
{
    c->noise_calls++;
    float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
    int32_t Px = (int32_t)fx, Py = (int32_t)fy, Pz = (int32_t)fz;
    float x = px - fx, y = py - fy, z = pz - fz;
    float ux = fade(x), uy = fade(y), uz = fade(z);
    /* (TEXTURE_SIZE - |P|) % TEXTURE_SIZE for P<0, else P % 128  ==  P & 127 */
    uint32_t X = (uint32_t)Px & 127u, Y = (uint32_t)Py & 127u, Z = (uint32_t)Pz & 127u;
    const uint8_t* t = c->nz->perm2d + (X + Y * 128u) * 4u;
    uint32_t a0 = t[0] + Z, a1 = t[1] + Z, b0 = t[2] + Z, b1 = t[3] + Z; /* Pu.x, Pu.y, Pu.z, Pu.w */
    float x1 = x + -1.0f, y1 = y + -1.0f, z1 = z + -1.0f;
    float g000 = gradperm(c, a0, x, y, z);
    float g100 = gradperm(c, b0, x1, y, z);
    float g010 = gradperm(c, a1, x, y1, z);
    float g110 = gradperm(c, b1, x1, y1, z);
    float g001 = gradperm(c, a0 + 1u, x, y, z1);
    float g101 = gradperm(c, b0 + 1u, x1, y, z1);
    float g011 = gradperm(c, a1 + 1u, x, y1, z1);
    float g111 = gradperm(c, b1 + 1u, x1, y1, z1);
    float l0 = lerp(lerp(g000, g100, ux), lerp(g010, g110, ux), uy);
    float l1 = lerp(lerp(g001, g101, ux), lerp(g011, g111, ux), uy);
    return lerp(l0, l1, uz);
}

float ro_noise3d(const ro_noise* nz, float x, float y, float z)
{
    ro_frame fr;
    memset(&fr, 0, sizeof(fr));
    ctx c;
    ctx_init(&c, nz, &fr);
    return noise3d(&c, x, y, z);
}

void ro_noise3d_batch(const ro_noise* nz, const float* xyz, float* out, int64_t n)
{
    ro_frame fr;
    memset(&fr, 0, sizeof(fr));
    ctx c;
    ctx_init(&c, nz, &fr);
    for (int64_t i = 0; i < n; ++i) out[i] = noise3d(&c, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
}

/* ------------------------------------------------------------------------ */
/* FBM octave scales: pow(LUCAN, N) evaluated as at run time (R5). */
static float fbm_scale(float lucan, int n) { return ro_pow(lucan, (float)n); }

/* Media/nomadplains/shaders/terrain.hlsl:8-39 */
static float density_nomadplains(ctx* c, f3 p)
{
    float dist = ro_max(len3(sub3(p, c->eye)), 0.01f);
    float d = -p.y;
    f3 p1 = scale3(p, 0.4f);
    float s = 0.0f;
    float detail = ro_max(18.0f - ro_pow(dist, 0.33f), 2.0f);
    f3 q0 = scale3(p1, 0.006f);
    for (int N = 1; (float)N <= detail; ++N) {
        float S = fbm_scale(1.96f, N);
        float n = noise3d(c, q0.x * S, q0.y * (S * 0.35f), q0.z * S);
        s = DIVADD(n, S, s); /* s += noise/SCALE  (R2, R3) */
    }
    const float mountains = 0.1f;
    float expo = 0.68f + mountains;
    s = ro_pow(fabsf(MAD(s, 30.0f, 1.0f)) * 35.0f, expo); /* s*=30; pow(abs(s+1)*35, .68+m) */
    float steep = sat((noise3d(c, p1.x * 0.007138f, p1.z * 0.007138f, 0.0f) - 0.2f) * 6.0f) * 7.5f;
    float floorsize = steep * 1.8f;
    float t;
    t = sat((p1.y - 13.0f) * steep); s = MAD(-(t * t), floorsize, s);
    t = sat((p1.y - 16.0f) * steep); s = MAD(-(t * t), floorsize, s);
    t = sat((p1.y - 19.0f) * steep); s = MAD(-(t * t), floorsize, s);
    t = sat((p1.y - 22.0f) * steep); s = MAD(-(t * t), floorsize, s);
    s = MAD(ro_pow(sat((-p1.y + 10.0f) * 1.6f), 1.5f), 19.0f, s);
    return d + s;
}

/* Media/testing/shaders/terrain.hlsl:6-36 */
static float density_testing(ctx* c, f3 p)
{
    (void)c;
    float d = -p.y;
    return MAD(ro_sin(p.x * 0.1f) * ro_cos(p.z * 0.1f), 10.0f, d);
}

/* Media/simple/shaders/terrain.hlsl:7-48 */
static float density_simple(ctx* c, f3 p)
{
    float d = -p.y;
    f3 q = scale3(p, 0.006f);
    float n = noise3d(c, q.x * 1.0f, q.y * 0.0f, q.z * 1.0f) * 150.0f;
    f3 q2 = scale3(p, 0.002f);
    float w2 = ro_min(ro_max(MAD(-p.y, 1.5f, 50.0f), 0.0f), 36.0f);
    n = MAD(-MAD(noise3d(c, q2.x, q2.y, q2.z), 0.5f, 0.5f), w2, n);
    f3 q3 = scale3(p, 0.003f);
    float w3 = ro_min(ro_max(MAD(-p.y, 1.5f, 10.0f), 0.0f), 36.0f);
    n = MAD(-MAD(noise3d(c, q3.x, q3.y, q3.z), 0.5f, 0.5f), w3, n);
    /* `dist` is computed but unused (terrain.hlsl:37) */
    f3 q4 = scale3(p, 0.06f);
    for (int N = 1; (float)N <= 1.0f; ++N) {
        float S = fbm_scale(1.96f, N);
        n = DIVADD(noise3d(c, q4.x * S, q4.y * (S * 0.35f), q4.z * S), S, n);
    }
    return d + n;
}

/* Media/greenrocks/shaders/terrain.hlsl:4-32 */
static float density_greenrocks(ctx* c, f3 p)
{
    p.y = p.y - 170.0f;
    float d = 0.0f;
    d = d + -p.y;
    f3 pg = scale3(p, 0.01f);
    float g = noise3d(c, pg.x, pg.y, pg.z);
    f3 noh = v3(1.0f, MAD(fabsf(g), 1.4f, 0.1f), 1.0f);
    f3 pc = v3(p.x * 0.011f, p.y * 0.0013f, p.z * 0.011f);
    float g32 = g * 0.32f;
    for (int N = 1; (float)N <= 7.0f; ++N) {
        float S = fbm_scale(2.0f, N);
        float n = noise3d(c, MAD(pc.x, S, g32), MAD(pc.y, S, g32), MAD(pc.z, S, g32));
        d = DIVADD((fabsf(n) * 210.0f) * g, S, d);
    }
    d = d - 50.0f;
    f3 p2 = scale3(p, 0.002f);
    f3 p2n = v3(p2.x * noh.x, p2.y * noh.y, p2.z * noh.z);
    for (int N = 1; (float)N <= 5.0f; ++N) {
        float S = fbm_scale(2.0f, N);
        float n = noise3d(c, p2n.x * S, p2n.y * S, p2n.z * S);
        float inner = MAD(n + 0.1f, 0.5f, 0.5f);
        d = MAD(-inner, DIVR(220.0f, S), d);
    }
    return d;
}

static float get_density(ctx* c, f3 p)
{
    c->density_calls++;
    switch (c->fr->landscape) {
    case RO_TESTING: return density_testing(c, p);
    case RO_SIMPLE: return density_simple(c, p);
    case RO_GREENROCKS: return density_greenrocks(c, p);
    default: return density_nomadplains(c, p);
    }
}

/* getFog: nomadplains terrain.hlsl:42-45 returns 0; testing/simple return 0
 * before the live code (testing :56, simple :68); greenrocks :34-54 is live. */
static int fog_live(const ctx* c) { return c->fr->landscape == RO_GREENROCKS; }

static f4 get_fog(ctx* c, f3 p, float dist)
{
    f4 r = {0.0f, 0.0f, 0.0f, 0.0f};
    if (!fog_live(c)) return r;
    float fogd = 0.0f;
    float d = 0.0f;
    dist = sat(MAD(-dist, 0.0012f, 1.0f));
    float falloff = sat(MAD(-(dist * dist), 0.1f, 1.0f));
    if (falloff > 0.0f) {
        d = d + sat((-p.y - 2.0f) * 0.0003f);
        f3 q = scale3(p, 0.1261f);
        fogd = MAD(fabsf(noise3d(c, q.x, q.y, q.z)), 0.2f, 0.8f);
    }
    float fc = 0.9f * fogd;
    r.x = (fc * d) * dist;
    r.y = (fc * d) * dist;
    r.z = (fc * d) * dist;
    r.w = d * dist;
    return r;
}

/* ------------------------------------------------------------------------ */
typedef struct { f4 pd; f4 fcolord; float density; float steps; } ray_result;

/* Media/common/shaders/tracing.hlsl:47-105 (+ build extension max_steps) */
static ray_result trace_ray(ctx* c, f3 p, float dist, float enddist, float stepmod, f3 dir,
                            int calcfog, int skiprefine, int max_steps)
{
    ray_result rr;
    f4 f = {0.0f, 0.0f, 0.0f, 0.0f};
    float d = 0.0f;
    float total = 0.0f;
    float dirLength = len3(dir);
    /* tracing.hlsl:54: the R2 exception (the subtrahend's product is the fused one) */
    float step = MAD(-dist, c->one_minus_step_factor, (0.03f * stepmod) * dirLength);
    float lastStep = step;
    dir = v3(DIVR(dir.x, dirLength), DIVR(dir.y, dirLength), DIVR(dir.z, dirLength));
    if (calcfog) {
        float hd = dist * 0.5f;
        f3 mp = v3(MAD(dir.x * dist, 0.5f, p.x), MAD(dir.y * dist, 0.5f, p.y), MAD(dir.z * dist, 0.5f, p.z));
        f4 mf = get_fog(c, mp, hd);
        f.x = MAD(mf.x, dist, f.x); f.y = MAD(mf.y, dist, f.y);
        f.z = MAD(mf.z, dist, f.z); f.w = MAD(mf.w, dist, f.w);
    }
    f3 rayp = v3(0.0f, 0.0f, 0.0f);
    int iters = 0;
    while (dist < enddist && step > c->min_limit) {
        if (max_steps > 0 && iters >= max_steps) break;
        ++iters;
        total = total + 1.0f;
        rayp = v3(MAD(dir.x, dist, p.x), MAD(dir.y, dist, p.y), MAD(dir.z, dist, p.z));
        f4 fs = {0.0f, 0.0f, 0.0f, 0.0f};
        d = get_density(c, rayp);
#ifdef RO_STUDY
        ro_study_sample(c, rayp, d, calcfog, skiprefine, max_steps, iters, dist, enddist, step, lastStep);
#endif
        if (calcfog) {
            f4 g = get_fog(c, rayp, dist);
            fs.x = g.x * step; fs.y = g.y * step; fs.z = g.z * step; fs.w = g.w * step;
        }
        if (d > 0.0f) {
            if (skiprefine) break;
            dist = dist - lastStep;
            step = step * 0.3f;
            f.x = f.x - fs.x; f.y = f.y - fs.y; f.z = f.z - fs.z; f.w = f.w - fs.w;
        } else {
            float stepmult = 1.0f + ro_pow(fabsf(ro_min(d + 5.0f, 0.0f)), c->density_factor);
            step = step * c->step_factor;
            lastStep = step * stepmult;
            dist = dist + lastStep;
            f.x = f.x + fs.x; f.y = f.y + fs.y; f.z = f.z + fs.z; f.w = f.w + fs.w;
        }
    }
    rr.pd.x = rayp.x; rr.pd.y = rayp.y; rr.pd.z = rayp.z; rr.pd.w = dist;
    rr.fcolord = f;
    rr.density = d;
    rr.steps = total;
    return rr;
}

/* tracing.hlsl:107-116 */
static f3 get_normal(ctx* c, f4 pd)
{
    f3 p = v3(pd.x, pd.y, pd.z);
    float dist = len3(sub3(p, c->eye));
    float nd = dist * 0.005f;
    float dx = get_density(c, v3(p.x - nd, p.y - 0.0f, p.z - 0.0f)) - pd.w;
    float dy = get_density(c, v3(p.x - 0.0f, p.y - nd, p.z - 0.0f)) - pd.w;
    float dz = get_density(c, v3(p.x - 0.0f, p.y - 0.0f, p.z - nd)) - pd.w;
    return norm3(v3(dx, dy, dz));
}

/* tracing.hlsl:124-134 */
static void get_pixel_ray(const ctx* c, float px, float py, f3* outp, f3* outdir)
{
    const ro_frame* fr = c->fr;
    float sx = DIVADD(px + 0.5f, (float)fr->width, -0.5f) * 2.0f;
    float sy = DIVADD(py + 0.5f, (float)fr->height, -0.5f) * 2.0f;
    sx = sx * fr->projection[5]; /* Projection._22 */
    sy = sy * fr->projection[0]; /* Projection._11 */
    const float* m = fr->view_inverse;
    float r[3];
    for (int j = 0; j < 3; ++j)
        r[j] = MAD(1.0f, m[12 + j], MAD(1.0f, m[8 + j], MAD(sy, m[4 + j], sx * m[j])));
    *outp = v3(r[0], r[1], r[2]);
    *outdir = sub3(*outp, c->eye);
}

/* ------------------------------------------------------------------------ */
/* Media/common/shaders/sky.hlsl */
typedef struct { f3 mie, rayleigh; } sky_color;

typedef struct {
    float outerRadius, fScale, scaleOverScaleDepth, fKrESun, fKmESun, fKr4PI, fKm4PI;
    float invWL[3], att_k[3], mieK[3], g, g2, mie_a, one_plus_g2, two_g, rcp_samples;
} sky_consts;

static void sky_init(sky_consts* k)
{
    /* sky.hlsl:1-16, :74-80 folded per R7 */
    const double wl[3] = {0.650f, 0.570f, 0.475f};
    const double kr = 0.003f, km = 0.0025f, pi = 3.14159265f, eSun = 12.0f;
    k->outerRadius = (float)(200.0 * (double)1.025f);
    k->fScale = (float)(1.0 / ((double)k->outerRadius - 200.0));
    k->scaleOverScaleDepth = (float)((double)k->fScale / (double)0.19f);
    k->fKrESun = (float)(eSun * kr);
    k->fKmESun = (float)(eSun * km);
    k->fKr4PI = (float)(kr * 4.0 * pi);
    k->fKm4PI = (float)(km * 4.0 * pi);
    for (int i = 0; i < 3; ++i) {
        float wl4 = (float)pow(wl[i], 4.0);
        k->invWL[i] = (float)(1.0 / (double)wl4);
        /* exp(-fScatter * (v3InvWavelength * fKr4PI + fKm4PI)): constant vector (R2, R7) */
        k->att_k[i] = (float)((double)k->invWL[i] * (double)k->fKr4PI + (double)k->fKm4PI);
        k->mieK[i] = (float)((double)k->invWL[i] * (double)k->fKrESun);
    }
    k->g = -0.99f;
    k->g2 = k->g * k->g;
    k->mie_a = (float)(1.5 * ((1.0 - (double)k->g2) / (2.0 + (double)k->g2)));
    k->one_plus_g2 = (float)(1.0 + (double)k->g2);
    k->two_g = (float)(2.0 * (double)k->g);
    k->rcp_samples = (float)(1.0 / 3.0);
}

/* sky.hlsl:18-23 */
static f3 mod_ray_dir(f3 d) { return norm3(v3(d.x, sat(d.y), d.z)); }

/* sky.hlsl:26-36 */
static float get_space_color(ctx* c, f3 dir)
{
    dir = mod_ray_dir(dir);
    if (dir.y <= 0.0f) return 0.0f;
    float space = noise3d(c, dir.x * 500.0f, dir.y * 500.0f, dir.z * 500.0f);
    space = space - MAD(noise3d(c, dir.x * 150.2f, dir.y * 150.2f, dir.z * 150.2f), 0.5f, 0.13f);
    space = space - MAD(noise3d(c, dir.x * 200.2f, dir.y * 200.2f, dir.z * 200.2f), 0.5f, 0.5f);
    return (space * 1.0f) * sat(MAD(-c->sun.y, 2.7f, -0.5f));
}

/* sky.hlsl:39-43 */
static float sky_scale(float fCos)
{
    float x = 1.0f - fCos;
    float t = MAD(x, 5.25f, -6.80f);
    t = MAD(x, t, 3.83f);
    t = MAD(x, t, 0.459f);
    t = MAD(x, t, -0.00287f);
    return 0.19f * ro_exp(t);
}

/* sky.hlsl:83-137 (with applyPhase :64-72, phases :46-55; note the swapped
 * mie/rayleigh arguments at :131) */
static sky_color get_rayleigh_mie(const ctx* c, const sky_consts* k, f3 org)
{
    f3 rd = mod_ray_dir(org);
    float camHeight = MAD(c->eye.y, 0.001f, 200.0f);
    camHeight = ro_max(camHeight, 0.0f);
    float distToTop = k->outerRadius - camHeight;
    float far = MAD((1.0f - rd.y) * distToTop, 2.0f, distToTop);
    f3 start = v3(c->eye.x * 0.001f, camHeight, c->eye.z * 0.001f);
    float depth = ro_exp(k->scaleOverScaleDepth * (200.0f - camHeight));
    float fStartAngle = dot3(rd, norm3(start));
    float fStartOffset = depth * sky_scale(fStartAngle);
    float sampleLength = DIVR(far, 3.0f); /* far / fSamples; rcp(3.0f) == k->rcp_samples */
    float scaledLength = sampleLength * k->fScale;
    f3 sampleRay = scale3(rd, sampleLength);
    f3 sp = v3(MAD(sampleRay.x, 0.5f, start.x), MAD(sampleRay.y, 0.5f, start.y), MAD(sampleRay.z, 0.5f, start.z));
    float front[3] = {0.0f, 0.0f, 0.0f};
    for (int i = 0; i < 3; ++i) {
        float height = len3(sp);
        float dep = ro_exp(k->scaleOverScaleDepth * (200.0f - height));
        float fLight = DIVR(dot3(c->sun, sp), height);
        float fCam = DIVR(dot3(rd, sp), height);
        float fScatter = MAD(dep, sky_scale(fLight) - sky_scale(fCam), fStartOffset);
        float ds = dep * scaledLength;
        for (int j = 0; j < 3; ++j) {
            float att = ro_exp(-fScatter * k->att_k[j]);
            front[j] = MAD(att, ds, front[j]);
        }
        sp = v3(sp.x + sampleRay.x, sp.y + sampleRay.y, sp.z + sampleRay.z);
    }
    f3 mie = v3(front[0] * k->mieK[0], front[1] * k->mieK[1], front[2] * k->mieK[2]);
    f3 ray = v3(front[0] * k->fKmESun, front[1] * k->fKmESun, front[2] * k->fKmESun);
    f3 t = v3(-rd.x * far, -rd.y * far, -rd.z * far);
    /* applyPhase(rayleigh := mie, mie := ray, camDir := t) */
    float fCos = DIVR(dot3(c->sun, t), len3(t));
    float fCos2 = fCos * fCos;
    float mphase = DIVR(k->mie_a * (1.0f + fCos2), ro_pow(fabsf(MAD(-k->two_g, fCos, k->one_plus_g2)), 1.5f));
    float rphase = MAD(0.75f, fCos2, 0.75f);
    sky_color sc;
    sc.mie = scale3(ray, mphase);
    sc.rayleigh = scale3(mie, rphase);
    float m = sat(MAD(org.y, 0.5f, 0.5f) * 4.0f);
    sc.rayleigh = scale3(sc.rayleigh, m);
    float sy = sat(c->sun.y);
    sc.rayleigh.z = MAD(0.6f, sy, sc.rayleigh.z);
    sc.rayleigh.y = MAD(0.4f, sy, sc.rayleigh.y);
    sc.rayleigh.x = MAD(0.3f, sy, sc.rayleigh.x);
    return sc;
}

/* sky of n view directions for the known-answer tests: (mie.rgb, rayleigh.rgb, space) each */
void ro_sky(const ro_noise* nz, const ro_frame* fr, const float* dirs, float* out, int64_t n)
{
    sky_consts k;
    sky_init(&k);
    ctx c;
    ctx_init(&c, nz, fr);
    for (int64_t i = 0; i < n; ++i) {
        f3 d = v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        sky_color sc = get_rayleigh_mie(&c, &k, d);
        float* o = out + 7 * i;
        o[0] = sc.mie.x; o[1] = sc.mie.y; o[2] = sc.mie.z;
        o[3] = sc.rayleigh.x; o[4] = sc.rayleigh.y; o[5] = sc.rayleigh.z;
        o[6] = get_space_color(&c, d);
    }
}

/* ------------------------------------------------------------------------ */
/* getColor: Media/nomadplains/shaders/color.hlsl:8-72 (default),
 * testing/color.hlsl:12-44, simple/color.hlsl:8-74, greenrocks/color.hlsl:12-43 */
static f3 get_color(ctx* c, f3 p, f3 n, f3 d, float dist, uint64_t* shadow_steps)
{
    int ls = c->fr->landscape;
    float col[4];
    float spec_n_dot;
    if (ls == RO_NOMADPLAINS || ls == RO_SIMPLE) {
        /* blend / n1 / the 4- and 8-octave FBM are dead code (results unused) */
        col[0] = (float)(193.0 / 255.0); col[1] = (float)(131.0 / 255.0); col[2] = (float)(92.0 / 255.0); col[3] = 0.0f;
        float s = 0.0f;
        if (ls == RO_NOMADPLAINS) {
            f3 q = v3(p.y * 0.5f, p.x * 0.01f, p.z * 0.01f);
            for (int N = 1; (float)N <= 20.0f; ++N) {
                float S = fbm_scale(2.03f, N);
                s = DIVADD(fabsf(noise3d(c, q.x * S, q.y * S, q.z * S)), S, s);
            }
            for (int i = 0; i < 4; ++i) col[i] = MAD(-s, 0.5f, col[i]);
        } else {
            float detail = ro_max(16.0f - ro_pow(dist, 0.33f), 2.0f);
            f3 q = v3(p.y * 0.5f, p.x * 0.01f, p.z * 0.1f);
            for (int N = 1; (float)N <= detail; ++N) {
                float S = fbm_scale(2.03f, N);
                s = DIVADD(fabsf(noise3d(c, q.x * S, q.y * S, q.z * S)), S, s);
            }
            float w = ro_max(DIVR(200.0f - dist, 200.0f), 0.0f);
            for (int i = 0; i < 4; ++i) col[i] = MAD(-s, w, col[i]);
        }
        col[3] = 0.2f;
        f3 md = v3(-d.x, -d.y, -d.z);
        /* reflect(n, -d) = n - 2*dot(n,-d)*(-d) */
        float t2 = dot3(n, md);
        t2 = t2 + t2;
        f3 r = v3(MAD(-t2, md.x, n.x), MAD(-t2, md.y, n.y), MAD(-t2, md.z, n.z));
        spec_n_dot = dot3(c->sun, r);
    } else if (ls == RO_TESTING) {
        col[0] = 0.6f; col[1] = 0.5f; col[2] = 0.3f; col[3] = 0.1f;
        spec_n_dot = dot3(v3(-d.x, -d.y, -d.z), n);
    } else {
        col[0] = 0.6f; col[1] = 0.7f; col[2] = 0.3f; col[3] = 0.1f;
        spec_n_dot = dot3(v3(-d.x, -d.y, -d.z), n);
    }
    float brightness = dot3(n, c->sun);
    float mipf = ro_max(0.5f * ro_log2(dist), 0.0f);
    float precision = ro_max((mipf - 3.2f) * 3.0f, 1.0f) * 8.0f;
    ray_result rr = trace_ray(c, p, 0.4f, 100.0f, precision, c->sun, 1, 1, 0);
    *shadow_steps += (uint64_t)rr.steps;
    c->pixel_secondary_steps += rr.steps;
    if (rr.density > 0.0f) brightness = brightness * 0.1f;
    else brightness = sat(brightness - rr.fcolord.w);
    float specular = sat(ro_pow(ro_max(spec_n_dot, 0.0f), 40.0f)) * col[3];
    col[0] = col[0] + specular; col[1] = col[1] + specular; col[2] = col[2] + specular;
    /* color *= lerp(SHADOW_COLOR, 1, brightness): 1 - SHADOW_COLOR folded (R7) */
    static const float shc[4] = {0.08f, 0.12f, 0.14f, 0.6f};
    f3 out;
    float m[3];
    for (int i = 0; i < 3; ++i) m[i] = MAD(brightness, (float)(1.0 - (double)shc[i]), shc[i]);
    out.x = col[0] * m[0]; out.y = col[1] * m[1]; out.z = col[2] * m[2];
    return out;
}

/* ------------------------------------------------------------------------ */
/* antialiasing.hlsl:9-59 */
static const float aa_offsets_1[1][2] = {{0, 0}};
static const float aa_offsets_2[2][2] = {{4, 4}, {-4, -4}};
static const float aa_offsets_4[4][2] = {{-2, -6}, {6, -2}, {-6, 2}, {2, 6}};
static const float aa_offsets_8[8][2] = {{1, -3}, {-1, 3}, {5, 1}, {-3, -5}, {-5, 5}, {-7, -1}, {3, 7}, {7, -7}};
static const float aa_offsets_16[16][2] = {{1, 1}, {-1, 3}, {-3, 2}, {4, -1}, {-5, -2}, {2, 5}, {5, 3}, {3, -5},
                                           {-2, 6}, {0, -7}, {-4, -6}, {-6, 4}, {-8, 0}, {7, -4}, {6, 7}, {-7, -8}};
static const float (*aa_table(int n))[2]
{
    switch (n) {
    case 2: return aa_offsets_2;
    case 4: return aa_offsets_4;
    case 8: return aa_offsets_8;
    case 16: return aa_offsets_16;
    default: return aa_offsets_1;
    }
}

/* ------------------------------------------------------------------------ */
/* Build extension, BASELINE.json configs C3/C5 ("1-bounce AO"); the reference has
 * no ambient occlusion, so this definition is the build's own and
 * the GPU implements it identically:
 *   for each primary hit and k = 0..AO-1, one cosine-weighted hemisphere ray about
 *   the surface normal, direction from a PCG hash of (pixel, AA sample, k), marched
 *   like a shadow ray (traceRay(p, 0.4, 25, shadow stepmod, dir, no fog, skiprefine));
 *   ao = 1 - 0.6 * occluded / AO multiplies the saturated sample colour. */
#define RO_AO_END 25.0f
#define RO_AO_STRENGTH 0.6f

static uint32_t pcg_hash(uint32_t x)
{
    uint32_t st = x * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}

static f3 cross3(f3 a, f3 b)
{
    return v3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}

static f3 ao_dir(f3 n, uint32_t px, uint32_t py, uint32_t a, uint32_t k)
{
    uint32_t h = pcg_hash((px * 0x9E3779B1u) ^ (py * 0x85EBCA77u) ^ ((a * 16u + k) * 0xC2B2AE3Du));
    uint32_t h2 = pcg_hash(h);
    float u1 = (float)(h >> 8) * 0x1p-24f, u2 = (float)(h2 >> 8) * 0x1p-24f;
    float r = sqrtf(u1);
    float sn, cs;
    sincos_red(u2 * 6.2831855f, &sn, &cs);
    float sx = r * cs, sy = r * sn, sz = sqrtf(ro_max(1.0f - u1, 0.0f));
    f3 up = fabsf(n.x) > 0.9f ? v3(0.0f, 1.0f, 0.0f) : v3(1.0f, 0.0f, 0.0f);
    f3 tx = norm3(cross3(up, n));
    f3 ty = cross3(n, tx);
    return v3(fmaf(tx.x, sx, fmaf(ty.x, sy, n.x * sz)), fmaf(tx.y, sx, fmaf(ty.y, sy, n.y * sz)),
              fmaf(tx.z, sx, fmaf(ty.z, sy, n.z * sz)));
}

/* color.hlsl:47-50: the shadow ray's stepmod, reused by the AO rays */
static float shadow_precision(float dist)
{
    float mipf = ro_max(0.5f * ro_log2(dist), 0.0f);
    return ro_max((mipf - 3.2f) * 3.0f, 1.0f) * 8.0f;
}

static float ambient_occlusion(ctx* c, f3 p, f3 n, float dist, uint32_t px, uint32_t py, uint32_t a,
                               uint64_t* ao_steps, uint64_t* ao_rays)
{
    int ao = c->fr->ao_samples;
    float prec = shadow_precision(dist);
    int occ = 0;
    for (int k = 0; k < ao; ++k) {
        ray_result rr = trace_ray(c, p, 0.4f, RO_AO_END, prec, ao_dir(n, px, py, a, (uint32_t)k), 0, 1, 0);
        *ao_steps += (uint64_t)rr.steps;
        c->pixel_secondary_steps += rr.steps;
        *ao_rays += 1;
        if (rr.density > 0.0f) occ += 1;
    }
    return fmaf(-RO_AO_STRENGTH, (float)occ * rcp((float)ao), 1.0f);
}

/* tracescreen.hlsl:16-48 */
static f3 trace_sample(ctx* c, const sky_consts* k, f3 pp, f3 pdir, f3 pdn, float plane_x, float plane_y,
                       float* steps_out, uint64_t* prim_steps, uint64_t* hits, uint64_t* shadow_steps,
                       uint32_t px, uint32_t py, uint32_t a, float* ao_out, uint64_t* ao_steps, uint64_t* ao_rays)
{
    *ao_out = 1.0f;
    ray_result rr = trace_ray(c, pp, plane_x, plane_y, 1.0f, pdir, 1, 0, c->fr->max_steps);
    *steps_out += rr.steps;
    *prim_steps += (uint64_t)rr.steps;
    float skyAmount = rr.pd.w * 0.0005f;
    skyAmount = sat(skyAmount * skyAmount);
    sky_color scat = get_rayleigh_mie(c, k, pdn);
    f3 color;
    if (rr.density > 0.0f) {
        *hits += 1;
        f4 npd = {rr.pd.x, rr.pd.y, rr.pd.z, rr.density}; /* getNormal(float4(rr.pd.xyz, rr.density)) :31 */
        f3 n = get_normal(c, npd);
        color = get_color(c, v3(rr.pd.x, rr.pd.y, rr.pd.z), n, pdn, rr.pd.w, shadow_steps);
        if (c->fr->ao_samples > 0)
            *ao_out = ambient_occlusion(c, v3(rr.pd.x, rr.pd.y, rr.pd.z), n, rr.pd.w, px, py, a, ao_steps, ao_rays);
        color = v3(lerp(color.x, rr.fcolord.x, rr.fcolord.w), lerp(color.y, rr.fcolord.y, rr.fcolord.w),
                   lerp(color.z, rr.fcolord.z, rr.fcolord.w));
        color = v3(lerp(color.x, scat.rayleigh.x, skyAmount), lerp(color.y, scat.rayleigh.y, skyAmount),
                   lerp(color.z, scat.rayleigh.z, skyAmount));
    } else {
        float space = get_space_color(c, pdn);
        f3 sky = v3((scat.mie.x + scat.rayleigh.x) + space, (scat.mie.y + scat.rayleigh.y) + space,
                    (scat.mie.z + scat.rayleigh.z) + space);
        color = v3(lerp(sky.x, rr.fcolord.x, rr.fcolord.w), lerp(sky.y, rr.fcolord.y, rr.fcolord.w),
                   lerp(sky.z, rr.fcolord.z, rr.fcolord.w));
        color = v3(lerp(color.x, sky.x, skyAmount), lerp(color.y, sky.y, skyAmount), lerp(color.z, sky.z, skyAmount));
    }
    return color;
}

/* camerarays.hlsl:12-21 */
void ro_camerarays(const ro_noise* nz, const ro_frame* fr, float* camera_results, ro_stats* st)
{
    ro_camerarays_steps(nz, fr, camera_results, NULL, st);
}

void ro_camerarays_steps(const ro_noise* nz, const ro_frame* fr, float* camera_results, float* steps_out,
                         ro_stats* st)
{
    uint64_t noise = 0, steps = 0, dens = 0;
    int nt = fr->threads > 0 ? fr->threads : 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : noise, steps, dens) num_threads(nt ? nt : omp_get_max_threads())
    for (int i = 0; i < 1024; ++i) {
        ctx c;
        ctx_init(&c, nz, fr);
        int tx = i % 32, ty = i / 32;
        uint32_t pxs = (uint32_t)(DIVR((float)tx, 31.0f) * (float)fr->width);
        uint32_t pys = (uint32_t)(DIVR((float)ty, 31.0f) * (float)fr->height);
        f3 p, dir;
        get_pixel_ray(&c, (float)pxs, (float)pys, &p, &dir);
        ray_result rr = trace_ray(&c, p, 0.01f, 5000.0f, 2.0f, dir, 0, 1, 0);
        if (rr.density < 0.0f) rr.pd.w = 5000.0f;
        camera_results[4 * i + 0] = rr.pd.x;
        camera_results[4 * i + 1] = rr.pd.y;
        camera_results[4 * i + 2] = rr.pd.z;
        camera_results[4 * i + 3] = rr.pd.w;
        if (steps_out) steps_out[i] = rr.steps;
        noise += c.noise_calls;
        dens += c.density_calls;
        steps += (uint64_t)rr.steps;
    }
    if (st) { st->noise3d_calls += noise; st->prepass_steps += steps; st->density_calls += dens; }
}

/* Terrain.cpp:356-396 */
static float get_depth(const float* cr, int x, int y)
{
    if (x < 0) x = 0;
    if (x >= 32) x = 31;
    if (y < 0) y = 0;
    if (y >= 32) y = 31;
    return cr[(y * 32 + x) * 4 + 3];
}
static float get_depth_interp(const float* cr, int x, int y)
{
    if (x < 0) { float m = get_depth(cr, x + 1, y); float d = get_depth(cr, x + 2, y) - m; return m - d; }
    if (x >= 32) { float m = get_depth(cr, x - 1, y); float d = get_depth(cr, x - 2, y) - m; return m - d; }
    if (y < 0) { float m = get_depth(cr, x, y + 1); float d = get_depth(cr, x, y + 2) - m; return m - d; }
    if (y >= 32) { float m = get_depth(cr, x, y - 1); float d = get_depth(cr, x, y - 2) - m; return m - d; }
    return get_depth(cr, x, y);
}
/* Terrain.cpp:398-439 (std::min/std::max argument order kept) */
void ro_set_target_depths(const float* cr, float* cell)
{
    for (int x = 0; x < 1024; ++x) {
        int xpos = x % 32, ypos = x / 32;
        float dmin = get_depth_interp(cr, xpos, ypos);
        float dmax = dmin;
        for (int xp = -2; xp <= 2; ++xp) {
            for (int yp = -2; yp <= 2; ++yp) {
                float d = get_depth_interp(cr, xpos + xp, ypos + yp);
                dmin = (dmin < d) ? dmin : d;  /* std::min(d, dmin) */
                dmax = (d < dmax) ? dmax : d;  /* std::max(d, dmax) */
            }
        }
        dmin = dmin * 0.96f - 0.01f;
        dmax = dmax * 1.22f + 0.4f;
        dmin = (0.01f < dmin) ? dmin : 0.01f;     /* std::max(nearZ, dmin) */
        dmax = (dmax < 5000.0f) ? dmax : 5000.0f; /* std::min(farZ, dmax) */
        cell[2 * x + 0] = dmin;
        cell[2 * x + 1] = dmax;
    }
}

static inline uint8_t unorm8(float v)
{
    return (uint8_t)rintf(sat(v) * 255.0f);
}

/* tracescreen.hlsl:50-76 */
void ro_tracescreen(const ro_noise* nz, const ro_frame* fr, const float* cell_distance, float* rgba32f,
                    uint8_t* rgba8, float* primary_steps, ro_stats* st)
{
    ro_tracescreen2(nz, fr, cell_distance, rgba32f, rgba8, primary_steps, NULL, st);
}

void ro_tracescreen2(const ro_noise* nz, const ro_frame* fr, const float* cell_distance, float* rgba32f,
                     uint8_t* rgba8, float* primary_steps, float* secondary_steps, ro_stats* st)
{
    sky_consts k;
    sky_init(&k);
    int W = fr->width, H = fr->height;
    int r0 = fr->row_begin < 0 ? 0 : fr->row_begin;
    int r1 = (fr->row_end <= 0 || fr->row_end > H) ? H : fr->row_end;
    int rs = fr->row_step > 0 ? fr->row_step : 1;
    int nrows = r1 > r0 ? (r1 - r0 + rs - 1) / rs : 0;
    int aa = fr->aa_samples;
    if (aa != 2 && aa != 4 && aa != 8 && aa != 16) aa = 1;
    const float (*offs)[2] = aa_table(aa);
    uint64_t noise = 0, pst = 0, sst = 0, hits = 0, rays = 0, dens = 0, aost = 0, aor = 0;
    int nt = fr->threads > 0 ? fr->threads : 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : noise, pst, sst, hits, rays, dens, aost, aor) num_threads(nt ? nt : omp_get_max_threads())
    for (int ri = 0; ri < nrows; ++ri) {
        int y = r0 + ri * rs;
        ctx c;
        ctx_init(&c, nz, fr);
        for (int x = 0; x < W; ++x) {
#ifdef RO_STUDY
            c.study_pixel = (int64_t)y * W + x;
#endif
            float pxf = (float)x, pyf = (float)y;
            float spx = DIVR(pxf, (float)W), spy = DIVR(pyf, (float)H);
            uint32_t cell = (uint32_t)MAD(floorf(spy * 32.0f), 32.0f, floorf(spx * 32.0f));
            float plane_x = cell_distance[2 * cell], plane_y = 5000.0f;
            float col[3] = {0.0f, 0.0f, 0.0f};
            float steps = 0.0f;
            c.pixel_secondary_steps = 0.0f;
            for (int a = 0; a < aa; ++a) {
                f3 p, dir;
                get_pixel_ray(&c, pxf + offs[a][0] * (1.0f / 16.0f), pyf + offs[a][1] * (1.0f / 16.0f), &p, &dir);
                f3 pdn = norm3(dir);
                float ao;
                f3 s = trace_sample(&c, &k, p, dir, pdn, plane_x, plane_y, &steps, &pst, &hits, &sst, (uint32_t)x,
                                    (uint32_t)y, (uint32_t)a, &ao, &aost, &aor);
                if (fr->ao_samples > 0) {
                    /* AO extension: ao multiplies the saturated sample (1.0 for misses) */
                    col[0] = col[0] + sat(s.x) * ao;
                    col[1] = col[1] + sat(s.y) * ao;
                    col[2] = col[2] + sat(s.z) * ao;
                } else {
                    col[0] = col[0] + sat(s.x);
                    col[1] = col[1] + sat(s.y);
                    col[2] = col[2] + sat(s.z);
                }
                rays += 1;
            }
            col[0] = DIVR(col[0], (float)aa); col[1] = DIVR(col[1], (float)aa); col[2] = DIVR(col[2], (float)aa);
            size_t o = (size_t)y * W + x;
            if (rgba32f) {
                rgba32f[4 * o + 0] = col[0]; rgba32f[4 * o + 1] = col[1];
                rgba32f[4 * o + 2] = col[2]; rgba32f[4 * o + 3] = 1.0f;
            }
            if (rgba8) {
                rgba8[4 * o + 0] = unorm8(col[0]); rgba8[4 * o + 1] = unorm8(col[1]);
                rgba8[4 * o + 2] = unorm8(col[2]); rgba8[4 * o + 3] = 255;
            }
            if (primary_steps) primary_steps[o] = steps;
            if (secondary_steps) secondary_steps[o] = c.pixel_secondary_steps;
        }
        noise += c.noise_calls;
        dens += c.density_calls;
    }
    if (st) {
        st->noise3d_calls += noise;
        st->primary_steps += pst;
        st->shadow_steps += sst;
        st->primary_hits += hits;
        st->primary_rays += rays;
        st->density_calls += dens;
        st->ao_steps += aost;
        st->ao_rays += aor;
    }
}

void ro_render_frame(const ro_noise* nz, const ro_frame* fr, float* camera_results, float* cell_distance,
                     float* rgba32f, uint8_t* rgba8, float* primary_steps, ro_stats* st)
{
    float cr_local[1024 * 4], cd_local[1024 * 2];
    float* cr = camera_results ? camera_results : cr_local;
    float* cd = cell_distance ? cell_distance : cd_local;
    ro_camerarays(nz, fr, cr, st);
    ro_set_target_depths(cr, cd);
    ro_tracescreen(nz, fr, cd, rgba32f, rgba8, primary_steps, st);
}

/* density probe for tests */
float ro_get_density(const ro_noise* nz, const ro_frame* fr, float x, float y, float z)
{
    ctx c;
    ctx_init(&c, nz, fr);
    return get_density(&c, v3(x, y, z));
}
void ro_get_density_batch(const ro_noise* nz, const ro_frame* fr, const float* xyz, float* out, int64_t n)
{
    ctx c;
    ctx_init(&c, nz, fr);
    for (int64_t i = 0; i < n; ++i) out[i] = get_density(&c, v3(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]));
}

/* ---- output path (test infrastructure for k_bgrx / the recorder) ---- */
/* RecorderWinAPI.cpp:244-253 */
void ro_bgrx(const uint8_t* frame, int width, int height, int stride, uint32_t* out)
{
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            uint32_t dwc;
            memcpy(&dwc, frame + (size_t)y * stride + (size_t)x * 4, 4);
            out[(size_t)y * width + x] = (dwc & 0x0000FF00u) | (dwc & 0x000000FFu) << 16 | (dwc & 0x00FF0000u) >> 16;
        }
    }
}

/* RecorderWinAPI.cpp:196-197 (rtStart = 0; rtDuration = 10^7 / frameRate for integer rates)
 * and :264-274 (per-sample duration, rtStart += duration) */
void ro_sample_times(int frame_rate, int fixed_speed, const float* frame_times, int n, uint64_t* sample_time,
                     uint64_t* duration)
{
    const uint64_t rt_duration = 10000000ull / (uint64_t)frame_rate;
    uint64_t rt_start = 0;
    for (int i = 0; i < n; i++) {
        uint64_t d = rt_duration;
        if (!fixed_speed) d = (uint64_t)(10000000.0f * frame_times[i]);
        sample_time[i] = rt_start;
        duration[i] = d;
        rt_start += d;
    }
}
