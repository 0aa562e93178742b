// rt_shader.h -- device implementation of the reference HLSL hot path.
//
// Functions follow Media/common/shaders/{noise,tracing,sky,tracescreen,
// camerarays}.hlsl and Media/<landscape>/shaders/{terrain,color}.hlsl
// (citations per function), evaluated under the numeric rules of rt_math.h so
// results are bit-identical to the CPU oracle.  Layout decisions (tables in
// LDS, packed gradient codes, octave tables in the constant block) are MI355X
// choices and documented in DESIGN.md.
#pragma once

#include "rt_math.h"
#include "rt_types.h"

namespace rts {

using rtm::f3;
using rtm::fma;

// ---------------------------------------------------------------------------
// Noise lattice view (both tables live in LDS for the kernel's lifetime).
//   perm2d: texPerm2D texels (R8G8B8A8_UINT), texel (x,y) at x + y*128 (64 KiB).
//   grad:   CBNoise.permGradients as float4, stored lane-private: entry i for
//           lane slot s (= lane & 15) at grad[i*16 + s] (32 KiB).  A ds_read_b128
//           wave instruction serves 16-lane groups; giving each lane of a group its
//           own 16-byte bank slot makes every gradient fetch conflict-free however
//           random the 8 corner indices are.
struct NoiseView {
    const uint32_t* perm2d;
    const float4* grad;
    uint32_t slot;
    mutable uint32_t calls; // noise3d evaluations (read only by the STATS kernels; dead otherwise)
};

__device__ __forceinline__ float fade(float t)
{
    return ((t * t) * t) * fma(t, fma(t, 6.0f, -15.0f), 10.0f);
}

// gradperm (noise.hlsl:145-150): dot(permGradients[i % 128].xyz, p), HLSL dot (R4).
// The LDS copy stores w = -0.0, and fma(gx, x, -0.0) == gx*x bit for bit (x + -0 == x
// for every non-NaN x, signed zeros included), so consuming w costs nothing and keeps
// the fetch a full ds_read_b128 (4 LDS cycles) instead of the b96 form (8 cycles).
__device__ __forceinline__ float gdot(const float4& g, float x, float y, float z)
{
    return fma(g.z, z, fma(g.y, y, fma(g.x, x, g.w)));
}

// noise.hlsl:153-179 (live `#if 1` block)
__device__ __forceinline__ float noise3d(const NoiseView& nz, float px, float py, float pz)
{
    nz.calls += 1;
    float fx = rtm::floor(px), fy = rtm::floor(py), fz = rtm::floor(pz);
    int32_t Px = (int32_t)fx, Py = (int32_t)fy, Pz = (int32_t)fz;
    float x = px - fx, y = py - fy, z = pz - fz;
    float ux = fade(x), uy = fade(y), uz = fade(z);
    // P & 127 == the HLSL negative-safe modulo (noise.hlsl:159-164)
    uint32_t X = (uint32_t)Px & 127u, Y = (uint32_t)Py & 127u, Z = (uint32_t)Pz & 127u;
    uint32_t t = nz.perm2d[X + (Y << 7)];
    // Pu = texel + Pu.z per channel (bytes <= 127+127+1: no carry), % 128
    uint32_t zz = Z * 0x01010101u;
    uint32_t w0 = (t + zz) & 0x7f7f7f7fu;               // Pu.x, Pu.y, Pu.z, Pu.w
    uint32_t w1 = (t + zz + 0x01010101u) & 0x7f7f7f7fu; // Pu.* + ONE_PIXEL
    const float4* gb = nz.grad + nz.slot;
    const float4 ga0 = gb[(w0 & 0xffu) << 4];
    const float4 ga1 = gb[((w0 >> 8) & 0xffu) << 4];
    const float4 gb0 = gb[((w0 >> 16) & 0xffu) << 4];
    const float4 gb1 = gb[(w0 >> 24) << 4];
    const float4 ha0 = gb[(w1 & 0xffu) << 4];
    const float4 ha1 = gb[((w1 >> 8) & 0xffu) << 4];
    const float4 hb0 = gb[((w1 >> 16) & 0xffu) << 4];
    const float4 hb1 = gb[(w1 >> 24) << 4];
    float x1 = x + -1.0f, y1 = y + -1.0f, z1 = z + -1.0f;
    float g000 = gdot(ga0, x, y, z);
    float g100 = gdot(gb0, x1, y, z);
    float g010 = gdot(ga1, x, y1, z);
    float g110 = gdot(gb1, x1, y1, z);
    float g001 = gdot(ha0, x, y, z1);
    float g101 = gdot(hb0, x1, y, z1);
    float g011 = gdot(ha1, x, y1, z1);
    float g111 = gdot(hb1, x1, y1, z1);
    float l0 = rtm::lerp(rtm::lerp(g000, g100, ux), rtm::lerp(g010, g110, ux), uy);
    float l1 = rtm::lerp(rtm::lerp(g001, g101, ux), rtm::lerp(g011, g111, ux), uy);
    return rtm::lerp(l0, l1, uz);
}

// ---------------------------------------------------------------------------
// Per-frame state visible to device code (cbuffer contents + derived tables).
struct Ctx {
    NoiseView nz;
    const RtConsts* k;
    f3 eye;
    f3 sun;
};

// Media/nomadplains/shaders/terrain.hlsl:8-39
__device__ __forceinline__ float density_nomadplains(const Ctx& c, f3 p)
{
    float dist = rtm::max(rtm::length(rtm::sub(p, c.eye)), 0.01f);
    float d = -p.y;
    f3 p1 = rtm::scale(p, 0.4f);
    float s = 0.0f;
    float detail = rtm::max(18.0f - rtm::pow_nonneg(dist, 0.33f), 2.0f);
    f3 q0 = rtm::scale(p1, 0.006f);
    // N = 1 .. floor(detail); detail <= 17.79 so N <= 17 (RT_NP_OCTAVES)
    #pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES; ++N) {
        if (!((float)N <= detail)) break;
        float S = c.k->np_scale[N];
        float n = noise3d(c.nz, q0.x * S, q0.y * c.k->np_scale_y[N], q0.z * S);
        s = fma(n, c.k->np_rcp[N], s);
    }
    s = rtm::pow_nonneg(rtm::abs(fma(s, 30.0f, 1.0f)) * 35.0f, c.k->np_expo);
    float steep = rtm::sat((noise3d(c.nz, p1.x * 0.007138f, p1.z * 0.007138f, 0.0f) - 0.2f) * 6.0f) * 7.5f;
    float floorsize = steep * 1.8f;
    float t;
    t = rtm::sat((p1.y - 13.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((p1.y - 16.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((p1.y - 19.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((p1.y - 22.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    s = fma(rtm::pow_nonneg(rtm::sat((-p1.y + 10.0f) * 1.6f), 1.5f), 19.0f, s);
    return d + s;
}

// Media/testing/shaders/terrain.hlsl:6-36
__device__ __forceinline__ float density_testing(const Ctx&, f3 p)
{
    float d = -p.y;
    return fma(rtm::sin(p.x * 0.1f) * rtm::cos(p.z * 0.1f), 10.0f, d);
}

// Media/simple/shaders/terrain.hlsl:7-48
__device__ __forceinline__ float density_simple(const Ctx& c, f3 p)
{
    float d = -p.y;
    f3 q = rtm::scale(p, 0.006f);
    float n = noise3d(c.nz, q.x * 1.0f, q.y * 0.0f, q.z * 1.0f) * 150.0f;
    f3 q2 = rtm::scale(p, 0.002f);
    float w2 = rtm::min(rtm::max(fma(-p.y, 1.5f, 50.0f), 0.0f), 36.0f);
    n = fma(-fma(noise3d(c.nz, q2.x, q2.y, q2.z), 0.5f, 0.5f), w2, n);
    f3 q3 = rtm::scale(p, 0.003f);
    float w3 = rtm::min(rtm::max(fma(-p.y, 1.5f, 10.0f), 0.0f), 36.0f);
    n = fma(-fma(noise3d(c.nz, q3.x, q3.y, q3.z), 0.5f, 0.5f), w3, n);
    f3 q4 = rtm::scale(p, 0.06f);
    float S = c.k->np_scale[1];
    n = fma(noise3d(c.nz, q4.x * S, q4.y * c.k->np_scale_y[1], q4.z * S), c.k->np_rcp[1], n);
    return d + n;
}

// Media/greenrocks/shaders/terrain.hlsl:4-32
__device__ __forceinline__ float density_greenrocks(const Ctx& c, f3 p)
{
    p.y = p.y - 170.0f;
    float d = 0.0f;
    d = d + -p.y;
    f3 pg = rtm::scale(p, 0.01f);
    float g = noise3d(c.nz, pg.x, pg.y, pg.z);
    float nohy = fma(rtm::abs(g), 1.4f, 0.1f);
    f3 pc = rtm::mk(p.x * 0.011f, p.y * 0.0013f, p.z * 0.011f);
    float g32 = g * 0.32f;
#pragma unroll
    for (int N = 1; N <= 7; ++N) {
        float S = (float)(1 << N); // pow(2, N) is exact under R5
        float n = noise3d(c.nz, fma(pc.x, S, g32), fma(pc.y, S, g32), fma(pc.z, S, g32));
        d = fma((rtm::abs(n) * 210.0f) * g, rtm::rcp(S), d);
    }
    d = d - 50.0f;
    f3 p2 = rtm::scale(p, 0.002f);
    f3 p2n = rtm::mk(p2.x * 1.0f, p2.y * nohy, p2.z * 1.0f);
#pragma unroll
    for (int N = 1; N <= 5; ++N) {
        float S = (float)(1 << N);
        float n = noise3d(c.nz, p2n.x * S, p2n.y * S, p2n.z * S);
        float inner = fma(n + 0.1f, 0.5f, 0.5f);
        d = fma(-inner, 220.0f * rtm::rcp(S), d);
    }
    return d;
}

template <int L>
__device__ __forceinline__ float get_density(const Ctx& c, f3 p)
{
    if constexpr (L == RT_TESTING) return density_testing(c, p);
    else if constexpr (L == RT_SIMPLE) return density_simple(c, p);
    else if constexpr (L == RT_GREENROCKS) return density_greenrocks(c, p);
    else return density_nomadplains(c, p);
}

template <int L>
struct FogLive {
    static constexpr bool value = (L == RT_GREENROCKS);
};

struct f4 {
    float x, y, z, w;
};

// Media/greenrocks/shaders/terrain.hlsl:34-54 (other landscapes return 0)
template <int L>
__device__ __forceinline__ f4 get_fog(const Ctx& c, f3 p, float dist)
{
    f4 r = {0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (!FogLive<L>::value) {
        return r;
    } else {
        float fogd = 0.0f;
        float d = 0.0f;
        dist = rtm::sat(fma(-dist, 0.0012f, 1.0f));
        float falloff = rtm::sat(fma(-(dist * dist), 0.1f, 1.0f));
        if (falloff > 0.0f) {
            d = d + rtm::sat((-p.y - 2.0f) * 0.0003f);
            f3 q = rtm::scale(p, 0.1261f);
            fogd = fma(rtm::abs(noise3d(c.nz, q.x, q.y, q.z)), 0.2f, 0.8f);
        }
        float fc = 0.9f * fogd;
        float v = (fc * d) * dist;
        r.x = v;
        r.y = v;
        r.z = v;
        r.w = d * dist;
        return r;
    }
}

struct RayResult {
    f4 pd;
    f4 fc;
    float density;
    float steps;
};

// Media/common/shaders/tracing.hlsl:47-105 (+ build extension max_steps)
template <int L, bool CALCFOG, bool SKIPREFINE>
__device__ __forceinline__ RayResult trace_ray(const Ctx& c, f3 p, float dist, float enddist, float stepmod, f3 dir,
                                               int max_steps)
{
    constexpr bool FOG = CALCFOG && FogLive<L>::value;
    const RtConsts* k = c.k;
    RayResult rr;
    f4 f = {0.0f, 0.0f, 0.0f, 0.0f};
    float d = 0.0f;
    float total = 0.0f;
    float dirLength = rtm::length(dir);
    float step = fma(-dist, k->one_minus_step_factor, (0.03f * stepmod) * dirLength);
    float lastStep = step;
    float il = rtm::rcp(dirLength);
    dir = rtm::scale(dir, il);
    if constexpr (FOG) {
        float hd = dist * 0.5f;
        f3 mp = rtm::mk(fma(dir.x * dist, 0.5f, p.x), fma(dir.y * dist, 0.5f, p.y), fma(dir.z * dist, 0.5f, p.z));
        f4 mf = get_fog<L>(c, mp, hd);
        f.x = fma(mf.x, dist, f.x);
        f.y = fma(mf.y, dist, f.y);
        f.z = fma(mf.z, dist, f.z);
        f.w = fma(mf.w, dist, f.w);
    }
    f3 rayp = rtm::mk(0.0f, 0.0f, 0.0f);
    int iters = 0;
    const float minl = k->min_limit;
    const float sf = k->step_factor;
    const float df = k->density_factor;
    while (dist < enddist && step > minl) {
        if (max_steps > 0 && iters >= max_steps) break;
        ++iters;
        total = total + 1.0f;
        rayp = rtm::mk(fma(dir.x, dist, p.x), fma(dir.y, dist, p.y), fma(dir.z, dist, p.z));
        d = get_density<L>(c, rayp);
        f4 fs = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (FOG) {
            f4 g = get_fog<L>(c, rayp, dist);
            fs.x = g.x * step;
            fs.y = g.y * step;
            fs.z = g.z * step;
            fs.w = g.w * step;
        }
        if (d > 0.0f) {
            if constexpr (SKIPREFINE) break;
            dist = dist - lastStep;
            step = step * 0.3f;
            f.x = f.x - fs.x;
            f.y = f.y - fs.y;
            f.z = f.z - fs.z;
            f.w = f.w - fs.w;
        } else {
            float stepmult = 1.0f + rtm::pow_nonneg(rtm::abs(rtm::min(d + 5.0f, 0.0f)), df);
            step = step * sf;
            lastStep = step * stepmult;
            dist = dist + lastStep;
            f.x = f.x + fs.x;
            f.y = f.y + fs.y;
            f.z = f.z + fs.z;
            f.w = f.w + fs.w;
        }
    }
    rr.pd.x = rayp.x;
    rr.pd.y = rayp.y;
    rr.pd.z = rayp.z;
    rr.pd.w = dist;
    rr.fc = f;
    rr.density = d;
    rr.steps = total;
    return rr;
}

// tracing.hlsl:107-116
template <int L>
__device__ __forceinline__ f3 get_normal(const Ctx& c, f4 pd)
{
    f3 p = rtm::mk(pd.x, pd.y, pd.z);
    float dist = rtm::length(rtm::sub(p, c.eye));
    float nd = dist * 0.005f;
    float dx = get_density<L>(c, rtm::mk(p.x - nd, p.y - 0.0f, p.z - 0.0f)) - pd.w;
    // serialise the three independent density evaluations (register pressure)
    asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z), "+v"(nd) : "v"(dx));
    float dy = get_density<L>(c, rtm::mk(p.x - 0.0f, p.y - nd, p.z - 0.0f)) - pd.w;
    asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z), "+v"(nd) : "v"(dy));
    float dz = get_density<L>(c, rtm::mk(p.x - 0.0f, p.y - 0.0f, p.z - nd)) - pd.w;
    return rtm::normalize(rtm::mk(dx, dy, dz));
}

// tracing.hlsl:124-134 (x scaled by Projection._22, y by _11, as written)
__device__ __forceinline__ void get_pixel_ray(const Ctx& c, float px, float py, f3* outp, f3* outdir)
{
    const RtConsts* k = c.k;
    float sx = fma(px + 0.5f, k->rcp_w, -0.5f) * 2.0f;
    float sy = fma(py + 0.5f, k->rcp_h, -0.5f) * 2.0f;
    sx = sx * k->proj22;
    sy = sy * k->proj11;
    const float* m = k->view_inverse;
    float r0 = fma(1.0f, m[12], fma(1.0f, m[8], fma(sy, m[4], sx * m[0])));
    float r1 = fma(1.0f, m[13], fma(1.0f, m[9], fma(sy, m[5], sx * m[1])));
    float r2 = fma(1.0f, m[14], fma(1.0f, m[10], fma(sy, m[6], sx * m[2])));
    *outp = rtm::mk(r0, r1, r2);
    *outdir = rtm::sub(*outp, c.eye);
}

// ---------------------------------------------------------------------------
// Media/common/shaders/sky.hlsl
__device__ __forceinline__ f3 mod_ray_dir(f3 d) { return rtm::normalize(rtm::mk(d.x, rtm::sat(d.y), d.z)); }

// sky.hlsl:26-36
__device__ __forceinline__ float get_space_color(const Ctx& c, f3 dir)
{
    dir = mod_ray_dir(dir);
    if (dir.y <= 0.0f) return 0.0f;
    float space = noise3d(c.nz, dir.x * 500.0f, dir.y * 500.0f, dir.z * 500.0f);
    // serialise the three independent lattice evaluations (register pressure)
    asm volatile("" : "+v"(dir.x), "+v"(dir.y), "+v"(dir.z) : "v"(space));
    space = space - fma(noise3d(c.nz, dir.x * 150.2f, dir.y * 150.2f, dir.z * 150.2f), 0.5f, 0.13f);
    asm volatile("" : "+v"(dir.x), "+v"(dir.y), "+v"(dir.z) : "v"(space));
    space = space - fma(noise3d(c.nz, dir.x * 200.2f, dir.y * 200.2f, dir.z * 200.2f), 0.5f, 0.5f);
    return (space * 1.0f) * rtm::sat(fma(-c.sun.y, 2.7f, -0.5f));
}

// sky.hlsl:39-43
__device__ __forceinline__ float sky_scale(float fCos)
{
    float x = 1.0f - fCos;
    float t = fma(x, 5.25f, -6.80f);
    t = fma(x, t, 3.83f);
    t = fma(x, t, 0.459f);
    t = fma(x, t, -0.00287f);
    return 0.19f * rtm::exp(t);
}

struct SkyColor {
    f3 mie, rayleigh;
};

// sky.hlsl:83-137 (applyPhase :64-72 with the swapped mie/rayleigh arguments of :131)
__device__ __forceinline__ SkyColor get_rayleigh_mie(const Ctx& c, f3 org)
{
    const RtConsts* k = c.k;
    f3 rd = mod_ray_dir(org);
    float far = fma((1.0f - rd.y) * k->sky_dist_to_top, 2.0f, k->sky_dist_to_top);
    f3 start = rtm::mk(k->sky_start[0], k->sky_start[1], k->sky_start[2]);
    float fStartAngle = rtm::dot(rd, rtm::mk(k->sky_start_n[0], k->sky_start_n[1], k->sky_start_n[2]));
    float fStartOffset = k->sky_depth0 * sky_scale(fStartAngle);
    float sampleLength = far * k->sky_rcp_samples;
    float scaledLength = sampleLength * k->sky_fscale;
    f3 sampleRay = rtm::scale(rd, sampleLength);
    f3 sp = rtm::mk(fma(sampleRay.x, 0.5f, start.x), fma(sampleRay.y, 0.5f, start.y), fma(sampleRay.z, 0.5f, start.z));
    float fr0 = 0.0f, fr1 = 0.0f, fr2 = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float height = rtm::length(sp);
        float dep = rtm::exp(k->sky_sos * (200.0f - height));
        float ih = rtm::rcp(height);
        float fLight = rtm::dot(c.sun, sp) * ih;
        float fCam = rtm::dot(rd, sp) * ih;
        float fScatter = fma(dep, sky_scale(fLight) - sky_scale(fCam), fStartOffset);
        float ds = dep * scaledLength;
        fr0 = fma(rtm::exp(-fScatter * k->sky_att[0]), ds, fr0);
        fr1 = fma(rtm::exp(-fScatter * k->sky_att[1]), ds, fr1);
        fr2 = fma(rtm::exp(-fScatter * k->sky_att[2]), ds, fr2);
        sp = rtm::mk(sp.x + sampleRay.x, sp.y + sampleRay.y, sp.z + sampleRay.z);
    }
    f3 mie = rtm::mk(fr0 * k->sky_mie_k[0], fr1 * k->sky_mie_k[1], fr2 * k->sky_mie_k[2]);
    f3 ray = rtm::mk(fr0 * k->sky_km_esun, fr1 * k->sky_km_esun, fr2 * k->sky_km_esun);
    f3 t = rtm::mk(-rd.x * far, -rd.y * far, -rd.z * far);
    float fCos = rtm::dot(c.sun, t) * rtm::rcp(rtm::length(t));
    float fCos2 = fCos * fCos;
    float mphase = (k->sky_mie_a * (1.0f + fCos2)) *
                   rtm::rcp(rtm::pow_nonneg(rtm::abs(fma(-k->sky_two_g, fCos, k->sky_one_plus_g2)), 1.5f));
    float rphase = fma(0.75f, fCos2, 0.75f);
    SkyColor sc;
    sc.mie = rtm::scale(ray, mphase);
    sc.rayleigh = rtm::scale(mie, rphase);
    float m = rtm::sat(fma(org.y, 0.5f, 0.5f) * 4.0f);
    sc.rayleigh = rtm::scale(sc.rayleigh, m);
    float sy = rtm::sat(c.sun.y);
    sc.rayleigh.z = fma(0.6f, sy, sc.rayleigh.z);
    sc.rayleigh.y = fma(0.4f, sy, sc.rayleigh.y);
    sc.rayleigh.x = fma(0.3f, sy, sc.rayleigh.x);
    return sc;
}

// ---------------------------------------------------------------------------
// getColor up to (not including) the shadow march: albedo, brightness and the
// shadow-ray step modifier.  Media/nomadplains/shaders/color.hlsl:8-50,
// testing/color.hlsl:12-22, simple/color.hlsl:8-52, greenrocks/color.hlsl:12-22.
struct ShadePre {
    float col[3];   // albedo rgb (color.a handled via spec_k)
    float spec_k;   // color.a
    float spec_dot; // fresnel argument
    float brightness;
    float precision;
};

template <int L>
__device__ __forceinline__ ShadePre shade_pre(const Ctx& c, f3 p, f3 n, f3 d, float dist)
{
    ShadePre r;
    if constexpr (L == RT_NOMADPLAINS || L == RT_SIMPLE) {
        float c0 = c.k->albedo[0], c1 = c.k->albedo[1], c2 = c.k->albedo[2];
        float s = 0.0f;
        if constexpr (L == RT_NOMADPLAINS) {
            f3 q = rtm::mk(p.y * 0.5f, p.x * 0.01f, p.z * 0.01f);
            #pragma unroll 1
            for (int N = 1; N <= 20; ++N) {
                float S = c.k->col_scale[N];
                s = fma(rtm::abs(noise3d(c.nz, q.x * S, q.y * S, q.z * S)), c.k->col_rcp[N], s);
            }
            c0 = fma(-s, 0.5f, c0);
            c1 = fma(-s, 0.5f, c1);
            c2 = fma(-s, 0.5f, c2);
        } else {
            float detail = rtm::max(16.0f - rtm::pow_nonneg(dist, 0.33f), 2.0f);
            f3 q = rtm::mk(p.y * 0.5f, p.x * 0.01f, p.z * 0.1f);
            for (int N = 1; N <= RT_COL_OCTAVES; ++N) {
                if (!((float)N <= detail)) break;
                float S = c.k->col_scale[N];
                s = fma(rtm::abs(noise3d(c.nz, q.x * S, q.y * S, q.z * S)), c.k->col_rcp[N], s);
            }
            float w = rtm::max((200.0f - dist) * c.k->rcp200, 0.0f);
            c0 = fma(-s, w, c0);
            c1 = fma(-s, w, c1);
            c2 = fma(-s, w, c2);
        }
        r.col[0] = c0;
        r.col[1] = c1;
        r.col[2] = c2;
        r.spec_k = 0.2f;
        f3 md = rtm::mk(-d.x, -d.y, -d.z);
        float t2 = rtm::dot(n, md);
        t2 = t2 + t2;
        f3 rf = rtm::mk(fma(-t2, md.x, n.x), fma(-t2, md.y, n.y), fma(-t2, md.z, n.z));
        r.spec_dot = rtm::dot(c.sun, rf);
    } else {
        r.col[0] = c.k->albedo[0];
        r.col[1] = c.k->albedo[1];
        r.col[2] = c.k->albedo[2];
        r.spec_k = c.k->albedo[3];
        r.spec_dot = rtm::dot(rtm::mk(-d.x, -d.y, -d.z), n);
    }
    r.brightness = rtm::dot(n, c.sun);
    float mipf = rtm::max(0.5f * rtm::log2_nonneg(dist), 0.0f);
    r.precision = rtm::max((mipf - 3.2f) * 3.0f, 1.0f) * 8.0f;
    return r;
}

// getColor after the shadow march (color.hlsl:53-71)
__device__ __forceinline__ f3 shade_post(const Ctx& c, const ShadePre& s, float shadow_density, float shadow_fog_w)
{
    float b = s.brightness;
    if (shadow_density > 0.0f) b = b * 0.1f;
    else b = rtm::sat(b - shadow_fog_w);
    float specular = rtm::sat(rtm::pow_nonneg(rtm::max(s.spec_dot, 0.0f), 40.0f)) * s.spec_k;
    float c0 = s.col[0] + specular, c1 = s.col[1] + specular, c2 = s.col[2] + specular;
    const RtConsts* k = c.k;
    return rtm::mk(c0 * fma(b, k->one_minus_shadow[0], k->shadow_color[0]),
                   c1 * fma(b, k->one_minus_shadow[1], k->shadow_color[1]),
                   c2 * fma(b, k->one_minus_shadow[2], k->shadow_color[2]));
}

__device__ __forceinline__ uint32_t unorm8(float v) { return (uint32_t)rtm::rint(rtm::sat(v) * 255.0f); }

} // namespace rts
