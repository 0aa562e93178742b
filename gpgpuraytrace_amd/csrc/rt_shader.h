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
#include "rt_variants.h"

namespace rts {

using rtm::f3;
using rtm::fma;

// ---------------------------------------------------------------------------
// Noise lattice view: one LDS image for the kernel's lifetime (rt_kernels.hip load_noise_lds):
//   byte 0      perm2D texels (R8G8B8A8_UINT), texel (x,y) at (x + y*128) * 4 (64 KiB).  At image
//               offset 0 the texel address is the masked lattice offset itself (no base add).
//   kLdsGxy     gxy: CBNoise.permGradients re-laid as PAIRS.  The z+1 corners of noise3d
//               (noise.hlsl:166-168, Pu + ONE_PIXEL) index gradient (i+1)&127 where the z corners
//               index i, so entry i holds gradients i and i+1 side by side:
//                 gxy[i] = (g[i].x, g[i+1].x, g[i].y, g[i+1].y)   16 B
//                 gz[i]  = (g[i].z, g[i+1].z)                      8 B (of a 16-B slot)
//               One pair of loads yields both z-layers of a lattice column in register pairs that
//               v_pk_fma_f32 consumes as they land (no shuffles), and only the four z-layer
//               indices need extracting.  Entries are lane-private: entry i for lane slot s at
//               kLdsGxy + i*256 + (s&15)*16, so one v_perm_b32 builds the whole address
//               (base byte from so16, index byte from the texel, slot byte from so16); the b128
//               loads are conflict-free however random the indices, the b64 loads 2-way.
//   kLdsGz      gz at the same slot layout (ds_read_b64 ... offset:32768 from the gxy address).
//   then        the nomadplains FBM octave table (oct).
constexpr uint32_t kLdsGxy = 0x10000u, kLdsGz = 0x18000u;
typedef float v2f __attribute__((ext_vector_type(2)));

struct NoiseView {
    const char* img;    // the LDS image (perm2D texels at its offset 0)
    const float4* oct;  // nomadplains FBM octave N: (S, 0.35 S, 1/S, 0), N = 0 .. RT_NP_OCTAVES + 2
    uint32_t so16;  // kLdsGxy | (lane & 15) * 16: byte 2 = the gxy plane's base >> 16, byte 0 = the lane's slot
    // noise3d evaluations, read only by the STATS kernels (dead otherwise): low word = this lane's
    // calls, high word = wave iterations (the wave's first active lane adds 1 << 32 per call), so
    // calls / (64 * iterations) is the SIMD lane utilisation of the noise work
    mutable uint64_t calls;
    // k_trace's STATS kernels count in LDS instead ({lane calls, wave iterations}, added by the
    // wave's first active lane per call): no per-lane 64-bit counter held across its loops.
    // nullptr elsewhere (then `calls` counts).
    __attribute__((address_space(3))) unsigned long long* lds_calls;
    // k_trace work kind of the caller (RT_PHASE_*): a diagnostic build (-DRT_COUNT_PHASE=k, scripts/
    // phase_util.sh) counts only that kind's noise, to split the lane utilisation by phase
    uint32_t phase;
};
enum { RT_PHASE_OTHER = 0, RT_PHASE_PRIMARY = 1, RT_PHASE_LONG = 2, RT_PHASE_SHADE = 3 };

__device__ __forceinline__ void count_noise(const NoiseView& nz)
{
#ifdef RT_COUNT_PHASE
    if (nz.phase != RT_COUNT_PHASE) return;
#endif
    // the active lanes as a ballot (convergent: evaluated where the call is; a plain read of EXEC
    // can be hoisted out of the FBM loop, crediting later octaves' wave iterations to a lane that
    // already left it, which undercounted iterations before ABI 4)
    const uint64_t ex = __ballot(1);
    if (nz.lds_calls) {
        if (__lane_id() == (uint32_t)__builtin_ctzll(ex)) {
            __atomic_fetch_add(&nz.lds_calls[0], (unsigned long long)__popcll(ex), __ATOMIC_RELAXED);
            __atomic_fetch_add(&nz.lds_calls[1], 1ull, __ATOMIC_RELAXED);
        }
        return;
    }
    nz.calls += 1ull + ((uint64_t)(__lane_id() == (uint32_t)__builtin_ctzll(ex)) << 32);
}

__device__ __forceinline__ v2f v2(float a, float b)
{
    v2f r = {a, b};
    return r;
}
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

// fade (noise.hlsl:133-136): t*t*t*(t*(t*6-15)+10)
__device__ __forceinline__ float fade(float t)
{
    return ((t * t) * t) * fma(t, fma(t, 6.0f, -15.0f), 10.0f);
}
__device__ __forceinline__ v2f fade2(v2f t)
{
    return ((t * t) * t) * vfma(t, vfma(t, v2(6.0f, 6.0f), v2(-15.0f, -15.0f)), v2(10.0f, 10.0f));
}

// gradperm (noise.hlsl:145-150) for the z and z+1 corners of one lattice column:
// dot(permGradients[i % 128].xyz, p) as the HLSL dot of rule R4,
// fma(g.z, p.z, fma(g.y, p.y, g.x * p.x)), evaluated element-wise on the pair.
__device__ __forceinline__ v2f gdot2(const float4& gxy, const float2& gz, float x, float y, v2f zz)
{
    v2f r = v2(gxy.x, gxy.y) * v2(x, x);
    r = vfma(v2(gxy.z, gxy.w), v2(y, y), r);
    return vfma(v2(gz.x, gz.y), zz, r);
}

// The lattice part of noise3d once the cell is known: the perm2D texel t of (Px, Py), Z = Pz & 127,
// the fractions (x, y, z), x - 1, y - 1 and the fades (ux, uy, uz): the eight gradient dots and
// the trilinear lerp.
__device__ __forceinline__ float noise3d_lattice(const NoiseView& nz, uint32_t t, uint32_t Z, float x, float y,
                                                 float x1, float y1, float z, float ux_, float uy_, float uz)
{
    // Pu = texel + Pu.z per channel (bytes <= 127+127: no carry), % 128
#if RT_Z_MAD24
    // (A/B) the replication as one v_mad_u32_u24 (4.2 issue cycles) instead of the v_mad_u64_u32 (4.9) LLVM picks
    uint32_t w;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(w) : "v"(Z), "s"(0x01010101u), "v"(t));
    w &= 0x7f7f7f7fu;
#else
    uint32_t w = (t + Z * 0x01010101u) & 0x7f7f7f7fu; // AA, AB, BA, BB column indices at z
#endif
    // entry i of either plane starts at byte i*256: one v_perm_b32 per corner builds
    // base | (index byte << 8) | lane slot ({w, so16} byte pick: 4+k = byte k of w, 0 / 2 = bytes
    // 0 / 2 of so16, 12 = 0); gz is the same address + 32768 (the load's offset field)
    auto gxy_at = [&](uint32_t sel) {
        return *reinterpret_cast<const float4*>(nz.img + __builtin_amdgcn_perm(w, nz.so16, sel));
    };
    auto gz_at = [&](uint32_t sel) {
        return *reinterpret_cast<const float2*>(nz.img + (kLdsGz - kLdsGxy) + __builtin_amdgcn_perm(w, nz.so16, sel));
    };
    const float4 a0 = gxy_at(0x0c020400u), a1 = gxy_at(0x0c020500u), b0 = gxy_at(0x0c020600u), b1 = gxy_at(0x0c020700u);
    const float2 za0 = gz_at(0x0c020400u), za1 = gz_at(0x0c020500u), zb0 = gz_at(0x0c020600u), zb1 = gz_at(0x0c020700u);
    const v2f zz = v2(z, z + -1.0f);
    v2f g00 = gdot2(a0, za0, x, y, zz);   // (g000, g001)
    v2f g10 = gdot2(b0, zb0, x1, y, zz);  // (g100, g101)
    v2f g01 = gdot2(a1, za1, x, y1, zz);  // (g010, g011)
    v2f g11 = gdot2(b1, zb1, x1, y1, zz); // (g110, g111)
    // lerp(a, b, t) = fma(t, b - a, a) element-wise: x, then y, then z
    v2f ux = v2(ux_, ux_), uy = v2(uy_, uy_);
    v2f lx0 = vfma(ux, g10 - g00, g00);
    v2f lx1 = vfma(ux, g11 - g01, g01);
    v2f l = vfma(uy, lx1 - lx0, lx0); // (l0, l1)
    return fma(uz, l.y - l.x, l.x);
}

// The first half of noise3d (noise.hlsl:153-164): the cell of p and its perm2D texel.  Split from
// the lattice half so an FBM loop can fetch octave N+1's texel while octave N's gradient loads
// are in flight (noise_fbm below).
struct NoiseCell {
    v2f xy;     // fractions x, y
    float z;    // fraction z
    uint32_t Z; // Pz & 127
    uint32_t t; // perm2D texel of (Px & 127, Py & 127)
};

// FAST: the integer half without v_cvt_i32_f32 or shifts.  gfx950 issues v_cvt_*, v_floor,
// shifts, v_perm and the 3-operand integer ops at half the rate of FP32 add / mul / fma and
// v_and / v_add_u32 (profiles/r02/ubench_cost_model.md), so the lattice integers come from the
// float floor values by the magic-number add: for an integer f with |f| < 2^22, the bits of
// f + 1.5 * 2^23 hold (2^22 + f) in their low 23 bits, so bits & 127 == f & 127; those of
// fma(f, 4, 1.5 * 2^23) hold ((f & 127) << 2) under the mask 0x1fc when |4 f| < 2^22, and those of
// fma(f, 512, 1.5 * 2^23) hold ((f & 127) << 9) under the mask 0xfe00 when |512 f| < 2^22.  The
// caller guarantees |coordinate| < kFastCellRange = 2^13 (floor keeps it).  Same bits as the
// general path.
constexpr float kFastCellRange = 8192.0f;
constexpr float kMagic = 12582912.0f; // 1.5 * 2^23

// Byte offset of perm2D texel (floor x & 127, floor y & 127) in the LDS image (see FAST below).
template <bool FAST>
__device__ __forceinline__ uint32_t texel_offset(float fx, float fy)
{
    if constexpr (FAST) {
        // (y << 9) & 0xfe00 | (x << 2) & 0x1fc: two full-rate fma + one v_and + one v_and_or
        const uint32_t mx4 = rtm::bits(fma(fx, 4.0f, kMagic)), my9 = rtm::bits(fma(fy, 512.0f, kMagic));
        return (my9 & 0xfe00u) | (mx4 & 0x1fcu);
    } else {
        // texel (Px & 127, Py & 127) at byte ((Py & 127) << 9) | ((Px & 127) << 2): the low
        // term stays below 512, so add-then-mask needs no separate Py mask
        const uint32_t Px = (uint32_t)(int32_t)fx, Py = (uint32_t)(int32_t)fy;
        return ((Py << 9) + ((Px << 2) & 0x1fcu)) & 0xfffcu;
    }
}

// Pz & 127 (the z-layer index)
template <bool FAST>
__device__ __forceinline__ uint32_t layer_index(float fz)
{
    if constexpr (FAST) return rtm::bits(fz + kMagic) & 127u;
    else return (uint32_t)(int32_t)fz & 127u;
}

template <bool FAST = false>
__device__ __forceinline__ NoiseCell noise3d_cell(const NoiseView& nz, float px, float py, float pz)
{
    NoiseCell c;
    const float fx = rtm::floor(px), fy = rtm::floor(py), fz = rtm::floor(pz);
    c.xy = v2(px, py) - v2(fx, fy);
    c.z = pz - fz;
    // P & 127 == the HLSL negative-safe modulo (noise.hlsl:159-164)
    c.Z = layer_index<FAST>(fz);
    c.t = *reinterpret_cast<const uint32_t*>(nz.img + texel_offset<FAST>(fx, fy));
    return c;
}

__device__ __forceinline__ float noise3d_finish(const NoiseView& nz, const NoiseCell& c)
{
    const v2f uxy = fade2(c.xy);
    const v2f xy1 = c.xy + v2(-1.0f, -1.0f);
    return noise3d_lattice(nz, c.t, c.Z, c.xy.x, c.xy.y, xy1.x, xy1.y, c.z, uxy.x, uxy.y, fade(c.z));
}

// noise.hlsl:153-179 (live `#if 1` block); noise3d_raw does not count the call
__device__ __forceinline__ float noise3d_raw(const NoiseView& nz, float px, float py, float pz)
{
    return noise3d_finish(nz, noise3d_cell(nz, px, py, pz));
}

// noise3d(px, py, 0) (nomadplains' steep noise, terrain.hlsl:26).  z = 0 makes Pz = 0 and
// fade(z) = 0, so noise3d is the z-layer's bilinear lerp l0 (fma(+0, l1 - l0, l0) == l0), and
// each z-layer gradient dot loses its z term (fma(g.z, +0, r) == r).  Both identities hold up
// to the sign of a zero, and add/mul/fma inputs that differ only in zero signs give results
// that differ only in zero signs: every nonzero value, the result included, is bit-identical to
// noise3d_raw's.  The caller only forms sat((n - 0.2) * 6), where a zero's sign cannot show.
template <bool FAST = false>
__device__ __forceinline__ float noise3d_z0(const NoiseView& nz, float px, float py)
{
    const float fx = rtm::floor(px), fy = rtm::floor(py);
    const v2f xy = v2(px, py) - v2(fx, fy);
    const v2f uxy = fade2(xy);
    const v2f xy1 = xy + v2(-1.0f, -1.0f);
    const uint32_t w = *reinterpret_cast<const uint32_t*>(nz.img + texel_offset<FAST>(fx, fy)) & 0x7f7f7f7fu;
    auto g_at = [&](uint32_t sel) {
        return *reinterpret_cast<const float4*>(nz.img + __builtin_amdgcn_perm(w, nz.so16, sel));
    };
    const float4 a0 = g_at(0x0c020400u), a1 = g_at(0x0c020500u), b0 = g_at(0x0c020600u), b1 = g_at(0x0c020700u);
    const float x = xy.x, y = xy.y, x1 = xy1.x, y1 = xy1.y;
    const float g00 = fma(a0.z, y, a0.x * x), g10 = fma(b0.z, y, b0.x * x1);
    const float g01 = fma(a1.z, y1, a1.x * x), g11 = fma(b1.z, y1, b1.x * x1);
    const float lx0 = fma(uxy.x, g10 - g00, g00), lx1 = fma(uxy.x, g11 - g01, g01);
    return fma(uxy.y, lx1 - lx0, lx0);
}

__device__ __forceinline__ float noise3d(const NoiseView& nz, float px, float py, float pz)
{
    count_noise(nz);
    return noise3d_raw(nz, px, py, pz);
}

// ---------------------------------------------------------------------------
// Per-frame state visible to device code (cbuffer contents + derived tables).
// k: the launch's constant block (a kernel argument, so its loads are scalar); kf: the
// block of the frame being traced, for the fields that change per frame (ViewInverse, the
// eye-dependent sky terms; Eye and SunDirection are copied into eye / sun).  kf == k except
// in frame batches.
// A frame's constant block as the kernels read it: in the constant address space, so that its
// uniform loads are scalar (the pointer comes from a FrameTable in memory, where a plain pointer
// would be generic and every read a flat load waiting on both memory counters).
typedef const __attribute__((address_space(4))) RtConsts* KPtr;

struct Ctx {
    NoiseView nz;
    const RtConsts* k;
    KPtr kf;
    f3 eye;
    f3 sun;
};

// The FBM's octave count (Media/nomadplains/shaders/terrain.hlsl:16-22): N runs 1 ..
// floor(detail), detail = max(18 - pow(dist, 0.33), 2), dist = max(length(p - Eye), 0.01).
// detail in [2, 17.79] so N <= 17 (RT_NP_OCTAVES), and (float)N <= detail <=> N <= (int)detail.
// Only this integer leaves the expression.  np_octaves_exact is the rule-R5 evaluation (the
// oracle's); np_octaves_estimate gets t ~ 18 - dist^0.33 from the hardware v_log_f32/v_exp_f32
// of d2 = dot(p - Eye, p - Eye) (no sqrt, no polynomial pow) and flags lanes whose t lies within
// kOctEps of an integer, where the estimate and the exact value could floor differently.  Away
// from integers the two agree: tests/test_gpu_parity.py sweeps every finite d2 >= 0 and checks
// (rt_debug_math op 12) that each unflagged estimate equals np_octaves_exact.
constexpr float kOctEps = 1.0f / 2048.0f;

__device__ __forceinline__ int np_octaves_exact(float d2)
{
    const float dist = rtm::max(rtm::sqrt(d2), 0.01f);
    return (int)rtm::max(18.0f - rtm::pow_nonneg(dist, 0.33f), 2.0f);
}

__device__ __forceinline__ int np_octaves_estimate(float d2, bool* near)
{
    // dist^0.33 = 2^(0.165 * log2(d2))
    const float t = 18.0f - __builtin_amdgcn_exp2f(0.165f * __builtin_amdgcn_logf(d2));
    const float ft = rtm::floor(t);
    *near = rtm::abs((t - ft) - 0.5f) > 0.5f - kOctEps;
    const int n = (int)ft;
    return n < 2 ? 2 : (n > RT_NP_OCTAVES ? RT_NP_OCTAVES : n);
}

__device__ __forceinline__ int np_octaves(const Ctx& c, f3 p)
{
    const f3 v = rtm::sub(p, c.eye);
    const float d2 = rtm::dot(v, v);
    bool near;
    int n = np_octaves_estimate(d2, &near);
    if (near) n = np_octaves_exact(d2); // skipped (execz) unless some lane sits near an integer
    return n;
}

// The four terrace subtractions of nomadplains/terrain.hlsl:30-37.  t = saturate((y - h) *
// steep) is +0 wherever (y - 13) * steep <= 0 (steep == 0, or y <= 13 <= h), and then
// fma(-(t*t), floorsize, s) == s bit for bit (s + -0 == s, also for s == +-0): a wave none of
// whose samples has (y - 13) * steep > 0 skips all four.
__device__ __forceinline__ float terraces(float s, float y, float steep)
{
    if (!__ballot((y - 13.0f) * steep > 0.0f)) return s;
    const float floorsize = steep * 1.8f;
    float t;
    t = rtm::sat((y - 13.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((y - 16.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((y - 19.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    t = rtm::sat((y - 22.0f) * steep);
    s = fma(-(t * t), floorsize, s);
    return s;
}

// nomadplains' FBM (terrain.hlsl:16-24): sum over N = 1 .. n_oct of noise3d(q0 * (S, 0.35 S, S)) / S,
// in octave order (the octave constants come from the LDS image: no scalar loads in the loop).
template <bool FAST>
__device__ __forceinline__ float np_fbm(const Ctx& c, f3 q0, int n_oct)
{
    float s = 0.0f;
#if RT_OCT_SMEM && !defined(RT_EXTRA_OCTAVE)
    // The octave constants by scalar loads from the launch's constant block: every lane inside the loop
    // is at the same octave N, so N is uniform (an SGPR), and the loop reads no LDS for them (4 LDS-array
    // cycles of ~40 per octave; rt_variants.h RT_OCT_SMEM)
    const KPtr kc = (KPtr)c.k;
    int N = 1;
#if RT_OCT_SCALAR_EXIT
    int Ne;
#endif
    #pragma unroll 1
    do {
        count_noise(c.nz);
        const float sx = kc->np_scale[N], sy = kc->np_scale_y[N], w = kc->np_rcp[N];
        s = fma(noise3d_finish(c.nz, noise3d_cell<FAST>(c.nz, q0.x * sx, q0.y * sy, q0.z * sx)), w, s);
        ++N;
#if RT_OCT_SCALAR_EXIT
        // (A/B) the exit compares an opaque SGPR copy of N against each lane's count (one v_cmp), where loop
        // strength reduction counts every lane down (a v_add and a v_cmp per octave); N itself still
        // strides the constant loads
        Ne = N;
        asm volatile("" : "+s"(Ne));
    } while (Ne <= n_oct);
#else
    } while (N <= n_oct);
#endif
#elif !defined(RT_EXTRA_OCTAVE)
    // The octave-table pointer is the trip counter: a per-lane register from the start (the asm
    // keeps it out of SGPRs, which would cost a v_mov per iteration for the LDS address), one
    // v_add and one v_cmp against the lane's end per octave.  n_oct >= 2, so a do-while is exact.
    typedef float v4f __attribute__((ext_vector_type(4)));
    // volatile: one ds_read_b128 (4 LDS cycles, lane groups of 16 on one broadcast address) rather
    // than the b96 the compiler narrows an unused .w to (8 cycles: lane groups of 8)
    typedef __attribute__((address_space(3))) const volatile v4f lds_f4;
    uint32_t op = (uint32_t)(uintptr_t)(lds_f4*)(c.nz.oct + 1); // LDS byte address of octave 1
    asm volatile("" : "+v"(op));
    const uint32_t oe = op + (uint32_t)n_oct * 16u;
    #pragma unroll 1
    do {
        const v4f oc = *(lds_f4*)(uintptr_t)op;
        count_noise(c.nz);
        s = fma(noise3d_finish(c.nz, noise3d_cell<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x)), oc.z, s);
        op += 16u;
        asm("" : "+v"(op)); // opaque to loop strength reduction (which would add a second counter)
    } while (op != oe);
#else // cost experiment: RT_EXTRA_OCTAVE dead octaves per sample (weight 0: fma(v, 0, s) == s, s is never -0)
    #pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES + RT_EXTRA_OCTAVE; ++N) {
        if (N > n_oct + RT_EXTRA_OCTAVE) break;
        const float4 oc = c.nz.oct[N];
        count_noise(c.nz);
        s = fma(noise3d_finish(c.nz, noise3d_cell<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x)),
                N <= n_oct ? oc.z : 0.0f, s);
    }
#endif
    return s;
}

// Media/nomadplains/shaders/terrain.hlsl:8-39.  The steep noise, noise3d(x, z, 0), is evaluated
// by noise3d_z0.
__device__ __forceinline__ float density_nomadplains(const Ctx& c, f3 p)
{
    float d = -p.y;
    f3 p1 = rtm::scale(p, 0.4f);
    float s = 0.0f;
    f3 q0 = rtm::scale(p1, 0.006f);
    const int n_oct = np_octaves(c, p);
    // The octave cells take the short integer path (noise3d_cell<true>) when every lattice
    // coordinate of the wave's noises stays below kFastCellRange = 2^13 in magnitude: |q0| * S_n <
    // 2^13 for the lane's last octave n (S grows with N; the steep noise's coordinates are 1.19 |q0|
    // < S_1 |q0|).  2^13 is the bound of the magic-number texel offset (texel_offset: |512 f| < 2^22).
    // Wave-uniform, so the sample runs one of two copies.
    const float qm = rtm::max(rtm::max(rtm::abs(q0.x), rtm::abs(q0.y)), rtm::abs(q0.z));
    const bool fast = !__ballot(!(qm * c.nz.oct[n_oct].x < kFastCellRange));
    s = fast ? np_fbm<true>(c, q0, n_oct) : np_fbm<false>(c, q0, n_oct);
    s = rtm::pow_nonneg(rtm::abs(fma(s, 30.0f, 1.0f)) * 35.0f, c.k->np_expo);
    count_noise(c.nz);
    const float sn = fast ? noise3d_z0<true>(c.nz, p1.x * 0.007138f, p1.z * 0.007138f)
                          : noise3d_z0<false>(c.nz, p1.x * 0.007138f, p1.z * 0.007138f);
    float steep = rtm::sat((sn - 0.2f) * 6.0f) * 7.5f;
    s = terraces(s, p1.y, steep);
    // floor lift: pow(0, 1.5) == 0 exactly, so a wave whose bases are all 0 skips the pow
    const float lb = rtm::sat((-p1.y + 10.0f) * 1.6f);
    s = fma(__ballot(lb != 0.0f) ? rtm::pow_nonneg(lb, 1.5f) : 0.0f, 19.0f, s);
    return d + s;
}

#if RT_FBM_EXIT
// (A/B build, rt_variants.h RT_FBM_EXIT) density_nomadplains with an exact early exit.  d = -y + F(s) + G
// with F(s) = pow(|30 s + 1| 35, expo) and G (terraces + floor lift) independent of the FBM sum s.  After
// K octaves the rest add at most B (P[n] - P[K]) in magnitude (P: the octave weights' prefix sums, the
// LDS octave table's w column; B = kNoiseBound >= max |noise3d| for the {-1,0,1} edge gradients).  If
// every s in that interval gives d in [-5 + m, -m] (m: rounding margin), the march takes the no-hit
// unit step whatever the exact d is (stepmult = 1 + pow(0, df) = 1), so the sample returns -2.5 in
// place of d.  `allow` false (the march could exit after this sample) keeps the sample exact; the
// exact path is density_nomadplains's operation sequence, bit for bit.
constexpr float kNoiseBound = 1.05f; // grid maximum 1.0364 of sum_c w_c (two largest |f - c|), + slack
// octaves from LDS table address op up to (not including) oe, as np_fbm's loop
template <bool FAST>
__device__ __forceinline__ float fbm_range(const Ctx& c, f3 q0, uint32_t op, uint32_t oe, float s)
{
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const volatile v4f lds_f4;
    #pragma unroll 1
    do {
        const v4f oc = *(lds_f4*)(uintptr_t)op;
        count_noise(c.nz);
        s = fma(noise3d_finish(c.nz, noise3d_cell<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x)), oc.z, s);
        op += 16u;
        asm("" : "+v"(op));
    } while (op != oe);
    return s;
}
__device__ __forceinline__ float density_nomadplains_x(const Ctx& c, f3 p, bool allow)
{
    constexpr int K = RT_FBM_EXIT;
    float d = -p.y;
    f3 p1 = rtm::scale(p, 0.4f);
    f3 q0 = rtm::scale(p1, 0.006f);
    const int n_oct = np_octaves(c, p);
    const float qm = rtm::max(rtm::max(rtm::abs(q0.x), rtm::abs(q0.y)), rtm::abs(q0.z));
    const bool fast = !__ballot(!(qm * c.nz.oct[n_oct].x < kFastCellRange));
    count_noise(c.nz);
    const float sn = fast ? noise3d_z0<true>(c.nz, p1.x * 0.007138f, p1.z * 0.007138f)
                          : noise3d_z0<false>(c.nz, p1.x * 0.007138f, p1.z * 0.007138f);
    const float steep = rtm::sat((sn - 0.2f) * 6.0f) * 7.5f;
    const float lb = rtm::sat((-p1.y + 10.0f) * 1.6f);
    const float lift = __ballot(lb != 0.0f) ? rtm::pow_nonneg(lb, 1.5f) : 0.0f;
    uint32_t op = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float4*)(c.nz.oct + 1);
    asm volatile("" : "+v"(op));
    const int k1 = n_oct < K ? n_oct : K;
    const uint32_t o1 = op + (uint32_t)k1 * 16u, oe = op + (uint32_t)n_oct * 16u;
    float s = 0.0f;
    s = fast ? fbm_range<true>(c, q0, op, o1, s) : fbm_range<false>(c, q0, op, o1, s);
    op = o1;
    bool skip = false;
    const bool cand = allow && n_oct > K;
    if (__ballot(cand)) {
        const float G = fma(lift, 19.0f, terraces(0.0f, p1.y, steep));
        if (cand) {
            const float m = 0.01f + 1e-5f * rtm::abs(p.y);
            const float f_hi_ok = p.y - G - m, f_lo_ok = p.y - G - 5.0f + m; // d <= -m, d >= -5 + m
            const float P = c.nz.oct[n_oct].w - c.nz.oct[K].w;
            const float R = kNoiseBound * P * 1.0001f + 1e-6f * (rtm::abs(s) + 1.0f);
            const float u_lo = fma(s - R, 30.0f, 1.0f), u_hi = fma(s + R, 30.0f, 1.0f);
            const float a_lo = u_lo >= 0.0f ? u_lo : (u_hi <= 0.0f ? -u_hi : 0.0f);
            const float a_hi = rtm::max(-u_lo, u_hi);
            const float F_lo = rtm::pow_nonneg(a_lo * 35.0f, c.k->np_expo) * (1.0f - 1e-5f);
            const float F_hi = rtm::pow_nonneg(a_hi * 35.0f, c.k->np_expo) * (1.0f + 1e-5f);
            skip = F_lo >= f_lo_ok && F_hi <= f_hi_ok;
        }
    }
    if (!skip && n_oct > k1) {
        s = fast ? fbm_range<true>(c, q0, op, oe, s) : fbm_range<false>(c, q0, op, oe, s);
    }
    if (skip) return -2.5f;
    s = rtm::pow_nonneg(rtm::abs(fma(s, 30.0f, 1.0f)) * 35.0f, c.k->np_expo);
    s = terraces(s, p1.y, steep);
    s = fma(lift, 19.0f, s);
    return d + s;
}
#endif

// density_nomadplains with the FBM spread over a segment of LPR lanes that march ONE
// ray together (the camerarays prepass: 1024 latency-bound rays for 256 CUs).  The 18 noise values of a sample are numbered
// v = 0 (the steep noise) and v = N (octave N = 1..17); lane j of the segment evaluates
// v = j, j + LPR, j + 2 LPR, ... (rounds), then every lane gathers the values in v order
// and runs the same fma chain, so the result is bit-identical to density_nomadplains.
// `base` = first lane of the segment within the wave; every lane of a segment must be
// active (the gathers read all of them).
template <int LPR>
struct SegOctaves {
    static constexpr int NV = RT_NP_OCTAVES + 1;   // values per sample
    static constexpr int R = (NV + LPR - 1) / LPR; // rounds per lane
    float sx[R], sy[R];                            // noise-input scales of this lane's values
    float rcp[RT_NP_OCTAVES + 1];                  // octave weights 1/S (uniform)
};

template <int LPR>
__device__ __forceinline__ SegOctaves<LPR> seg_octaves(const Ctx& c, uint32_t j)
{
    SegOctaves<LPR> g;
#pragma unroll
    for (int r = 0; r < SegOctaves<LPR>::R; ++r) {
        const uint32_t v = (uint32_t)(r * LPR) + j;
        const uint32_t o = v >= 1u && v <= (uint32_t)RT_NP_OCTAVES ? v : 1u;
        g.sx[r] = c.k->np_scale[o];
        g.sy[r] = c.k->np_scale_y[o];
    }
#pragma unroll
    for (int N = 1; N <= RT_NP_OCTAVES; ++N) g.rcp[N] = c.k->np_rcp[N];
    return g;
}

// The weighted sum for segments of LPR <= 16 lanes (a segment then lies inside one 16-lane DPP row):
// octave N's value is nv[N / LPR] of lane base + N % LPR, and the segment's first lane reads it with a
// DPP row shift (v_mov_b32 row_shl:k, lane i <- lane i + k of its row) that the fma takes as its
// operand: no LDS round trip, no lane-index VGPR, and the chain's 17 fmas are its only serial part.
// The other lanes of the segment run the same instructions on values from the wrong lanes; the
// caller broadcasts the first lane's result (seg_bcast).
template <int LPR, int N, int R>
__device__ __forceinline__ float seg_chain_dpp(const float (&nv)[R], const float (&rcp)[RT_NP_OCTAVES + 1], float s)
{
    if constexpr (N > RT_NP_OCTAVES) {
        return s;
    } else {
        constexpr int k = N % LPR;
        float x;
        if constexpr (k == 0) x = nv[N / LPR];
        else x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(nv[N / LPR]), 0x100 + k, 0xf, 0xf, false));
        return seg_chain_dpp<LPR, N + 1>(nv, rcp, fma(x, rcp[N], s));
    }
}

// every lane of an LPR-lane segment (LPR 4, 8 or 16) <- the segment's first lane, in DPP moves:
// quad_perm [0,0,0,0] (each quad <- its lane 0), then row_shr:4 into banks 1 and 3 and row_shr:8 into
// banks 2 and 3 (the lanes outside the bank mask keep their value)
template <int LPR>
__device__ __forceinline__ float seg_bcast(float x)
{
    static_assert(LPR == 4 || LPR == 8 || LPR == 16, "DPP broadcast within one 16-lane row");
    int v = __float_as_int(x);
    v = __builtin_amdgcn_update_dpp(v, v, 0x00, 0xf, 0xf, false);
    if constexpr (LPR >= 8) v = __builtin_amdgcn_update_dpp(v, v, 0x114, 0xf, 0xa, false);
    if constexpr (LPR >= 16) v = __builtin_amdgcn_update_dpp(v, v, 0x118, 0xf, 0xc, false);
    return __int_as_float(v);
}

// LOWREG (LPR 32 only; the DPP form holds no gathered values): the octave values are gathered one at a
// time inside the weighted sum (each gather waits for the previous fma), so one gathered value is live
// instead of all 18.  LOWREG (any LPR): each round's octave scales come from the LDS octave table
// (nz.oct: the same np_scale / np_scale_y values) instead of registers: for callers that hold other
// rays' state across the march (k_trace's primary_seg).
template <int LPR, bool LOWREG = false>
__device__ __forceinline__ float density_nomadplains_seg(const Ctx& c, const SegOctaves<LPR>& g, f3 p, uint32_t j,
                                                         uint32_t base, uint32_t* octaves)
{
    constexpr int NV = SegOctaves<LPR>::NV, R = SegOctaves<LPR>::R;
    float d = -p.y;
    f3 p1 = rtm::scale(p, 0.4f);
    f3 q0 = rtm::scale(p1, 0.006f);
    // N = 1 .. floor(detail) in order.  A dead octave's value is +0 instead of being
    // skipped: fma(+0, w, s) == s bit for bit because s is never -0 (it starts at +0 and
    // an exact cancellation rounds to +0), so the serial chain needs no selects.  A round
    // no lane of the wave needs (all its octaves dead) is not evaluated at all.
    const int n_oct = np_octaves(c, p);
    float nv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t v = (uint32_t)(r * LPR) + j;
        const bool need = v < (uint32_t)NV && (v == 0u || (int)v <= n_oct);
        float n = 0.0f;
        // RT_SEG_ILP (not LOWREG): every round is evaluated, so the rounds' LDS round trips overlap
        // (no branch between them); a dead round's value is masked to +0 below
        if ((RT_SEG_ILP && !LOWREG) || __ballot(need)) {
            float sx = g.sx[r], sy = g.sy[r];
            if constexpr (LOWREG) { // the same scales from the LDS octave table, per round (no VGPRs held)
                typedef __attribute__((address_space(3))) const float lds_f;
                const uint32_t o = v >= 1u && v <= (uint32_t)RT_NP_OCTAVES ? v : 1u;
                const lds_f* sc = (const lds_f*)(c.nz.oct + o);
                sx = sc[0];
                sy = sc[1];
            }
            float nx = q0.x * sx, ny = q0.y * sy, nzz = q0.z * sx;
            if (r == 0 && v == 0u) {
                nx = p1.x * 0.007138f;
                ny = p1.z * 0.007138f;
                nzz = 0.0f;
            }
            n = noise3d_raw(c.nz, nx, ny, nzz);
        }
        nv[r] = need ? n : 0.0f;
    }
    float s = 0.0f, on0;
    constexpr bool kDpp = RT_SEG_DPP && LPR <= 16;
    if constexpr (kDpp) {
        s = seg_chain_dpp<LPR, 1>(nv, g.rcp, s);
        on0 = nv[0]; // (the first lane's own v = 0)
    } else if constexpr (LOWREG) {
#pragma unroll
        for (int N = 1; N <= RT_NP_OCTAVES; ++N) {
            int idx = (int)(base + (uint32_t)(N % LPR));
            asm volatile("" : "+v"(idx) : "v"(s)); // this gather after the previous fma
            s = fma(__shfl(nv[N / LPR], idx, 64), g.rcp[N], s);
        }
        on0 = __shfl(nv[0], (int)base, 64);
    } else {
        float on[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) on[v] = __shfl(nv[v / LPR], (int)(base + (uint32_t)(v % LPR)), 64);
#pragma unroll
        for (int N = 1; N <= RT_NP_OCTAVES; ++N) s = fma(on[N], g.rcp[N], s);
        on0 = on[0];
    }
    *octaves = (uint32_t)n_oct;
    s = rtm::pow_nonneg_flat(rtm::abs(fma(s, 30.0f, 1.0f)) * 35.0f, c.k->np_expo);
    float steep = rtm::sat((on0 - 0.2f) * 6.0f) * 7.5f;
    s = terraces(s, p1.y, steep);
    // floor lift: pow(0, 1.5) == 0 exactly, so a wave whose bases are all 0 (every
    // sample above y = 25, the common case) skips the polynomial
    const float lb = rtm::sat((-p1.y + 10.0f) * 1.6f);
    const float lift = __ballot(lb != 0.0f) ? rtm::pow_nonneg_flat(lb, 1.5f) : 0.0f;
    s = fma(lift, 19.0f, s);
    if constexpr (kDpp) return seg_bcast<LPR>(d + s); // the first lane's density to its segment
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
    // serialise the four independent lattice evaluations (register pressure)
    asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z) : "v"(n));
    f3 q2 = rtm::scale(p, 0.002f);
    float w2 = rtm::min(rtm::max(fma(-p.y, 1.5f, 50.0f), 0.0f), 36.0f);
    n = fma(-fma(noise3d(c.nz, q2.x, q2.y, q2.z), 0.5f, 0.5f), w2, n);
    asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z) : "v"(n));
    f3 q3 = rtm::scale(p, 0.003f);
    float w3 = rtm::min(rtm::max(fma(-p.y, 1.5f, 10.0f), 0.0f), 36.0f);
    n = fma(-fma(noise3d(c.nz, q3.x, q3.y, q3.z), 0.5f, 0.5f), w3, n);
    asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z) : "v"(n));
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
#pragma unroll 1
    for (int N = 1; N <= 7; ++N) {
        float S = (float)(1 << N); // pow(2, N) is exact under R5
        float n = noise3d(c.nz, fma(pc.x, S, g32), fma(pc.y, S, g32), fma(pc.z, S, g32));
        d = fma((rtm::abs(n) * 210.0f) * g, rtm::rcp(S), d);
    }
    d = d - 50.0f;
    f3 p2 = rtm::scale(p, 0.002f);
    f3 p2n = rtm::mk(p2.x * 1.0f, p2.y * nohy, p2.z * 1.0f);
#pragma unroll 1
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
    float sd; // the last sample's distance (pd.xyz = p + dir * sd)
};

// Media/common/shaders/tracing.hlsl:47-105 (+ build extension max_steps) as an
// explicit state machine: march_begin = the prologue (:49-66), march_live = the
// loop condition (:68, the max_steps cap and SKIPREFINE's break on a hit),
// march_step = one loop body (:70-103).  trace_ray runs it to completion; the
// lane-refill kernels advance each lane's ray one step at a time and hand a lane
// a new ray as soon as its old one leaves the loop.
template <int L, bool CALCFOG>
struct March {
    static constexpr bool FOG = CALCFOG && FogLive<L>::value;
    f3 p, dir;
    float sd; // the distance of the last density sample: that sample is at p + dir * sd (march_result)
    float dist, step, lastStep, d;
    f4 f;
    int iters;
    bool fog; // calcfog at run time (AO rays share the shadow lanes but march without fog)
};

template <int L, bool CALCFOG>
__device__ __forceinline__ void march_begin(const Ctx& c, March<L, CALCFOG>& m, f3 p, float dist, float stepmod, f3 dir,
                                            bool fog = true)
{
    m.fog = fog;
    const RtConsts* k = c.k;
    m.f = {0.0f, 0.0f, 0.0f, 0.0f};
    m.d = 0.0f;
    float dirLength = rtm::length(dir);
    // tracing.hlsl:54, the one R2 exception: the subtrahend's product is fused
    m.step = fma(-dist, k->one_minus_step_factor, (0.03f * stepmod) * dirLength);
    m.lastStep = m.step;
    float il = rtm::rcp(dirLength);
    dir = rtm::scale(dir, il);
    if constexpr (March<L, CALCFOG>::FOG) if (fog) {
        float hd = dist * 0.5f;
        f3 mp = rtm::mk(fma(dir.x * dist, 0.5f, p.x), fma(dir.y * dist, 0.5f, p.y), fma(dir.z * dist, 0.5f, p.z));
        f4 mf = get_fog<L>(c, mp, hd);
        m.f.x = fma(mf.x, dist, m.f.x);
        m.f.y = fma(mf.y, dist, m.f.y);
        m.f.z = fma(mf.z, dist, m.f.z);
        m.f.w = fma(mf.w, dist, m.f.w);
    }
    m.p = p;
    m.dir = dir;
    m.dist = dist;
    m.sd = 0.0f;
    m.iters = 0;
}

template <int L, bool CALCFOG, bool SKIPREFINE>
__device__ __forceinline__ bool march_live(const Ctx& c, const March<L, CALCFOG>& m, float enddist, int max_steps)
{
    if (SKIPREFINE && m.d > 0.0f) return false; // tracing.hlsl:84 `break` on a hit
    return m.dist < enddist && m.step > c.k->min_limit && !(max_steps > 0 && m.iters >= max_steps);
}

template <int L, bool CALCFOG, bool SKIPREFINE, class Density, bool FLAT = false>
__device__ __forceinline__ void march_step_with(const Ctx& c, March<L, CALCFOG>& m, Density density)
{
    const RtConsts* k = c.k;
    ++m.iters;
    const f3 rayp = rtm::mk(fma(m.dir.x, m.dist, m.p.x), fma(m.dir.y, m.dist, m.p.y), fma(m.dir.z, m.dist, m.p.z));
    m.sd = m.dist;
    m.d = density(rayp);
    f4 fs = {0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (March<L, CALCFOG>::FOG) if (m.fog) {
        f4 g = get_fog<L>(c, rayp, m.dist);
        fs.x = g.x * m.step;
        fs.y = g.y * m.step;
        fs.z = g.z * m.step;
        fs.w = g.w * m.step;
    }
    // without fog fs is +0 and m.f stays +0 (+0 + +0 == +0 - +0 == +0): no updates
    constexpr bool kFog = March<L, CALCFOG>::FOG;
    if (m.d > 0.0f) {
        if constexpr (SKIPREFINE) return;
        m.dist = m.dist - m.lastStep;
        m.step = m.step * 0.3f;
        if constexpr (kFog) {
            m.f.x = m.f.x - fs.x;
            m.f.y = m.f.y - fs.y;
            m.f.z = m.f.z - fs.z;
            m.f.w = m.f.w - fs.w;
        }
    } else {
        const float sx = rtm::abs(rtm::min(m.d + 5.0f, 0.0f));
        float stepmult;
        // pow(0, y > 0) == 0: a wave of zero bases (all samples within 5 of the
        // surface) skips the polynomial
        if constexpr (FLAT) stepmult = 1.0f + (__ballot(sx != 0.0f) ? rtm::pow_nonneg_flat(sx, k->density_factor) : 0.0f);
        else stepmult = 1.0f + rtm::pow_nonneg(sx, k->density_factor);
        m.step = m.step * k->step_factor;
        m.lastStep = m.step * stepmult;
        m.dist = m.dist + m.lastStep;
        if constexpr (kFog) {
            m.f.x = m.f.x + fs.x;
            m.f.y = m.f.y + fs.y;
            m.f.z = m.f.z + fs.z;
            m.f.w = m.f.w + fs.w;
        }
    }
}

template <int L, bool CALCFOG, bool SKIPREFINE>
__device__ __forceinline__ void march_step(const Ctx& c, March<L, CALCFOG>& m)
{
    march_step_with<L, CALCFOG, SKIPREFINE>(c, m, [&](f3 q) { return get_density<L>(c, q); });
}

template <int L, bool CALCFOG>
__device__ __forceinline__ RayResult march_result(const March<L, CALCFOG>& m)
{
    RayResult rr;
    // the last sample's position, recomputed from its distance with the step's own fma (no step:
    // rayp's initial 0); carrying one distance instead of the position frees 2 VGPRs per march
    const bool stepped = m.iters > 0;
    rr.pd.x = stepped ? fma(m.dir.x, m.sd, m.p.x) : 0.0f;
    rr.pd.y = stepped ? fma(m.dir.y, m.sd, m.p.y) : 0.0f;
    rr.pd.z = stepped ? fma(m.dir.z, m.sd, m.p.z) : 0.0f;
    rr.sd = m.sd;
    rr.pd.w = m.dist;
    rr.fc = m.f;
    rr.density = m.d;
    rr.steps = (float)m.iters; // `total` (:71) counts loop iterations
    return rr;
}

template <int L, bool CALCFOG, bool SKIPREFINE>
__device__ __forceinline__ RayResult trace_ray(const Ctx& c, f3 p, float dist, float enddist, float stepmod, f3 dir,
                                               int max_steps)
{
    March<L, CALCFOG> m;
    march_begin(c, m, p, dist, stepmod, dir);
    while (march_live<L, CALCFOG, SKIPREFINE>(c, m, enddist, max_steps)) march_step<L, CALCFOG, SKIPREFINE>(c, m);
    return march_result(m);
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
    sx = sx * c.kf->proj22;
    sy = sy * c.kf->proj11;
    const auto* m = c.kf->view_inverse;
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
    const KPtr kf = c.kf;
    float far = fma((1.0f - rd.y) * kf->sky_dist_to_top, 2.0f, kf->sky_dist_to_top);
    f3 start = rtm::mk(kf->sky_start[0], kf->sky_start[1], kf->sky_start[2]);
    float fStartAngle = rtm::dot(rd, rtm::mk(kf->sky_start_n[0], kf->sky_start_n[1], kf->sky_start_n[2]));
    float fStartOffset = kf->sky_depth0 * sky_scale(fStartAngle);
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
// color.hlsl:47-49: the shadow ray's stepmod from the hit distance (mip level)
__device__ __forceinline__ float shade_precision(float dist)
{
    float mipf = rtm::max(0.5f * rtm::log2_nonneg(dist), 0.0f);
    return rtm::max((mipf - 3.2f) * 3.0f, 1.0f) * 8.0f;
}

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
            #pragma unroll 1
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
    r.precision = shade_precision(dist);
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

// ---------------------------------------------------------------------------
// Build extension, BASELINE.json configs C3/C5 ("1-bounce AO"; the reference has no
// ambient occlusion, so the definition is the build's own, restated identically in
// oracle/rt_oracle.c ao_dir / ambient_occlusion): per primary hit, AO_SAMPLES
// cosine-weighted hemisphere rays about the normal, direction from a PCG hash of
// (pixel, AA sample, k), marched as traceRay(p, 0.4, 25, shadow stepmod, dir,
// no fog, skiprefine); ao = 1 - 0.6 * occluded / AO multiplies the saturated sample.
#define RT_AO_END 25.0f
#define RT_AO_STRENGTH 0.6f

__device__ __forceinline__ uint32_t pcg_hash(uint32_t x)
{
    uint32_t st = x * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}

__device__ __forceinline__ f3 cross3(f3 a, f3 b)
{
    return rtm::mk(fma(a.y, b.z, -(a.z * b.y)), fma(a.z, b.x, -(a.x * b.z)), fma(a.x, b.y, -(a.y * b.x)));
}

__device__ __forceinline__ f3 ao_dir(f3 n, uint32_t px, uint32_t py, uint32_t a, uint32_t k)
{
    uint32_t h = pcg_hash((px * 0x9E3779B1u) ^ (py * 0x85EBCA77u) ^ ((a * 16u + k) * 0xC2B2AE3Du));
    uint32_t h2 = pcg_hash(h);
    float u1 = (float)(h >> 8) * 0x1p-24f, u2 = (float)(h2 >> 8) * 0x1p-24f;
    float r = rtm::sqrt(u1);
    float sn, cs;
    rtm::sincos(u2 * 6.2831855f, &sn, &cs);
    float sx = r * cs, sy = r * sn, sz = rtm::sqrt(rtm::max(1.0f - u1, 0.0f));
    f3 up = rtm::abs(n.x) > 0.9f ? rtm::mk(0.0f, 1.0f, 0.0f) : rtm::mk(1.0f, 0.0f, 0.0f);
    f3 tx = rtm::normalize(cross3(up, n));
    f3 ty = cross3(n, tx);
    return rtm::mk(fma(tx.x, sx, fma(ty.x, sy, n.x * sz)), fma(tx.y, sx, fma(ty.y, sy, n.y * sz)),
                   fma(tx.z, sx, fma(ty.z, sy, n.z * sz)));
}

__device__ __forceinline__ float ao_factor(uint32_t occluded, int ao)
{
    return fma(-RT_AO_STRENGTH, (float)occluded * rtm::rcp((float)ao), 1.0f);
}

__device__ __forceinline__ uint32_t unorm8(float v) { return (uint32_t)rtm::rint(rtm::sat(v) * 255.0f); }

} // namespace rts
