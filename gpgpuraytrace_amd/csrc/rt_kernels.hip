// rt_kernels.hip -- HIP kernels for gfx950 (MI355X).
//
//   k_camerarays   <- Media/common/shaders/camerarays.hlsl:12-21
//   k_order        <- Graphics/Terrain.cpp:356-439 (setTargetDepths: host code in
//                     the reference; on the device here so a frame needs no
//                     GPU->CPU->GPU round trip)
//   k_order (+ the longest-first tile order), k_trace, k_finish
//                  <- Media/common/shaders/tracescreen.hlsl:16-76 (split pipeline below)
//   k_shard_copy   -- tile-cyclic shard pack/unpack for the multi-GPU gather
//
// k_trace is a persistent kernel: one 1024-thread workgroup per CU keeps the noise
// tables (128 KiB) in LDS and every wave pulls 8x8-pixel work units from a device-wide
// atomic queue, so a finished wave takes new work instead of idling until the slowest
// wave of its workgroup retires.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "rt_kernels.h"
#include "rt_shader.h"
#include "rt_variants.h"

using namespace rts;
using rtm::f3;

namespace {

// LDS image (rts::NoiseView): perm2D texels at offset 0 (64 KiB), the paired lane-private
// gradients gxy at kLdsGxy (32 KiB) and gz at kLdsGz (32 KiB, 8 of every 16 B used), then the
// nomadplains FBM octave constants (NoiseView::oct): (S, 0.35 S, 1/S, 0) for N = 0..RT_NP_OCTAVES + 2
// (the entries past the last octave are padding).  A kernel declares it as its ONLY static LDS array, so it sits
// at LDS address 0 and the texel address needs no base (other LDS a kernel needs is carved after it).
constexpr int kPermWords = 128 * 128;
constexpr int kNpOct = RT_NP_OCTAVES + 3;
constexpr int kOctWords = kNpOct * 4;
constexpr int kOctBase = (int)kLdsGz / 4 + (int)(kLdsGz - kLdsGxy) / 4; // words
constexpr int kNoiseLdsWords = kOctBase + kOctWords;
static_assert(kNoiseLdsWords % 4 == 0, "LDS carved after the noise image stays 16-byte aligned");
static_assert(kLdsGxy == (uint32_t)kPermWords * 4u, "gxy follows the perm2D texels");

__device__ __forceinline__ void load_noise_lds(uint32_t* lds, const uint32_t* __restrict__ perm2d,
                                               const float4* __restrict__ grad, const RtConsts* __restrict__ k)
{
    {
        float4* oct = reinterpret_cast<float4*>(lds + kOctBase);
        const int i = threadIdx.x;
        if (i < kNpOct) {
            const int n = i <= RT_NP_OCTAVES ? i : RT_NP_OCTAVES;
            float pre = 0.0f; // RT_FBM_EXIT: sum of the octave weights 1 .. n (the suffix bound's prefix)
#if RT_FBM_EXIT
            for (int m = 1; m <= n; ++m) pre += k->np_rcp[m];
#endif
            oct[i] = make_float4(k->np_scale[n], k->np_scale_y[n], k->np_rcp[n], pre);
        }
    }
    float4* gxy = reinterpret_cast<float4*>(lds + kLdsGxy / 4);
    float4* gz = reinterpret_cast<float4*>(lds + kLdsGz / 4); // gxy's slot layout, 8 of 16 B used
    for (int i = threadIdx.x; i < 128 * 16; i += blockDim.x) {
        int e = i >> 4;
        float4 g0 = grad[e], g1 = grad[(e + 1) & 127];
        gxy[i] = make_float4(g0.x, g1.x, g0.y, g1.y);
        gz[i] = make_float4(g0.z, g1.z, 0.0f, 0.0f);
    }
    uint4* p = reinterpret_cast<uint4*>(lds);
    const uint4* src = reinterpret_cast<const uint4*>(perm2d);
    for (int i = threadIdx.x; i < kPermWords / 4; i += blockDim.x) p[i] = src[i];
    __syncthreads();
}

// A buffer pointer read from a FrameTable, as a global-address-space pointer: plain pointers
// loaded from memory are generic, and their accesses flat instructions that wait on the LDS
// counter too.
template <class T>
__device__ __forceinline__ T __attribute__((address_space(1)))* gptr(T* p)
{
    return (T __attribute__((address_space(1)))*)p;
}
__device__ __forceinline__ void gstore(float4* p, float4 v)
{
    typedef float v4f __attribute__((ext_vector_type(4)));
    *(v4f __attribute__((address_space(1)))*)p = v4f{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ Ctx make_ctx(const RtConsts* k, const uint32_t* lds)
{
    Ctx c;
    c.nz.img = reinterpret_cast<const char*>(lds);
    c.nz.oct = reinterpret_cast<const float4*>(lds + kOctBase);
    c.nz.so16 = kLdsGxy | ((threadIdx.x & (RT_LDS_SLOTS - 1u)) * 16u);
    c.nz.calls = 0;
    c.nz.lds_calls = nullptr;
    c.nz.phase = RT_PHASE_OTHER;
    c.k = k;
    c.kf = (KPtr)k;
    c.eye = rtm::mk(k->eye[0], k->eye[1], k->eye[2]);
    c.sun = rtm::mk(k->sun[0], k->sun[1], k->sun[2]);
    return c;
}

// STATS kernels: a lane's noise count (NoiseView::calls) into the frame statistics
__device__ __forceinline__ void stats_noise(RtStats* stats, uint64_t calls)
{
    atomicAdd(&stats->noise_calls, (unsigned long long)(calls & 0xffffffffull));
    if (calls >> 32) atomicAdd(&stats->noise_waves, (unsigned long long)(calls >> 32));
}

__device__ __forceinline__ float uniform_f(float x)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

// prepass frame f of a batch: its camerarays block (camera) as kf, Eye/Sun uniform
__device__ __forceinline__ Ctx frame_ctx_cam(const Ctx& c, const FrameTable* __restrict__ ft, uint32_t f)
{
    Ctx cf = c;
    cf.kf = (KPtr)ft->kcam[f];
    cf.eye = rtm::mk(uniform_f(cf.kf->eye[0]), uniform_f(cf.kf->eye[1]), uniform_f(cf.kf->eye[2]));
    cf.sun = rtm::mk(uniform_f(cf.kf->sun[0]), uniform_f(cf.kf->sun[1]), uniform_f(cf.kf->sun[2]));
    return cf;
}

// ---------------------------------------------------------------------------
// camerarays.hlsl:12-21.  One thread per prepass cell (32x32).
// ft != null: frame blockIdx.y of a batch (its constants and CameraResults from the table).
template <int L, bool STATS>
__global__ void __launch_bounds__(64) k_camerarays(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                                   const float4* __restrict__ grad, float4* __restrict__ out,
                                                   RtStats* stats, const FrameTable* __restrict__ ft)
{
    if (ft) out = ft->cam[blockIdx.y];
    __shared__ __attribute__((aligned(16))) uint32_t lds[kNoiseLdsWords];
    load_noise_lds(lds, perm2d, grad, k);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= RT_CAMERA_RES * RT_CAMERA_RES) return;
    Ctx c = make_ctx(k, lds);
    if (ft) c = frame_ctx_cam(c, ft, blockIdx.y);
    int tx = i % RT_CAMERA_RES, ty = i / RT_CAMERA_RES;
    const float r31 = rtm::rcp(31.0f);
    uint32_t pxs = (uint32_t)(((float)tx * r31) * k->screen[0]);
    uint32_t pys = (uint32_t)(((float)ty * r31) * k->screen[1]);
    f3 p, dir;
    get_pixel_ray(c, (float)pxs, (float)pys, &p, &dir);
    RayResult rr = trace_ray<L, false, true>(c, p, RT_CAMERA_NEAR, RT_CAMERA_FAR, 2.0f, dir, 0);
    if (rr.density < 0.0f) rr.pd.w = RT_CAMERA_FAR;
    out[i] = make_float4(rr.pd.x, rr.pd.y, rr.pd.z, rr.pd.w);
    if constexpr (STATS) {
        atomicAdd(&stats->prepass_steps, (unsigned long long)rr.steps);
        stats_noise(stats, c.nz.calls);
    }
}

// camerarays.hlsl:12-21 for nomadplains with one 32-lane group per prepass ray:
// the prepass is 1024 sequential marches of ~350 steps, so it is bound by the
// latency of one step, and spreading each step's 17 FBM octaves + steep noise over
// a lane group (rts::density_nomadplains_seg<LPR>, LPR lanes per ray) shortens that chain ~4x.
template <bool STATS, int BS, int LPR>
__global__ void __launch_bounds__(BS) k_camerarays_group(const RtConsts* __restrict__ k,
                                                          const uint32_t* __restrict__ perm2d,
                                                          const float4* __restrict__ grad, float4* __restrict__ out,
                                                          RtStats* stats, const FrameTable* __restrict__ ft)
{
    constexpr int L = RT_NOMADPLAINS;
    if (ft) out = ft->cam[blockIdx.y];
    __shared__ __attribute__((aligned(16))) uint32_t lds[kNoiseLdsWords];
    load_noise_lds(lds, perm2d, grad, k);
    const int i = blockIdx.x * (BS / LPR) + (int)(threadIdx.x / LPR);
    if (i >= RT_CAMERA_RES * RT_CAMERA_RES) return; // whole groups leave together
    Ctx c = make_ctx(k, lds);
    if (ft) c = frame_ctx_cam(c, ft, blockIdx.y);
    const uint32_t j = threadIdx.x & (LPR - 1u), base = threadIdx.x & 63u & ~(LPR - 1u);
    const SegOctaves<LPR> g = seg_octaves<LPR>(c, j);
    int tx = i % RT_CAMERA_RES, ty = i / RT_CAMERA_RES;
    const float r31 = rtm::rcp(31.0f);
    uint32_t pxs = (uint32_t)(((float)tx * r31) * k->screen[0]);
    uint32_t pys = (uint32_t)(((float)ty * r31) * k->screen[1]);
    f3 p, dir;
    get_pixel_ray(c, (float)pxs, (float)pys, &p, &dir);
    March<L, false> st;
    march_begin(c, st, p, RT_CAMERA_NEAR, 2.0f, dir);
    uint32_t noise = 0;
    while (march_live<L, false, true>(c, st, RT_CAMERA_FAR, 0)) {
        auto dens = [&](f3 q) {
            uint32_t used;
            float d = density_nomadplains_seg<LPR>(c, g, q, j, base, &used);
            noise += used + 1u;
            return d;
        };
        march_step_with<L, false, true, decltype(dens), true>(c, st, dens);
    }
    RayResult rr = march_result(st);
    if (rr.density < 0.0f) rr.pd.w = RT_CAMERA_FAR;
    if (j == 0) {
        out[i] = make_float4(rr.pd.x, rr.pd.y, rr.pd.z, rr.pd.w);
        if constexpr (STATS) {
            atomicAdd(&stats->prepass_steps, (unsigned long long)rr.steps);
            atomicAdd(&stats->noise_calls, (unsigned long long)noise);
        }
    }
}

// ---------------------------------------------------------------------------
// Terrain.cpp:356-439 with the host's std::min/std::max argument order.  `depth(x, y)` reads the
// CameraResults depth of prepass ray (x, y) (coordinates already clamped to the 32 x 32 grid): from an
// LDS copy (k_order) or straight from the frame's CameraResults (the gated launch's lanes).
template <class Depth>
__device__ __forceinline__ float cd_get_depth(Depth depth, int x, int y)
{
    x = x < 0 ? 0 : (x >= RT_CAMERA_RES ? RT_CAMERA_RES - 1 : x);
    y = y < 0 ? 0 : (y >= RT_CAMERA_RES ? RT_CAMERA_RES - 1 : y);
    return depth(x, y);
}
template <class Depth>
__device__ __forceinline__ float cd_interp(Depth d, int x, int y)
{
    if (x < 0) {
        float m = cd_get_depth(d, x + 1, y);
        float dd = cd_get_depth(d, x + 2, y) - m;
        return m - dd;
    }
    if (x >= RT_CAMERA_RES) {
        float m = cd_get_depth(d, x - 1, y);
        float dd = cd_get_depth(d, x - 2, y) - m;
        return m - dd;
    }
    if (y < 0) {
        float m = cd_get_depth(d, x, y + 1);
        float dd = cd_get_depth(d, x, y + 2) - m;
        return m - dd;
    }
    if (y >= RT_CAMERA_RES) {
        float m = cd_get_depth(d, x, y - 1);
        float dd = cd_get_depth(d, x, y - 2) - m;
        return m - dd;
    }
    return cd_get_depth(d, x, y);
}

// setTargetDepths (Terrain.cpp:398-439) of cell (xpos, ypos): its (dmin, dmax) bracket from the 5 x 5
// neighbourhood of prepass depths
template <class Depth>
__device__ __forceinline__ float2 cell_bracket(Depth depth, int xpos, int ypos)
{
    float dmin = cd_interp(depth, xpos, ypos);
    float dmax = dmin;
    for (int xp = -2; xp <= 2; ++xp) {
        for (int yp = -2; yp <= 2; ++yp) {
            float d = cd_interp(depth, xpos + xp, ypos + yp);
            dmin = (dmin < d) ? dmin : d;
            dmax = (d < dmax) ? dmax : d;
        }
    }
    dmin = dmin * 0.96f - 0.01f;
    dmax = dmax * 1.22f + 0.4f;
    dmin = (RT_CAMERA_NEAR < dmin) ? dmin : RT_CAMERA_NEAR;
    dmax = (dmax < RT_CAMERA_FAR) ? dmax : RT_CAMERA_FAR;
    return make_float2(dmin, dmax);
}

// a prepass depth read straight from CameraResults another wave stored with sc1 (FusedPrepass, the
// gated launch): an sc1 global_load_dword, after the poll of the writers' flag or counter matched
__device__ __forceinline__ float cam_depth_sc1(const float4* cam, int x, int y)
{
    typedef const float __attribute__((address_space(1))) gfloat;
    return __hip_atomic_load((gfloat*)(reinterpret_cast<const float*>(cam + y * RT_CAMERA_RES + x) + 3),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// setTargetDepths of one frame by a 1024-thread block (thread = cell), depth scratch in LDS
__device__ __forceinline__ void cell_depths_frame(const float4* __restrict__ cam, float2* __restrict__ cells,
                                                  float* s_d)
{
    const int i = threadIdx.x;
    __syncthreads(); // s_d's previous frame is no longer read
    // sc1 (L1-bypassing) load: a fused prepass wrote these in another kernel (FusedPrepass; the
    // hand-off's loads are all global_load_dword sc1 after k_order's poll and barrier)
    s_d[i] = cam_depth_sc1(cam, i % RT_CAMERA_RES, i / RT_CAMERA_RES);
    __syncthreads();
    cells[i] = cell_bracket([&](int x, int y) { return s_d[y * RT_CAMERA_RES + x]; }, i % RT_CAMERA_RES,
                            i / RT_CAMERA_RES);
}

// ===========================================================================
// Screen pipeline: tracescreen.hlsl:16-76 over a batch of frames in four launches.
//   k_order     : longest-first 32x32 tile order per frame (scheduling only).
//   k_trace     : persistent; primary march (tracing.hlsl:47-105) per 8x8 unit, the hit
//                 shading + first shadow step, the long shadow / AO rays (LDS rings).
//   k_finish    : sky colour of the misses + in-order AA average + UNORM8.
// Sample t = (u*64 + j)*AA + a: AA sample a of lane-slot j of 8x8 unit u.
// A batch of n_frames frames: unit g of the launch is unit g % n_units of frame g / n_units
// (frame-major, so a frame's tail overlaps the next frame's units), and sample ids are
// global: frame f's sample t is f * frame_samples + t (frame_samples = n_units * 64 * AA).
struct UnitMap {
    uint32_t off_x, off_y, ext_x, ext_y, tiles32_x, tile_first, tile_stride, n_units;
    uint32_t n_frames, frame_samples;
    uint32_t frame_rot; // 1: frame f of a batch traces shard (tile_first + f) % tile_stride
    uint32_t order_batch; // k_order: 1 one longest-first order over the batch, 0 one per frame (frame-major)
    uint32_t cells_from_cam; // k_order first derives each frame's CellDistance from its CameraResults
    // 1: one sample per pixel, no float output, <= 1 AO ray per hit: hit pixels are finished in k_trace
    // where their last ray ends (fit_pixel), and k_finish only finishes the hits whose long shadow and
    // AO ray race (their bit in hitmask); with no AO, no k_finish at all
    uint32_t fit;
    // 1: one sample per pixel, no float output, >= 2 AO rays per hit: a hit whose shadow ends at its first
    // step (no long shadow) keeps its colour in its block's colour pool beside its AO counter slot, and the
    // AO ray that completes the count stores the pixel (fitm in k_trace); the rest go through k_finish,
    // flagged as with fit
    uint32_t fitm;
    // 1: out8[f] is this rank's PACKED shard buffer of frame f (k_shard_copy's layout: the shard's k-th tile
    // at k * 1024 pixels, rows of 32 within the tile), written in place of the framebuffer, so a sharded
    // batch needs no pack launch before its gather (RGBA8 only; rt_terrain_render_batch_packed)
    uint32_t packed;
};

// Where pixel (px, py) of lane `lane` of unit u goes in its frame's RGBA8 output: the framebuffer row-major,
// or (UnitMap::packed) the unit's tile u >> 4 of the shard at 1024 pixels each, row (sub >> 2) * 8 +
// (lane >> 3) and column (sub & 3) * 8 + (lane & 7) of the tile (sub = u & 15; unit_pixel's mapping)
__device__ __forceinline__ uint32_t out_index(const UnitMap& m, uint32_t u, uint32_t lane, uint32_t px, uint32_t py,
                                              uint32_t W)
{
    if (m.packed)
        return (u >> 4) * 1024u + ((u & 15u) >> 2) * 256u + (lane >> 3) * 32u + (u & 3u) * 8u + (lane & 7u);
    return py * W + px;
}
// the same from a frame's sample id tl = u * 64 + lane (one sample per pixel): its bits 0-2 (lane & 7) stay,
// 6-7 (u & 3) -> 3-4, 3-5 (lane >> 3) -> 5-7, 8-9 -> 8-9 (sub >> 2), 10.. (the shard's tile) stay
__device__ __forceinline__ uint32_t packed_index(uint32_t tl)
{
    return (tl & ~0xf8u) | ((tl >> 3) & 0x18u) | ((tl << 2) & 0xe0u);
}

__device__ __forceinline__ bool unit_pixel(const UnitMap& m, uint32_t f, uint32_t u, uint32_t lane, uint32_t W,
                                           uint32_t H, uint32_t* px, uint32_t* py)
{
    const uint32_t first = m.frame_rot ? (m.tile_first + f) % m.tile_stride : m.tile_first;
    // 8x8 units (16x4 and 32x2 measured 1% and 3% slower at C3: rows near the horizon
    // diverge more along x than an 8x8 block does along y)
    uint32_t T = (u >> 4) * m.tile_stride + first, sub = u & 15u;
    uint32_t gx = (T % m.tiles32_x) * 32u + (sub & 3u) * 8u + (lane & 7u);
    uint32_t gy = (T / m.tiles32_x) * 32u + (sub >> 2) * 8u + (lane >> 3);
    *px = gx + m.off_x;
    *py = gy + m.off_y;
    return gx < m.ext_x && gy < m.ext_y && *px < W && *py < H;
}

__device__ __forceinline__ bool sample_pixel(const UnitMap& m, uint32_t f, uint32_t t, uint32_t aa, uint32_t W,
                                             uint32_t H, uint32_t* px, uint32_t* py, uint32_t* a)
{
    uint32_t pix = t / aa;
    *a = t - pix * aa;
    return unit_pixel(m, f, pix >> 6, pix & 63u, W, H, px, py);
}

__device__ __forceinline__ uint32_t wave_fetch(uint32_t* counter, uint32_t lane, uint32_t n = 1u)
{
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(counter, n);
    return __builtin_amdgcn_readfirstlane(u);
}

// Set bits of `mask` below this lane (its rank among the lanes of `mask`): v_mbcnt_lo/hi, so no
// 64-bit lane mask stays live in VGPRs across the persistent kernels' loops.
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Per-sample RayResult of the primary march: 3 float4 (pd, fcolord, density).
// the unit index a wave takes first: wave-slot-major over the grid (row w holds order indices
// w * blocks .. w * blocks + blocks - 1, and wave slot w of each block takes the next one of its row in
// the order the blocks START), see k_trace
__device__ __forceinline__ uint32_t first_unit_index(uint32_t* __restrict__ counters, uint32_t lane)
{
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    return w * gridDim.x + wave_fetch(&counters[RT_CTR_FIRST + w], lane);
}

// A hit's record in its block's hit queue (the shading input; misses store none): the primary
// RayResult and the sample id t.  With fog live (greenrocks): 3 float4 (pd + dist, fcolord,
// (density, steps, -, t)).  Without, fcolord is 0 and is not stored, and the hit position is not
// either: the shading re-derives it from the pixel's ray and the last sample's distance
// (march_result's fma), so the record is one float4 (sd, dist, density, t).  The queue is a stack
// per block (hits shade in any order), written densely at its top: the few KiB near the top are
// rewritten over and over and stay in the XCD's L2 (write-back), instead of a sample-indexed array
// whose sparsely written lines (the hit lanes of each unit) each cost a write-back and a re-fetch,
// or a ring whose whole capacity cycles through the L2 (scripts/ubench_l2wb.hip: 16 KiB rewritten
// per block stays in L2, 64 KiB per block is written back on every pass).
template <int L>
struct HitRec {
    // float4 per record (RT_DIAG_HITPAD: a fog-free record padded to 2 with a zero float4, to see what the
    // hit stack's bytes cost in HBM writes)
    static constexpr uint32_t N = FogLive<L>::value ? 3u : (RT_DIAG_HITPAD ? 2u : 1u);
};
template <int L>
__device__ __forceinline__ void hit_store(float4* __restrict__ r, uint32_t t, const RayResult& rr)
{
    if constexpr (FogLive<L>::value) {
        r[0] = make_float4(rr.pd.x, rr.pd.y, rr.pd.z, rr.pd.w);
        r[1] = make_float4(rr.fc.x, rr.fc.y, rr.fc.z, rr.fc.w);
        r[2] = make_float4(rr.density, rr.steps, 0.0f, __uint_as_float(t));
    } else {
        r[0] = make_float4(rr.sd, rr.pd.w, rr.density, __uint_as_float(t));
        if constexpr (RT_DIAG_HITPAD) r[1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

// Longest-first tile order for k_trace.  A frame's critical path is its few
// grazing units (hundreds of march steps near the horizon); in screen order they
// start half-way through the queue and finish long after the rest.  The prepass
// cells already say where they are: a tile whose cells' depth bracket
// log2(far/near) is wide starts its rays far in front of the surface they hit (or
// graze).  One workgroup buckets the shard's 32x32 tiles by that key (64 buckets,
// descending); the order only decides which wave takes a unit when, never what
// it computes.
// The order spans the whole batch: entry i = (frame << 24) | tile, the batch's tiles of all frames
// longest-first.  Frame-major order (each frame longest-first in turn) left the last frame's
// grazing units to start in the last twelfth of the launch: at an 8-way shard, where a frame's
// share of the launch is shorter than one such unit, they set the batch time (k_trace 5.7 ms for
// 4.0 ms of work).  One workgroup; frame by frame it loads the frame's cell keys and buckets its
// tiles (the bucket bytes stay in LDS for the scatter pass when they fit).
constexpr uint32_t kOrderLdsBuckets = 144u * 1024u;
constexpr uint32_t kOrderBatchUnitsPerWave = 4u;
__global__ void __launch_bounds__(1024) k_order(const FrameTable* __restrict__ ft, UnitMap m,
                                                uint32_t* __restrict__ order, uint32_t* __restrict__ counters,
                                                const uint32_t* wait_ctl, uint32_t wait_total, uint32_t* zero_ctl,
                                                uint32_t* host_flag, uint32_t* gate, uint32_t* claims)
{
    __shared__ float s_key[RT_CAMERA_RES * RT_CAMERA_RES];
    __shared__ uint32_t s_hist[64];
    __shared__ uint8_t s_b[kOrderLdsBuckets];
    // k_trace's work counters start at zero (k_trace follows on the stream), and so do the counters
    // of the next batch's prepass that k_trace runs (FusedPrepass)
    if (blockIdx.x == 0 && threadIdx.x < RT_CTR_BYTES / 4) counters[threadIdx.x] = 0u;
    if (zero_ctl && blockIdx.x == 0 && threadIdx.x < 2) zero_ctl[threadIdx.x] = 0u;
    if (gate) { // the gated launch: this workgroup's frames' task masks, ray counters and tile claims start at zero
        const uint32_t g0 = m.order_batch ? 0u : blockIdx.x, g1 = m.order_batch ? m.n_frames : blockIdx.x + 1u;
        for (uint32_t i = g0 * RT_GATE_WORDS + threadIdx.x; i < g1 * RT_GATE_WORDS; i += blockDim.x) gate[i] = 0u;
        const uint32_t nt = m.n_units >> 4; // order entries per frame (this workgroup writes entries [g0 nt, g1 nt))
        for (uint32_t i = g0 * nt + threadIdx.x; i < g1 * nt; i += blockDim.x) claims[i] = 0u;
    }
    if (wait_ctl) {
        // this batch's prepass runs inside the previous batch's k_trace (FusedPrepass): wait until its
        // rays are in (each task stored its line with sc1, waited, then added to ctl[1]).  The tasks are
        // taken before that kernel's waves may leave, and they are finished by resident waves, so the
        // wait ends; the bound (0.5 s of the 100 MHz clock) turns a broken protocol into a flagged error
        // (rt_device_check) instead of a hang.
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(wait_ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < wait_total) {
                __builtin_amdgcn_s_sleep(8);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {
                    // fail safe: the frames of this batch may trace from incomplete CameraResults.  The
                    // device's sticky flag (rt_device_check) and the GPU's host-mapped word, which every
                    // later C-ABI call on this GPU reads (RT_ERR_STATE until rt_device_check clears it)
                    atomicOr(counters + RT_CTR_BYTES / 4, RT_FLAG_PREPASS_TIMEOUT);
                    if (host_flag) __hip_atomic_store(host_flag, RT_FLAG_PREPASS_TIMEOUT, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
        __syncthreads(); // every load of the CameraResults after the poll
    }
    // setTargetDepths (Terrain.cpp:398-439) of this workgroup's frames first: the device path's
    // CellDistance comes from the prepass's CameraResults (one launch fewer than a separate kernel)
    if (m.cells_from_cam) {
        const uint32_t c0 = m.order_batch ? 0u : blockIdx.x, c1 = m.order_batch ? m.n_frames : blockIdx.x + 1u;
        for (uint32_t f = c0; f < c1; ++f) cell_depths_frame(ft->cam[f], ft->cells[f], s_key);
        __syncthreads(); // the cells are stored before load_keys reads them (same workgroup)
    }
    if (threadIdx.x < 64) s_hist[threadIdx.x] = 0;
    const uint32_t n_tiles = m.n_units >> 4;
    const bool cached = n_tiles * m.n_frames <= kOrderLdsBuckets;
    uint32_t f = 0;
    auto load_keys = [&]() {
        __syncthreads(); // the previous frame's keys are no longer read
        const float2* cells = ft->cells[f];
        for (int i = threadIdx.x; i < RT_CAMERA_RES * RT_CAMERA_RES; i += blockDim.x) {
            float2 cd = cells[i];
            s_key[i] = __log2f(cd.y / cd.x);
        }
        __syncthreads();
    };
    auto bucket = [&](uint32_t tile) -> uint32_t {
        const RtConsts* k = ft->k[f];
        const uint32_t W = (uint32_t)k->width, H = (uint32_t)k->height;
        float key = 0.0f;
        // corner pixels of the tile: unit 0 lane 0, unit 3 lane 7, unit 12 lane 56, unit 15 lane 63
        for (uint32_t corner = 0; corner < 4; ++corner) {
            uint32_t px, py;
            uint32_t u = tile * 16u + (corner & 1u) * 3u + (corner >> 1) * 12u;
            uint32_t lane = (corner & 1u) * 7u + (corner >> 1) * 56u;
            if (!unit_pixel(m, f, u, lane, W, H, &px, &py)) {
                if (!unit_pixel(m, f, tile * 16u, 0u, W, H, &px, &py)) continue;
                px = px + (corner & 1u) * 31u < W ? px + (corner & 1u) * 31u : W - 1u;
                py = py + (corner >> 1) * 31u < H ? py + (corner >> 1) * 31u : H - 1u;
            }
            float spx = (float)px * k->rcp_w, spy = (float)py * k->rcp_h;
            uint32_t cell = (uint32_t)rtm::fma(rtm::floor(spy * 32.0f), 32.0f, rtm::floor(spx * 32.0f));
            key = fmaxf(key, s_key[cell]);
        }
        int b = (int)(key * 3.3f);
        return (uint32_t)(b < 0 ? 0 : (b > 63 ? 63 : b));
    };
    // frames [g0, g1) share one longest-first order: the whole batch (one workgroup), or frame
    // blockIdx.x alone (a workgroup per frame)
    {
        const uint32_t g0 = m.order_batch ? 0u : blockIdx.x, g1 = m.order_batch ? m.n_frames : blockIdx.x + 1u;
        for (f = g0; f < g1; ++f) {
            load_keys();
            for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) {
                const uint32_t b = bucket(t);
                if (cached) s_b[f * n_tiles + t] = (uint8_t)b;
                atomicAdd(&s_hist[b], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = g0 * n_tiles;
            for (int b = 63; b >= 0; --b) {
                uint32_t c = s_hist[b];
                s_hist[b] = run;
                run += c;
            }
        }
        for (f = g0; f < g1; ++f) {
            if (cached) __syncthreads();
            else load_keys();
            for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) {
                const uint32_t b = cached ? (uint32_t)s_b[f * n_tiles + t] : bucket(t);
                order[atomicAdd(&s_hist[b], 1u)] = (f << 24) | t;
            }
        }
    }
}

// Shading (tracescreen.hlsl:28-35, nomadplains/color.hlsl:8-72).  Per hit, the
// uniform work -- getNormal (3 densities), getColor up to the shadow ray (20-octave
// albedo FBM), the Rayleigh/Mie sky -- and the FIRST shadow-march step
// (color.hlsl:51).  About 70% of shadow rays end there (the surface faces away from
// the low sun, or the first sample is already inside the terrain) and those samples
// are finished on the spot; the rest become long shadow rays (2..~120 steps).
// A long ray's finishing inputs (albedo+specular rgb and brightness, fcolord with fog live,
// rayleigh rgb and skyAmount) go to a slot of its block's fin pool (fin_store), its march state to
// a 3-float4 record (long_pack).
constexpr uint32_t kShadowRec = 3;

// Lanes idle before a long-ray wave refills them: amortises the refill's divergent
// prologue against the idle lanes it leaves (knobs: rt_variants.h).
constexpr uint32_t kRefillIdle = RT_REFILL_IDLE;

// color.hlsl:53-71 after the shadow ray, then tracescreen.hlsl:33-35 fog and sky blends
__device__ __forceinline__ float4 shade_finish(const RtConsts* k, float4 cb, float4 fog, float4 ray,
                                               float shadow_density, float shadow_fog_w)
{
    float b = cb.w;
    if (shadow_density > 0.0f) b = b * 0.1f;
    else b = rtm::sat(b - shadow_fog_w);
    f3 col = rtm::mk(cb.x * fma(b, k->one_minus_shadow[0], k->shadow_color[0]),
                     cb.y * fma(b, k->one_minus_shadow[1], k->shadow_color[1]),
                     cb.z * fma(b, k->one_minus_shadow[2], k->shadow_color[2]));
    col = rtm::mk(rtm::lerp(col.x, fog.x, fog.w), rtm::lerp(col.y, fog.y, fog.w), rtm::lerp(col.z, fog.z, fog.w));
    col = rtm::mk(rtm::lerp(col.x, ray.x, ray.w), rtm::lerp(col.y, ray.y, ray.w), rtm::lerp(col.z, ray.z, ray.w));
    return make_float4(rtm::sat(col.x), rtm::sat(col.y), rtm::sat(col.z), 1.0f); // w = 1: a hit (AO applies)
}

// tracescreen.hlsl:22-27,36-38: the colour of a MISS sample (sky: Rayleigh/Mie + space noise, then the
// fog and sky-amount blends), saturated; w = 0 (no AO).  Computed where the primary march ends, so
// misses leave no RayResult behind.
__device__ __forceinline__ float4 miss_sample(const Ctx& c, float px, float py, float dist, f4 fog)
{
    f3 p, dir;
    get_pixel_ray(c, px, py, &p, &dir);
    f3 pdn = rtm::normalize(dir);
    float skyAmount = dist * 0.0005f;
    skyAmount = rtm::sat(skyAmount * skyAmount);
    SkyColor scat = get_rayleigh_mie(c, pdn);
    float space = get_space_color(c, pdn);
    f3 sky = rtm::mk((scat.mie.x + scat.rayleigh.x) + space, (scat.mie.y + scat.rayleigh.y) + space,
                     (scat.mie.z + scat.rayleigh.z) + space);
    f3 col = rtm::mk(rtm::lerp(sky.x, fog.x, fog.w), rtm::lerp(sky.y, fog.y, fog.w), rtm::lerp(sky.z, fog.z, fog.w));
    col = rtm::mk(rtm::lerp(col.x, sky.x, skyAmount), rtm::lerp(col.y, sky.y, skyAmount),
                  rtm::lerp(col.z, sky.z, skyAmount));
    return make_float4(rtm::sat(col.x), rtm::sat(col.y), rtm::sat(col.z), 0.0f);
}

// Loads of data another wave of this kernel (on this CU) wrote: bypass the CU's L1 (a line cached
// there earlier would be stale), served by the XCD's L2 the producer wrote through: `sc1` loads.
// Not nontemporal ones: an nt load marks the line evict-first, so the per-block LIFO hit stack and
// fin pool, whose few lines are rewritten over and over, were written back to HBM after every pop
// (profiles/r04/traffic_attribution.md).  ld_rec: record i (16-B units) of a block-local array (a
// uniform base, so a buffer load); ld_fresh: any address (the fin[t] fallback), waited at once.
typedef float v4f_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_rec(const float4* base, uint32_t i)
{
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(base), (short)0, 0x7fffffff, 0x00020000);
    const v4f_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16u), 0, 16 /* sc1 */);
    return make_float4(v.x, v.y, v.z, v.w);
}
// word i of a buffer with a uniform base (one offset register per lane): sc1 (another wave or workgroup
// wrote it in this launch) or plain
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* base, uint32_t i, bool sc1 = true)
{
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(base), (short)0, 0x7fffffff, 0x00020000);
    return sc1 ? __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4u), 0, 16 /* sc1 */)
               : __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4u), 0, 0);
}
__device__ __forceinline__ float4 ld_fresh(const float4* p)
{
    v4f_t v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return make_float4(v.x, v.y, v.z, v.w);
}

// A hit's finished sample.  With one sample per pixel only hits reach `samples` (misses are
// finished where their march ends) and every sample k_finish reads is a hit, so the record is the
// colour alone: 12 B (a float3 array over the same buffer); with AA, misses are stored too and w
// marks the hits (16 B).
// An opaque copy of a lane value: address arithmetic on it cannot be hoisted above this point, so a
// store's 64-bit address is formed where the store is (one VGPR live before it, not two).
__device__ __forceinline__ uint32_t late(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

__device__ __forceinline__ void sample_store(const RtConsts* k, float4* __restrict__ samples, uint32_t t, float4 v)
{
    t = late(t);
    if (k->aa_samples == 1) { // 3 floats at 12-byte stride (a float3 vector type would pad to 16)
        float* c = reinterpret_cast<float*>(samples) + 3u * t;
        c[0] = v.x;
        c[1] = v.y;
        c[2] = v.z;
    } else {
        samples[t] = v;
    }
}

// The AO extension's per-sample count of occluded AO rays: one byte per sample (at most 16 AO
// rays), four to a word, so a count's atomic add and k_finish's read touch a quarter of the lines
// a word per sample did (and the per-launch memset a quarter of the bytes).
__device__ __forceinline__ void ao_count(uint32_t* __restrict__ aocc, uint32_t t)
{
    atomicAdd(&aocc[t >> 2], 1u << ((t & 3u) * 8u));
}
// UnitMap::fitm with AO: a sample k_finish finishes carries kFinFlag in its byte (plain stores, k_trace)
constexpr uint32_t kFinFlag = 0x80u;
// UnitMap::fit with its one AO ray per hit: a hit whose shadow ray outlived its first step has two rays left,
// the long shadow S and the AO ray A, and whichever ends second stores the pixel (no k_finish).  Each ends
// with one device atomic OR on the sample's aocc byte -- kRaceS, or kRaceA | occluded -- and the one whose OR
// returns the other's bit is second.  S stores its colour (samples) and waits for it before its OR, so a
// second A reads it from the L2 with sc1; both rays of a hit are one block's (one CU, one L2).  The second
// clears the byte for the next launch.  k_finish's arithmetic (fit_pixel), so the same bits.
constexpr uint32_t kRaceS = 0x40u, kRaceA = 0x20u;
__device__ __forceinline__ uint32_t race_or(uint32_t* __restrict__ aocc, uint32_t t, uint32_t bits)
{
    const uint32_t sh = (t & 3u) * 8u;
    return (atomicOr(&aocc[late(t) >> 2], bits << sh) >> sh) & 0xffu;
}
// a hit's 12-byte colour record (sample_store, one sample per pixel), written by another wave: sc1, waited
__device__ __forceinline__ float4 ld_colour_fresh(const float4* samples, uint32_t t)
{
    typedef float v3f __attribute__((ext_vector_type(3)));
    const float* p = reinterpret_cast<const float*>(samples) + 3u * late(t);
    v3f v;
    asm volatile("global_load_dwordx3 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return make_float4(v.x, v.y, v.z, 1.0f);
}
__device__ __forceinline__ uint32_t ao_occluded(const uint32_t* __restrict__ aocc, uint32_t t)
{
    return (aocc[t >> 2] >> ((t & 3u) * 8u)) & 0x7fu;
}

struct ShadeHit {
    float4 cb, fog, ray;
    bool more; // the shadow ray is still marching after its first step
    f3 hp, n;  // hit position and normal (AO rays start here)
    float prec; // shadow-ray stepmod (AO rays reuse it)
    uint32_t px, py, a;
};


// frame f's context (f wave-uniform): its constant block (camera, sun) as cf.kf, its Eye and
// SunDirection in scalar registers; the launch's block c.k stays the source of every
// frame-invariant constant (scalar loads in the hot loops)
__device__ __forceinline__ Ctx frame_ctx(const Ctx& c, const FrameTable* __restrict__ ft, uint32_t f)
{
    Ctx cf = c;
    cf.kf = (KPtr)ft->k[f];
    cf.eye = rtm::mk(uniform_f(cf.kf->eye[0]), uniform_f(cf.kf->eye[1]), uniform_f(cf.kf->eye[2]));
    cf.sun = rtm::mk(uniform_f(cf.kf->sun[0]), uniform_f(cf.kf->sun[1]), uniform_f(cf.kf->sun[2]));
    return cf;
}

// the frame a global sample id belongs to
__device__ __forceinline__ uint32_t frame_of(const UnitMap& m, uint32_t t)
{
    return m.n_frames == 1u ? 0u : t / m.frame_samples;
}

// body(f) once per distinct frame f among the `valid` lanes, with exactly the lanes of
// frame f active (f wave-uniform).  A batch of hits or rays mixes frames only around the
// point where the frame-major unit order moves on to the next frame.
template <class Body>
__device__ __forceinline__ void per_frame(bool valid, uint32_t f_lane, Body body)
{
    uint64_t pend = __ballot(valid);
    while (pend) {
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)f_lane, (int)__builtin_ctzll(pend));
        const bool mine = valid && f_lane == f;
        pend &= ~__ballot(mine);
        if (mine) body(f);
    }
}

// Per-frame values a long ray needs on its own lane: the frame's Eye (the octave count of
// every density sample) and its normalised SunDirection (a shadow ray's direction).
struct FrameRays {
    float v[RT_MAX_BATCH][6];
    uint32_t* out8[RT_MAX_BATCH]; // the frames' RGBA8 framebuffers (UnitMap::fit: pixels stored by long rays)
};
__device__ __forceinline__ void frame_rays_load(FrameRays& s, const FrameTable* __restrict__ ft, uint32_t n_frames)
{
    if (threadIdx.x < n_frames) {
        const RtConsts* k = ft->k[threadIdx.x];
        const f3 sun = rtm::mk(k->sun[0], k->sun[1], k->sun[2]);
        const f3 sd = rtm::scale(sun, rtm::rcp(rtm::length(sun))); // tracing.hlsl:60-61
        s.v[threadIdx.x][0] = k->eye[0];
        s.v[threadIdx.x][1] = k->eye[1];
        s.v[threadIdx.x][2] = k->eye[2];
        s.v[threadIdx.x][3] = sd.x;
        s.v[threadIdx.x][4] = sd.y;
        s.v[threadIdx.x][5] = sd.z;
        s.out8[threadIdx.x] = ft->out8[threadIdx.x];
    }
}

// tracescreen.hlsl:22-35 (hit branch) through the first shadow-march step.  r0..r2: the hit's
// record (hit_store), t: the global sample id (buffers), tl: the sample within its frame (pixel).
template <int L>
__device__ __forceinline__ ShadeHit shade_hit(const Ctx& c, const UnitMap& m, float4 r0, float4 r1, float4 r2,
                                              uint32_t t, uint32_t tl, March<L, true>& st)
{
    const RtConsts* k = c.k;
    const uint32_t W = (uint32_t)k->width, H = (uint32_t)k->height, aa = (uint32_t)k->aa_samples;
    ShadeHit h;
    float4 pdw, dn;
    if constexpr (FogLive<L>::value) {
        pdw = r0;
        h.fog = r1;
        dn = r2;
    } else { // hit_store's fog-free layout; fcolord is 0
        (void)r1;
        (void)r2;
        pdw = make_float4(r0.x, 0.0f, 0.0f, r0.y); // (sd, -, -, dist) until the position is re-derived
        dn = make_float4(r0.z, 0.0f, 0.0f, 0.0f);
        h.fog = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    uint32_t px, py, a;
    sample_pixel(m, m.frame_rot ? (t - tl) / m.frame_samples : 0u, tl, aa, W, H, &px, &py, &a);
    h.px = px;
    h.py = py;
    h.a = a;
    f3 p, dir;
    get_pixel_ray(c, (float)px + k->aa_off[a][0], (float)py + k->aa_off[a][1], &p, &dir);
    if constexpr (!FogLive<L>::value) {
        // the primary march's last sample: march_begin's normalised direction, the step's fma
        const f3 md = rtm::scale(dir, rtm::rcp(rtm::length(dir)));
        const float sd = pdw.x;
        pdw = make_float4(fma(md.x, sd, p.x), fma(md.y, sd, p.y), fma(md.z, sd, p.z), pdw.w);
    }
    f3 hp = rtm::mk(pdw.x, pdw.y, pdw.z);
    h.hp = hp;
    // color.hlsl:51 traceRay(p, 0.4, 100, precision, SunDirection, fog, skiprefine): the first step,
    // taken before the normal and the colour (it needs neither; precision is the hit distance's),
    // so the colour's FBM and the step's density never hold their live values at the same time
    h.prec = shade_precision(pdw.w);
    march_begin(c, st, hp, 0.4f, h.prec, c.sun);
    if (march_live<L, true, true>(c, st, 100.0f, 0)) march_step<L, true, true>(c, st);
    h.more = march_live<L, true, true>(c, st, 100.0f, 0);
    f3 pdn = rtm::normalize(dir);
    float skyAmount = pdw.w * 0.0005f;
    skyAmount = rtm::sat(skyAmount * skyAmount);
    f4 pd = {pdw.x, pdw.y, pdw.z, dn.x}; // getNormal(float4(rr.pd.xyz, rr.density)) :31
    f3 n = get_normal<L>(c, pd);
    h.n = n;
    ShadePre sp = shade_pre<L>(c, hp, n, pdn, pdw.w);
    // color.hlsl:63-66: the specular term does not depend on the shadow
    float specular = rtm::sat(rtm::pow_nonneg(rtm::max(sp.spec_dot, 0.0f), 40.0f)) * sp.spec_k;
    SkyColor scat = get_rayleigh_mie(c, pdn);
    h.cb = make_float4(sp.col[0] + specular, sp.col[1] + specular, sp.col[2] + specular, sp.brightness);
    h.ray = make_float4(scat.rayleigh.x, scat.rayleigh.y, scat.rayleigh.z, skyAmount);
    return h;
}

// A long ray's `aux` word: an AO ray (sign bit set: kAuxAO, its occlusion counted in aocc for k_finish;
// or, with UnitMap::fit, kAuxAOCand | rgb24 = its hit's pixel if the ray is occluded, stored where the
// ray ends), or a shadow ray whose finishing inputs (fin_store) sit in its block's fin pool slot aux
// (< kFinSlots), or at fin[t] when the pool was empty (kAuxFinT).
constexpr uint32_t kAuxAO = 0xffffffffu, kAuxAOCand = 0x80000000u, kAuxFinT = 0x7ffffffeu;
__device__ __forceinline__ bool aux_ao(uint32_t aux) { return (int32_t)aux < 0; }
// With AO_SAMPLES >= 2 a hit's AO rays count their occlusion in a slot of the block's AO
// counters in LDS (kAuxAOSlot | slot, TraceQueues::ao_ctr): the ray that completes the count stores it,
// one plain byte store per hit; an idle lane holding kAuxSlotFree | slot returns the slot to the free list
// at its wave's next refill.  No free slot: the hit's rays count by device atomics (kAuxAO).
constexpr uint32_t kAuxAOSlot = 0xc0000000u, kAuxSlotFree = 0x60000000u;
__device__ __forceinline__ bool aux_ao_slot(uint32_t aux) { return (aux & 0xff000000u) == kAuxAOSlot; }
__device__ __forceinline__ bool aux_slot_free(uint32_t aux) { return (aux & 0xff000000u) == kAuxSlotFree; }

// Long-ray record (48 B): (p, dist), (step, aux, iters, t), (shadow fog | AO dir; a fog-free
// landscape's shadow leaves the third float4 unwritten).  A shadow ray's direction is SunDirection /
// length(SunDirection) (tracing.hlsl:60-61) for every ray; an AO ray carries its own (normalised)
// direction in the fog slot, since AO rays march without fog.  The density d is not kept: a stored
// ray is live, so its next step overwrites d before anything reads it; nor is lastStep, which only
// the refinement after a hit reads (tracing.hlsl:76-79) and SKIPREFINE rays break before it.
template <int L>
__device__ __forceinline__ void long_pack(const March<L, true>& st, uint32_t t, uint32_t aux, float4* r)
{
    r[0] = make_float4(st.p.x, st.p.y, st.p.z, st.dist);
    r[1] = make_float4(st.step, __uint_as_float(aux), __uint_as_float((uint32_t)st.iters), __uint_as_float(t));
    if (aux_ao(aux)) r[2] = make_float4(st.dir.x, st.dir.y, st.dir.z, 0.0f);
    else if constexpr (March<L, true>::FOG) r[2] = make_float4(st.f.x, st.f.y, st.f.z, st.f.w);
    // no fog: a shadow ray's f is +0 throughout (march_step), so r2 is neither written nor read
}

template <int L>
__device__ __forceinline__ uint32_t long_unpack(const float4 r0, const float4 r1, const float4 r2, f3 sun_dir,
                                                March<L, true>& st, uint32_t* aux)
{
    *aux = __float_as_uint(r1.y);
    st.p = rtm::mk(r0.x, r0.y, r0.z);
    st.dist = r0.w;
    st.step = r1.x;
    st.lastStep = 0.0f; // not read (SKIPREFINE)
    st.d = 0.0f;
    st.iters = (int)__float_as_uint(r1.z);
    if (aux_ao(*aux)) {
        st.dir = rtm::mk(r2.x, r2.y, r2.z);
        st.f = {0.0f, 0.0f, 0.0f, 0.0f};
        st.fog = false;
    } else {
        st.dir = sun_dir;
        // without fog the stored f is the +0 long_pack wrote: restating it as a constant lets the
        // compiler drop f from the long-ray loops' live state
        if constexpr (March<L, true>::FOG) st.f = {r2.x, r2.y, r2.z, r2.w};
        else st.f = {0.0f, 0.0f, 0.0f, 0.0f};
        st.fog = true;
    }
    return __float_as_uint(r1.w);
}

// AO ray k of a shaded hit, at its start (AO extension, rt_shader.h ao_dir)
template <int L>
__device__ __forceinline__ void ao_begin(const Ctx& c, const ShadeHit& h, uint32_t kk, March<L, true>& st)
{
    march_begin(c, st, h.hp, 0.4f, h.prec, ao_dir(h.n, h.px, h.py, h.a, kk), false);
}

// AO generator record (RT_AO_GEN, AO_SAMPLES >= 2): a shaded hit's AO rays as ONE ring record, expanded
// into its AO_SAMPLES rays at refill, one lane each (gen_begin), instead of AO_SAMPLES long-ray records
// pushed by the shading (64 hits x (1 + AO_SAMPLES) records per batch overflowed the LDS ring into the
// spill stack: C5's long-ray spills).  (hit position, stepmod), (n.x, aux, kGenMark, t),
// (n.y, n.z, px | py << 16, a): kGenMark in a long record's iters slot (a march has far fewer steps).
constexpr uint32_t kGenMark = 0xfffffff0u;
// generator records carry 2 .. 8 AO rays: a post-drain segment wave (8 rays) must be able to take one whole
__device__ __forceinline__ bool gen_on(const RtConsts* k)
{
    return RT_AO_GEN && k->ao_samples >= 2 && k->ao_samples <= 8 && 64u / (RT_SEG_LANES ? RT_SEG_LANES : 8u) >= 8u;
}
__device__ __forceinline__ bool rec_is_gen(float4 r1) { return __float_as_uint(r1.z) == kGenMark; }
__device__ __forceinline__ void gen_pack(const ShadeHit& h, uint32_t t, uint32_t aux, float4* r)
{
    r[0] = make_float4(h.hp.x, h.hp.y, h.hp.z, h.prec);
    r[1] = make_float4(h.n.x, __uint_as_float(aux), __uint_as_float(kGenMark), __uint_as_float(t));
    r[2] = make_float4(h.n.y, h.n.z, __uint_as_float(h.px | (h.py << 16)), __uint_as_float(h.a));
}
// AO ray kk of a generator record: ao_begin's march state (the state long_pack + long_unpack would
// carry: lastStep, d, f and sd are not read before the first step overwrites them)
template <int L>
__device__ __forceinline__ uint32_t gen_begin(const Ctx& c, float4 r0, float4 r1, float4 r2, uint32_t kk,
                                              March<L, true>& st, uint32_t* aux)
{
    *aux = __float_as_uint(r1.y);
    const uint32_t pp = __float_as_uint(r2.z);
    march_begin(c, st, rtm::mk(r0.x, r0.y, r0.z), 0.4f, r0.w,
                ao_dir(rtm::mk(r1.x, r2.x, r2.y), pp & 0xffffu, pp >> 16, __float_as_uint(r2.w), kk), false);
    return __float_as_uint(r1.w);
}

// The inputs a long shadow ray needs to finish its sample: (albedo + specular, brightness), fcolord
// (fog-live landscapes only; 0 otherwise) and (rayleigh, skyAmount): FinRec<L>::N float4 at f, a
// slot of the block's fin pool or fin[t].
template <int L>
struct FinRec {
    static constexpr uint32_t N = FogLive<L>::value ? 3u : 2u;
};
template <int L>
__device__ __forceinline__ void fin_store(float4* __restrict__ f, const ShadeHit& h)
{
    if constexpr (FogLive<L>::value) {
        f[0] = h.cb;
        f[1] = h.fog;
        f[2] = h.ray;
    } else {
        f[0] = h.cb;
        f[1] = h.ray;
    }
}

// UnitMap::fit: k_finish's arithmetic for a pixel of one sample, (0 + v * ao) * rcp(1) per channel, as
// UNORM8 (tracescreen.hlsl:67-75 with AA_SAMPLES 1), where the hit's last ray ends
__device__ __forceinline__ uint32_t fit_pixel(float4 v, float ao)
{
    const float ia = rtm::rcp(1.0f);
    return unorm8((0.0f + v.x * ao) * ia) | (unorm8((0.0f + v.y * ao) * ia) << 8) |
           (unorm8((0.0f + v.z * ao) * ia) << 16) | 0xff000000u;
}

// UnitMap::fit: store the final pixel of sample t (one sample per pixel) from a lane of any frame
__device__ __forceinline__ void fit_store(const RtConsts* k, const UnitMap& m, const FrameRays& fr, uint32_t t,
                                          uint32_t px8)
{
    const uint32_t f = frame_of(m, t), W = (uint32_t)k->width;
    const uint32_t tl = t - f * m.frame_samples;
    if (m.packed) { // out_index's packed position is a bit permutation of the sample id (one sample per pixel)
        gptr(fr.out8[f])[late(packed_index(tl))] = px8;
        return;
    }
    uint32_t px, py;
    unit_pixel(m, f, tl >> 6, t & 63u, W, (uint32_t)k->height, &px, &py);
    gptr(fr.out8[f])[(size_t)late(py) * W + px] = px8;
}

// A long ray left its loop: a shadow ray finishes its sample from its fin record (with fit and no AO,
// its pixel); an AO ray counts its occlusion for k_finish, or (fit) stores its hit's occluded pixel.
template <int L>
__device__ __forceinline__ void long_finish(const RtConsts* k, const UnitMap& m, const FrameRays& fr,
                                            const float4* __restrict__ fin, const float4* __restrict__ finp,
                                            float4* __restrict__ samples, uint32_t* __restrict__ aocc, uint32_t t,
                                            uint32_t aux, const March<L, true>& st)
{
    if (aux_ao(aux)) {
        if (RT_FIT_RACE && m.fit && aux == kAuxAO) { // fit: the AO ray of a hit with a long shadow races it (kRaceS)
            const uint32_t occ = st.d > 0.0f ? 1u : 0u;
            if (race_or(aocc, t, kRaceA | occ) & kRaceS) { // second: the shadow's colour is in
                if (!(RT_DIAG_SKIP & 2)) fit_store(k, m, fr, t, fit_pixel(ld_colour_fresh(samples, t), ao_factor(occ, 1)));
                reinterpret_cast<uint8_t*>(aocc)[late(t)] = 0u;
            }
            return;
        }
        if (st.d > 0.0f) {
            if (aux == kAuxAO) {
                // (RT_FIT_RACE 0) fit: the hit's one AO ray, after the shading's kFinFlag store (ordered by the push)
                if (!RT_FIT_RACE && m.fit) reinterpret_cast<uint8_t*>(aocc)[late(t)] = (uint8_t)(kFinFlag | 1u);
                // one AO ray per hit: its count has one writer, a plain byte store (no device atomic)
                else if (k->ao_samples == 1) reinterpret_cast<uint8_t*>(aocc)[late(t)] = 1u;
                else if (!(RT_DIAG_SKIP & 8)) ao_count(aocc, t);
            } else if (!(RT_DIAG_SKIP & 2)) {
                fit_store(k, m, fr, t, aux | 0xff000000u);
            }
        }
    } else {
        constexpr uint32_t FR = FinRec<L>::N;
        float4 f0, f1, fog = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (aux == kAuxFinT) { // the pool was empty: fin[t] (rare)
            const float4* f = fin + (size_t)FR * t;
            f0 = ld_fresh(f);
            if constexpr (FogLive<L>::value) fog = ld_fresh(f + 1);
            f1 = ld_fresh(f + FR - 1u);
        } else {
            f0 = ld_rec(finp, FR * aux);
            if constexpr (FogLive<L>::value) fog = ld_rec(finp, FR * aux + 1u);
            f1 = ld_rec(finp, FR * aux + FR - 1u);
        }
        const float4 v = shade_finish(k, f0, fog, f1, st.d, st.f.w);
        if (m.fit && k->ao_samples == 0) {
            if (!(RT_DIAG_SKIP & 2)) fit_store(k, m, fr, t, fit_pixel(v, 1.0f));
        } else if (RT_FIT_RACE && m.fit) { // its AO ray races it (kRaceA): the colour first, in L2 before the OR
            sample_store(k, samples, t, v);
            __builtin_amdgcn_s_waitcnt(0);
            const uint32_t ob = race_or(aocc, t, kRaceS);
            if (ob & kRaceA) { // second
                if (!(RT_DIAG_SKIP & 2)) fit_store(k, m, fr, t, fit_pixel(v, ao_factor(ob & 1u, 1)));
                reinterpret_cast<uint8_t*>(aocc)[late(t)] = 0u;
            }
        } else if (!(RT_DIAG_SKIP & 4)) {
            sample_store(k, samples, t, v);
        }
    }
}

// ===========================================================================
// Fused trace (default pipeline): the primary march, the hit shading and the long
// shadow rays in ONE persistent kernel, so the latency-bound shading phases run in
// the shadow of the VALU-bound primary march instead of after it.  Each CU keeps
// two block-local queues, fed and drained by its own 16 waves:
//   hits  : the records of primary hits (hit_store; pushed by a wave when it finishes a unit),
//           a stack per block in HBM (its top lines live in the XCD's L2);
//   longs : march state of shadow rays still live after their first step (pushed
//           by a wave when it finishes a shading batch), a ring in LDS.
// A wave's next job, in priority order: march long shadows (lane refill from the
// ring) when enough are queued; shade a batch of 64 queued hits; march the next
// primary unit from the global longest-first queue.  Queue operations hold a
// per-block LDS lock.  Every hand-off stays on one CU: the producer's global stores
// (hit records, fin) complete (s_waitcnt) before the push publishes them, and the consumer
// reads them with L1-bypassing loads from the XCD's L2.  A full long ring spills to the block's
// spill stack in HBM (the same block consumes it, so the hand-off stays on one CU like the LDS
// ring's own): a block never hands work to another kernel.
constexpr uint32_t kLongRing = 570; // fills the CU's LDS: 128 KiB tables + 4 KiB plane + the ring
// A block's fin pool: slots of FinRec<L>::N float4 in HBM for the finishing inputs of its long
// shadow rays, handed out from a LIFO free list in LDS, so the few hundred slots in use at a time
// are the same lines over and over and stay in the XCD's L2 (fin[t] instead: a sparse write and a
// re-fetch per long shadow).  An empty pool falls back to fin[t].
constexpr uint32_t kFinSlots = RT_FIN_SLOTS;
// AO counter slots per block (AO_SAMPLES >= 2; the LDS the ring and the tables leave)
constexpr uint32_t kAoSlots = RT_AO_SLOTS;
static_assert(kAoSlots % 2u == 0u && kAoSlots <= 256u && kAoSlots <= RT_AO_POOL_SLOTS,
              "AO slots: pairs of u16 counters, u8 indices, a colour each in the pool");
constexpr uint32_t kLongBatch = RT_LONG_BATCH; // queued long rays that make a wave switch to them
constexpr uint32_t kCompactLive = RT_COMPACT_LIVE; // live lanes below which a dry wave hands its rays back
// After the unit queue drains (nomadplains): a long-ray wave left with at most kSegHandBack live rays
// and an empty ring hands them back, and a wave that finds at most kSegQueue rays queued marches them
// as segments of kSegLanes lanes per ray (density_nomadplains_seg: the octaves spread over the
// segment), cutting the per-step latency that sets a launch's last few hundred microseconds.
constexpr uint32_t kSegLanes = RT_SEG_LANES, kSegHandBack = RT_SEG_HANDBACK, kSegQueue = RT_SEG_QUEUE;
// a prepass task (FusedPrepass / GatedPrepass: 8 rays) is marched by kPrepassSplit waves of 64 / RT_PREPASS_LPR rays
constexpr uint32_t kPrepassSplit = RT_FUSE_RAYS_PER_TASK / (64u / RT_PREPASS_LPR);
static_assert(kPrepassSplit >= 1u && RT_PREPASS_LPR >= RT_FUSE_RAYS_PER_TASK && RT_PREPASS_LPR <= 32, "prepass lanes per ray");
// A primary unit's last few rays (nomadplains): once at most kPrimarySeg rays of an 8x8 unit are
// still marching, they continue as segments of 64 / kPrimarySeg lanes per ray (primary_seg in
// k_trace) instead of keeping 64 lanes on a few rays' octave loops.  0: off.
constexpr uint32_t kPrimarySeg = RT_PRIMARY_SEG;
static_assert(kPrimarySeg == 0u || kPrimarySeg == 4u || kPrimarySeg == 8u || kPrimarySeg == 16u, "lanes per ray");
// The instrumented (STATS) kernels take the same segment tail (their counters cost registers there:
// they spill, the product does not), so their march and noise counts pass through the product's code.
constexpr bool kStatsPrimarySeg = RT_STATS_PRIMARY_SEG != 0;

// STATS kernels: a k_trace block's march-step and hit counters (LDS atomics; the block's last wave
// adds them to the frame statistics)
struct BlockStats {
    enum { PRIMARY = 0, SHADOW = 1, AO = 2, HITS = 3, NOISE = 4, NOISE_WAVES = 5 };
    unsigned long long v[6];
    uint32_t done, pad;
};

struct TraceQueues {
    uint32_t lock;
    uint32_t h_top, pad0; // the block's hit stack (HBM, hit_cap records): records [0, h_top) are queued
    uint32_t l_head, l_tail;
    uint32_t active;  // waves inside a primary unit or a shading batch (they may still push)
    uint32_t drained; // the global unit queue is exhausted
    uint32_t pad;
    uint32_t ls_top; // the block's long-ray spill stack (HBM, long_spill_cap records): [0, ls_top) queued
    uint32_t pad1;
    uint32_t f_top;            // free slots of the block's fin pool: fin_free[0, f_top)
    uint32_t overflow;         // RT_FLAG_*: a queue push past its bound was dropped (published at exit)
    // the gated launch (GatedPrepass), per block so that no wave holds them in registers: the block's tile
    // scan position, every frame's prepass seen done, the frames whose CellDistance is seen flagged
    uint32_t gscan, gate_all, gate_cells;
    uint32_t near_end; // a wave of this block took one of the last RT_NEAR_UNITS x (wave slots) units

    float4 longs[kLongRing * kShadowRec];
    uint16_t fin_free[kFinSlots];
    uint32_t ao_ctr[kAoSlots / 2]; // AO slot s: bits 16 (s & 1) + 0..4 rays finished, + 5..9 occluded
    uint8_t ao_free[kAoSlots];     // free AO slots: ao_free[0, ao_top)
    uint32_t ao_top;
};

// A fresh read of a ring field another wave may have written: a relaxed workgroup-scope atomic
// load.  (A volatile read kept its generic pointer -- the address-space inference leaves volatile
// accesses alone -- so every ring poll was a flat load with system-scope cache bits, waiting on
// the vector memory counter too, with the fields' 64-bit flat addresses held in VGPRs.)
template <class T>
__device__ __forceinline__ T vload(const T& x)
{
    return __hip_atomic_load(&x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void q_lock(uint32_t* lock, uint32_t lane)
{
    if (lane == 0) {
        while (atomicCAS(lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void q_unlock(uint32_t* lock, uint32_t lane)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) atomicExch(lock, 0u);
}

// Diagnostic builds only (rt_variants.h): the live-lane histogram and k_trace's per-wave timeline
// (RT_WT_FIELDS u64 per wave slot, scripts/wave_trace.py).
RT_DIAG_LIVE_HIST(__device__ unsigned long long g_live_hist[65];)
WT(__device__ unsigned long long g_wave_trace[RT_WT_MAX_WAVES * RT_WT_FIELDS];)

// k_trace's block: 16 waves (4 per SIMD, 128 VGPRs each) for the fog-free landscapes; the fog-live
// one (greenrocks: fog state in every march and record) and simple (its two-plane density) need
// more than 128 VGPRs and run 12 waves (3 per SIMD, up to 168 VGPRs) instead of spilling.
template <int L>
struct TraceThreads {
    static constexpr uint32_t value = 64u * ((L == RT_GREENROCKS || L == RT_SIMPLE) ? RT_TRACE_WAVES_WIDE : RT_TRACE_WAVES_FAST);
};
static_assert(RT_CTR_FIRST + RT_TRACE_WAVES_FAST <= RT_CTR_BYTES / 4 && RT_CTR_FIRST + RT_TRACE_WAVES_WIDE <= RT_CTR_BYTES / 4,
              "a first-unit counter per wave slot inside the zeroed work counters");

// GATED: the gated launch's instantiation (GatedPrepass, opt-in RT_DEVICE_GATED; nomadplains, no STATS).  The
// product instantiations (GATED false) carry none of its task, scan and claim paths.
template <int L, bool STATS, bool GATED = false>
__global__ void __launch_bounds__(TraceThreads<L>::value) k_trace(const RtConsts* __restrict__ k, const FrameTable* __restrict__ ft,
                                                const uint32_t* __restrict__ perm2d,
                                                const float4* __restrict__ grad,
                                                UnitMap m, const uint32_t* __restrict__ order,
                                                uint64_t* __restrict__ hitmask, float4* __restrict__ samples,
                                                float4* __restrict__ fin, float4* __restrict__ finpool,
                                                float4* __restrict__ cpool,
                                                float4* __restrict__ hitq,
                                                float4* __restrict__ spill_long, uint32_t hit_cap,
                                                uint32_t long_spill_cap,
                                                uint32_t* __restrict__ aocc, uint32_t* __restrict__ counters,
                                                RtStats* stats, uint32_t long_batch, uint32_t refill_idle,
                                                uint32_t compact_live, uint32_t long_ring_cap, uint32_t fin_slots,
                                                FusedPrepass np, GatedPrepass gp)
{
    // one LDS array (the noise image at address 0, then the frame table, the rings and the STATS
    // kernels' block counters)
    __shared__ __attribute__((aligned(16))) uint32_t
        lds[kNoiseLdsWords + (sizeof(FrameRays) + sizeof(TraceQueues) + sizeof(BlockStats)) / 4];
    FrameRays& s_fr = *reinterpret_cast<FrameRays*>(lds + kNoiseLdsWords);
    TraceQueues& q = *reinterpret_cast<TraceQueues*>(lds + kNoiseLdsWords + sizeof(FrameRays) / 4);
    BlockStats& s_st =
        *reinterpret_cast<BlockStats*>(lds + kNoiseLdsWords + (sizeof(FrameRays) + sizeof(TraceQueues)) / 4);
    frame_rays_load(s_fr, ft, m.n_frames);
    if (threadIdx.x == 0) {
        q.lock = 0;
        q.h_top = 0;
        q.l_head = q.l_tail = 0;
        q.active = 0;
        q.drained = 0;
        q.ls_top = 0;
        q.f_top = fin_slots;
        q.overflow = 0;
        q.gscan = q.gate_all = q.gate_cells = 0;
        q.near_end = 0;
        if constexpr (STATS) s_st = BlockStats{};
    }
    for (uint32_t i = threadIdx.x; i < fin_slots; i += blockDim.x) q.fin_free[i] = (uint16_t)i;
    for (uint32_t i = threadIdx.x; i < kAoSlots; i += blockDim.x) {
        q.ao_free[i] = (uint8_t)i;
        if (i < kAoSlots / 2u) q.ao_ctr[i] = 0u;
    }
    if (threadIdx.x == 0) q.ao_top = kAoSlots;
    load_noise_lds(lds, perm2d, grad, k);
    const uint32_t lane = __lane_id(); // v_mbcnt of constants: rematerialisable (threadIdx & 63 spilled)
    Ctx c = make_ctx(k, lds); // k: frame-invariant constants (per-frame ones: frame_ctx / s_fr)
    if constexpr (STATS) c.nz.lds_calls = (__attribute__((address_space(3))) unsigned long long*)&s_st.v[BlockStats::NOISE];
    const uint32_t W = (uint32_t)k->width, H = (uint32_t)k->height, aa = (uint32_t)k->aa_samples;
    const int max_steps = k->max_steps;
    const uint32_t n_total = (uint32_t)__builtin_amdgcn_readfirstlane(m.n_units * m.n_frames); // units (an SGPR)
    // this block's hit stack and long-ray spill stack (hit_cap / long_spill_cap records per block)
    constexpr uint32_t HR = HitRec<L>::N;
    float4* const hq = hitq + (size_t)blockIdx.x * hit_cap * HR;
    float4* const finp = finpool + (size_t)blockIdx.x * kFinSlots * FinRec<L>::N;
    float4* const cpl = cpool + (size_t)blockIdx.x * RT_AO_POOL_SLOTS; // fitm: the AO slots' hit colours
    float4* const lspill = spill_long + (size_t)blockIdx.x * long_spill_cap * kShadowRec;
    // queued work of the block: long rays in the LDS ring + spill stack, hits in the hit queue
    auto queued_long = [&]() { return vload(q.l_tail) - vload(q.l_head) + vload(q.ls_top); };
    auto queued_hits = [&]() { return vload(q.h_top); };
    // STATS: march steps and hits go to the block's LDS counters (no VGPRs held across the loops)
    auto stat = [&](int i, uint32_t v) {
        if constexpr (STATS) atomicAdd(&s_st.v[i], (unsigned long long)v);
    };

    // wt: begin, end, t_unit, t_shade, t_long, n_unit, n_shade, n_long, last unit end, t_idle, hw_id, xcc_id,
    // loop iterations, long rays finished (lane), max long-ray iters (lane), last iteration, max primary iters (lane)
    WT(unsigned long long wt[RT_WT_FIELDS] = {}; wt[10] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
       wt[11] = __builtin_amdgcn_s_getreg((31 << 11) | 20); uint32_t wl_rays = 0, wl_maxit = 0, wp_maxit = 0;)
    // push the lanes' long rays (shadow continuations or AO starts) to the ring, or to the
    // block's spill stack when the LDS ring is full (stored before the tail publishes them)
    auto push_recs = [&](bool want, auto pack) {
        const uint64_t lb = __ballot(want);
        if (!lb) return;
        const uint32_t n = (uint32_t)__popcll(lb), rank = lane_rank(lb);
        q_lock(&q.lock, lane);
        const uint32_t lh = vload(q.l_head), lt = vload(q.l_tail);
        if (lt - lh + n <= long_ring_cap) {
            if (want) pack(&q.longs[((lt + rank) % kLongRing) * kShadowRec]);
            if (lane == 0) q.l_tail = lt + n;
        } else {
            // the spill stack's bound (rt_spill_caps) holds by the work priorities; a push past it is
            // dropped and flagged (rt_device_check), never written over queued rays
            const uint32_t stl = (uint32_t)__builtin_amdgcn_readfirstlane(vload(q.ls_top));
            const bool fits = stl + n <= long_spill_cap;
            if (want && fits) pack(lspill + (size_t)(stl + rank) * kShadowRec);
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) {
                q.ls_top = fits ? stl + n : stl;
                q.overflow |= fits ? 0u : RT_FLAG_SPILL_OVERFLOW;
            }
        }
        q_unlock(&q.lock, lane);
    };
    auto push_long = [&](bool want, const March<L, true>& st, uint32_t t, uint32_t aux) {
        push_recs(want, [&](float4* r) { long_pack(st, t, aux, r); });
    };

#if RT_AO_GEN
    // Refill (the lock held; RT_AO_GEN with AO generator records): fill up to nslots ray slots from the
    // ring (from its head) and then the spill stack (from its top), whole records only, a generator
    // record filling AO_SAMPLES consecutive slots.  Candidate record i is lane i's; slot `slot` (want)
    // finds its record by a binary search over the records' first slots.  Sets the slot's ray; returns
    // the records taken from the ring (take) and the spill stack (more).
    auto refill_gen = [&](uint32_t head, uint32_t tail, uint32_t sl, uint32_t nslots, uint32_t slot, bool want,
                          March<L, true>& st, uint32_t& t, uint32_t& aux, bool& live, Ctx& cl, uint32_t* more_out) {
        const uint32_t A = (uint32_t)k->ao_samples, avail = tail - head;
        const uint32_t ci = late(lane);
        const bool cand = ci < avail + sl && ci < nslots; // (a record takes at least one slot)
        float4 r1 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (cand) r1 = ci < avail ? q.longs[((head + ci) % kLongRing) * kShadowRec + 1u]
                                  : ld_rec(lspill, (sl - 1u - (ci - avail)) * kShadowRec + 1u);
        const uint64_t gb = __ballot(cand && rec_is_gen(r1));
        const uint32_t gens_before = lane_rank(gb);
        const uint32_t start = ci + (A - 1u) * gens_before; // first slot of candidate ci
        const uint32_t cnt = ((gb >> ci) & 1ull) ? A : 1u;
        const uint64_t tb = __ballot(cand && start + cnt <= nslots);
        const uint32_t ncand = (uint32_t)__popcll(tb); // whole records that fit (a prefix of the candidates)
        const uint32_t take = ncand < avail ? ncand : avail;
        *more_out = ncand - take;
        uint32_t cc = 0;
        for (uint32_t step = 32u; step != 0u; step >>= 1u) {
            const uint32_t nx = cc + step;
            const uint32_t s2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((nx & 63u) << 2), (int)start);
            if (nx < ncand && s2 <= slot) cc = nx;
        }
        const uint32_t kk = slot - (uint32_t)__builtin_amdgcn_ds_bpermute((int)(cc << 2), (int)start);
        const uint32_t ncc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(cc << 2), (int)cnt); // slots of record cc
        if (want && cc < ncand && kk < ncc) { // (slots past the last whole record stay empty)
            float4 q0, q1, q2;
            if (cc < avail) {
                const float4* r = &q.longs[((head + cc) % kLongRing) * kShadowRec];
                q0 = r[0];
                q1 = r[1];
                q2 = r[2];
            } else {
                const uint32_t ri = (sl - 1u - (cc - avail)) * kShadowRec;
                q0 = ld_rec(lspill, ri);
                q1 = ld_rec(lspill, ri + 1u);
                q2 = ld_rec(lspill, ri + 2u);
            }
            if (rec_is_gen(q1)) t = gen_begin<L>(c, q0, q1, q2, kk, st, &aux);
            else t = long_unpack(q0, q1, q2, rtm::mk(0.0f, 0.0f, 0.0f), st, &aux);
            const float* fr = s_fr.v[frame_of(m, t)];
            cl.eye = rtm::mk(fr[0], fr[1], fr[2]);
            if (!aux_ao(aux)) st.dir = rtm::mk(fr[3], fr[4], fr[5]);
            live = true;
        }
        return take;
    };
#endif

    // the fin pool slots of finished shadow rays (idle lanes whose aux is a slot) go back to the free
    // list; the lock is held
    auto free_fin_locked = [&](bool live, uint32_t& aux) {
        const bool pend = !live && aux < kFinSlots;
        const uint64_t pb = __ballot(pend);
        if (pb) {
            const uint32_t top = vload(q.f_top);
            if (pend) {
                q.fin_free[top + lane_rank(pb)] = (uint16_t)aux;
                aux = kAuxAO;
            }
            if (lane == 0) q.f_top = top + (uint32_t)__popcll(pb);
        }
        if constexpr (kAoSlots > 0u) { // and the AO slots of completed counts
            const bool pa = !live && aux_slot_free(aux);
            const uint64_t ab = __ballot(pa);
            if (ab) {
                const uint32_t top = vload(q.ao_top);
                if (pa) {
                    q.ao_free[top + lane_rank(ab)] = (uint8_t)(aux & 255u);
                    aux = kAuxAO;
                }
                if (lane == 0) q.ao_top = top + (uint32_t)__popcll(ab);
            }
        }
    };
    // an AO ray with a counter slot left the march: count it; the ray that completes the hit's count stores
    // it (one byte that only this lane writes), clears the slot and keeps it to free (kAuxSlotFree)
    auto ao_slot_finish = [&](const March<L, true>& st, uint32_t t, uint32_t& aux) {
        const uint32_t sl = aux & 255u, sh = (sl & 1u) * 16u;
        const uint32_t occ1 = st.d > 0.0f ? 1u : 0u;
        const uint32_t old = atomicAdd(&q.ao_ctr[sl >> 1], (1u | (occ1 << 5)) << sh) >> sh;
        if ((old & 31u) + 1u == (uint32_t)k->ao_samples) {
            const uint32_t occ = ((old >> 5) & 31u) + occ1;
            if (m.fitm && !(old & (1u << 10))) { // no long shadow: the pixel, from the colour the shading left
                const float4 v = ld_rec(cpl, sl);
                const uint32_t at = __float_as_uint(v.w);
                if (!(RT_DIAG_SKIP & 2)) gptr(s_fr.out8[at >> 23])[at & 0x7fffffu] = fit_pixel(v, ao_factor(occ, k->ao_samples));
            } else if (occ != 0u) { // k_finish's count (fitm: after the shading's kFinFlag)
                reinterpret_cast<uint8_t*>(aocc)[late(t)] = (uint8_t)((m.fitm ? kFinFlag : 0u) | occ);
            }
            atomicAnd(&q.ao_ctr[sl >> 1], ~(0xffffu << sh));
            aux = kAuxSlotFree | sl;
        } else {
            aux = kAuxAO;
        }
    };

    // RT_SEG_DRAIN_ALL: after the drain every long ray goes to the segment waves (nomadplains only: the other
    // landscapes have no segment march, so their waves keep refilling)
    // (2: no refill after the drain, but a wave keeps the rays it holds: new rays go to segment waves only)
    constexpr bool kSegDrainAll = RT_SEG_DRAIN_ALL != 0 && L == RT_NOMADPLAINS && kSegLanes > 0u;
    constexpr bool kSegDrainHandAll = RT_SEG_DRAIN_ALL == 1 && kSegDrainAll;
    // ---- a batch of long rays, lane refill from the ring ----
    auto do_shadow = [&]() {
        March<L, true> st;
        st.d = 0.0f;
        st.iters = 0;
        bool live = false;
        uint32_t t = 0, aux = kAuxAO; // aux: the lane's ray (long_pack); on an idle lane, a fin slot to free
        Ctx cl = c; // cl.eye: the frame of the lane's ray (set on refill)
        cl.nz.phase = RT_PHASE_LONG;
        for (;;) {
            if (live && !march_live<L, true, true>(cl, st, aux_ao(aux) ? RT_AO_END : 100.0f, 0)) {
                WT(wl_rays++; wl_maxit = max(wl_maxit, (uint32_t)st.iters);)
                stat(aux_ao(aux) ? BlockStats::AO : BlockStats::SHADOW, (uint32_t)st.iters);
                if (kAoSlots > 0u && aux_ao_slot(aux)) ao_slot_finish(st, t, aux);
                else long_finish<L>(k, m, s_fr, fin, finp, samples, aocc, t, aux, st);
                live = false;
            }
            const uint64_t idle = __ballot(!live);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= refill_idle && queued_long() != 0u && !(kSegDrainAll && vload(q.drained) != 0u)) {
                q_lock(&q.lock, lane);
                free_fin_locked(live, aux);
                const uint32_t head = vload(q.l_head), tail = vload(q.l_tail);
#if RT_AO_GEN
                if (gen_on(k)) { // AO generator records: whole records into the idle lanes
                    const uint32_t sl = vload(q.ls_top);
                    uint32_t more;
                    const bool idl = (idle >> lane) & 1ull;
                    const uint32_t take = refill_gen(head, tail, sl, nidle, lane_rank(idle), idl, st, t, aux, live, cl, &more);
                    if (more) __builtin_amdgcn_s_waitcnt(0);
                    if (lane == 0) {
                        q.l_head = head + take;
                        q.ls_top = sl - more;
                    }
                    q_unlock(&q.lock, lane);
                    goto refilled;
                }
#endif
                {
                const uint32_t take = (tail - head) < nidle ? (tail - head) : nidle;
                // the block's spill stack tops up what the LDS ring cannot give (from its top)
                const uint32_t sl = vload(q.ls_top);
                const uint32_t more = sl < nidle - take ? sl : nidle - take;
                const uint32_t rank = lane_rank(idle);
                const bool mine = ((idle >> lane) & 1ull) && rank < take + more;
                auto take_ray = [&](float4 r0, float4 r1, float4 r2) {
                    t = long_unpack(r0, r1, r2, rtm::mk(0.0f, 0.0f, 0.0f), st, &aux);
                    const float* fr = s_fr.v[frame_of(m, t)];
                    cl.eye = rtm::mk(fr[0], fr[1], fr[2]);
                    if (!aux_ao(aux)) st.dir = rtm::mk(fr[3], fr[4], fr[5]);
                    live = true;
                };
                if (mine && rank < take) {
                    const float4* r = &q.longs[((head + rank) % kLongRing) * kShadowRec];
                    take_ray(r[0], r[1], r[2]);
                } else if (mine) {
                    const uint32_t ri = (sl - more + rank - take) * kShadowRec;
                    take_ray(ld_rec(lspill, ri), ld_rec(lspill, ri + 1u), ld_rec(lspill, ri + 2u));
                }
                if (more) __builtin_amdgcn_s_waitcnt(0); // the spill records are read before a push reuses them
                if (lane == 0) {
                    q.l_head = head + take;
                    q.ls_top = sl - more;
                }
                q_unlock(&q.lock, lane);
                }
            }
#if RT_AO_GEN
            refilled:
#endif
            const uint64_t lv = __ballot(live);
            // The ring ran dry and few lanes are left: rather than march them on
            // mostly empty lanes, hand them back to the ring (another wave will merge
            // them with new rays) and go do other work, while there still is some.
            const bool drained_now = vload(q.drained) != 0u;
            bool hand_back = lv != 0ull && (uint32_t)__popcll(lv) < compact_live && queued_long() == 0u && !drained_now;
            if constexpr (L == RT_NOMADPLAINS && kSegLanes > 0u) // after the drain: few rays go to segment waves
                hand_back = hand_back || (drained_now && lv != 0ull && (kSegDrainHandAll ||
                                          ((uint32_t)__popcll(lv) <= kSegHandBack && queued_long() == 0u)));
            if (lv == 0ull || hand_back) {
                if (__ballot(!live && (aux < kFinSlots || aux_slot_free(aux)))) {
                    q_lock(&q.lock, lane);
                    free_fin_locked(live, aux);
                    q_unlock(&q.lock, lane);
                }
                if (hand_back) push_long(live, st, t, aux);
                c.nz.calls = cl.nz.calls;
                return;
            }
            RT_DIAG_LONG_STEPS(if (live && (RT_COUNT_LONG_STEPS == 1 || (RT_COUNT_LONG_STEPS == 2) == (vload(q.drained) != 0u))) {
                cl.nz.phase = RT_COUNT_PHASE;
                count_noise(cl.nz);
                cl.nz.phase = RT_PHASE_LONG;
            })
            WT(wt[26]++;)
            if (live) march_step<L, true, true>(cl, st);
        }
    };

    // ---- after the drain: up to 64 / kSegLanes queued long rays, a segment of lanes per ray ----
    auto do_shadow_seg = [&]() {
        if constexpr (L == RT_NOMADPLAINS && kSegLanes > 0u) {
            constexpr uint32_t LPR = kSegLanes ? kSegLanes : 8u, RPW = 64u / LPR; // (8 only to compile the discarded branch when off)
            // late(): the segment's lane values (and the octave scales derived from them) are formed
            // here, not hoisted into the kernel's prologue where they would stay live throughout
            March<L, true> st;
            st.d = 0.0f;
            st.iters = 0;
            uint32_t t = 0, aux = kAuxAO;
            bool live = false;
            Ctx cl = c;
            cl.nz.phase = RT_PHASE_LONG;
            q_lock(&q.lock, lane);
            const uint32_t head = vload(q.l_head), tail = vload(q.l_tail);
            uint32_t take = (tail - head) < RPW ? (tail - head) : RPW;
            const uint32_t sl = vload(q.ls_top);
            uint32_t more = sl < RPW - take ? sl : RPW - take;
#if RT_AO_GEN
            if (gen_on(k)) { // AO generator records: whole records into the segments
                take = refill_gen(head, tail, sl, RPW, late(lane) / LPR, true, st, t, aux, live, cl, &more);
            } else
#endif
            if (const uint32_t grp = late(lane) / LPR; grp < take + more) { // every lane of the segment unpacks the same record
                float4 r0, r1, r2;
                if (grp < take) {
                    const float4* r = &q.longs[((head + grp) % kLongRing) * kShadowRec];
                    r0 = r[0];
                    r1 = r[1];
                    r2 = r[2];
                } else {
                    const uint32_t ri = (sl - more + grp - take) * kShadowRec;
                    r0 = ld_rec(lspill, ri);
                    r1 = ld_rec(lspill, ri + 1u);
                    r2 = ld_rec(lspill, ri + 2u);
                }
                t = long_unpack(r0, r1, r2, rtm::mk(0.0f, 0.0f, 0.0f), st, &aux);
                const float* fr = s_fr.v[frame_of(m, t)];
                cl.eye = rtm::mk(fr[0], fr[1], fr[2]);
                if (!aux_ao(aux)) st.dir = rtm::mk(fr[3], fr[4], fr[5]);
                live = true;
            }
            __builtin_amdgcn_s_waitcnt(0); // the spill records are read before their slots can be reused
            if (lane == 0) {
                q.l_head = head + take;
                q.ls_top = sl - more;
            }
            q_unlock(&q.lock, lane);
            const uint32_t lid = late(lane);
            const uint32_t j = lid & (LPR - 1u), base = lid & ~(LPR - 1u);
            const SegOctaves<LPR> g = seg_octaves<LPR>(c, j);
            for (;;) {
                if (live && !march_live<L, true, true>(cl, st, aux_ao(aux) ? RT_AO_END : 100.0f, 0)) {
                    if (j == 0u) { // every lane of the segment holds the same ray: its first lane finishes it
                        stat(aux_ao(aux) ? BlockStats::AO : BlockStats::SHADOW, (uint32_t)st.iters);
                        if (kAoSlots > 0u && aux_ao_slot(aux)) ao_slot_finish(st, t, aux);
                        else long_finish<L>(k, m, s_fr, fin, finp, samples, aocc, t, aux, st);
                    }
                    live = false;
                }
                if (!__ballot(live)) break;
                WT(wt[25]++;)
                if (live) {
                    auto dens = [&](f3 q0) {
                        uint32_t used;
                        const float d = density_nomadplains_seg<LPR>(cl, g, q0, j, base, &used);
                        if constexpr (STATS) { // the same noise count as density_nomadplains: octaves + steep noise
                            if (j == 0u) atomicAdd(&s_st.v[BlockStats::NOISE], (unsigned long long)(used + 1u));
                            if (lane == (uint32_t)__builtin_ctzll(__ballot(1)))
                                atomicAdd(&s_st.v[BlockStats::NOISE_WAVES], (unsigned long long)SegOctaves<LPR>::R);
                        }
                        return d;
                    };
                    march_step_with<L, true, true, decltype(dens), true>(cl, st, dens);
                }
            }
            // the segments' finished shadows return their fin pool slots (one lane per segment holds it)
            uint32_t fa = j == 0u ? aux : kAuxAO;
            if (__ballot(fa < kFinSlots || aux_slot_free(fa))) {
                q_lock(&q.lock, lane);
                free_fin_locked(false, fa);
                q_unlock(&q.lock, lane);
            }
        }
    };

    // ---- a primary unit's last <= kPrimarySeg live rays, a segment of 64 / kPrimarySeg lanes per ray ----
    // lb: the unit's live rays; st: every lane's march (the finished rays' final states stay in
    // their lanes).  The live rays' states move to their segments (ray r of lb to lanes r*LPR ..),
    // march there with the density's octaves spread over the segment (density_nomadplains_seg,
    // bit-identical to density_nomadplains; pow_nonneg_flat for the step factor, bit-identical to
    // pow_nonneg) and come back when every segment's ray has left the march.
    auto primary_seg = [&](const Ctx& cf, March<L, true>& st, bool lv, uint64_t lb, float spx, float spy) {
        if constexpr (L == RT_NOMADPLAINS && kPrimarySeg > 0u && (!STATS || kStatsPrimarySeg)) {
            constexpr uint32_t LPR = 64u / (kPrimarySeg ? kPrimarySeg : 8u);
            const uint32_t lid = late(lane);
            const uint32_t j = lid & (LPR - 1u), grp = lid / LPR, base = lid & ~(LPR - 1u);
            const uint32_t n = (uint32_t)__popcll(lb);
            // the lane of live ray grp (scalar loop over lb's <= kPrimarySeg set bits)
            uint32_t src = lid;
            uint64_t rem = lb;
            for (uint32_t r = 0; r < n; ++r) {
                const uint32_t sl = (uint32_t)__builtin_ctzll(rem);
                rem &= rem - 1ull;
                src = grp == r ? sl : src;
            }
            March<L, true> sg;
            sg.p = rtm::mk(__shfl(st.p.x, (int)src), __shfl(st.p.y, (int)src), __shfl(st.p.z, (int)src));
            sg.dir = rtm::mk(__shfl(st.dir.x, (int)src), __shfl(st.dir.y, (int)src), __shfl(st.dir.z, (int)src));
            sg.sd = __shfl(st.sd, (int)src);
            sg.dist = __shfl(st.dist, (int)src);
            sg.step = __shfl(st.step, (int)src);
            sg.lastStep = __shfl(st.lastStep, (int)src);
            sg.d = __shfl(st.d, (int)src);
            sg.iters = __shfl(st.iters, (int)src);
            sg.f = {0.0f, 0.0f, 0.0f, 0.0f}; // no fog in nomadplains (March::FOG is false)
            sg.fog = false;
            bool live = grp < n;
            const SegOctaves<LPR> g = seg_octaves<LPR>(cf, j);
            for (;;) {
                if (live && !march_live<L, true, false>(cf, sg, RT_CAMERA_FAR, max_steps)) live = false;
                if (!__ballot(live)) break;
                if (live) {
                    auto dens = [&](f3 q0) {
                        uint32_t used;
                        const float d = density_nomadplains_seg<LPR, true>(cf, g, q0, j, base, &used);
                        if constexpr (STATS) { // the same noise count as density_nomadplains: octaves + steep noise
                            if (j == 0u) atomicAdd(&s_st.v[BlockStats::NOISE], (unsigned long long)(used + 1u));
                            if (lane == (uint32_t)__builtin_ctzll(__ballot(1)))
                                atomicAdd(&s_st.v[BlockStats::NOISE_WAVES], (unsigned long long)SegOctaves<LPR>::R);
                        }
                        return d;
                    };
                    march_step_with<L, true, false, decltype(dens), true>(cf, sg, dens);
                }
            }
            // back to the rays' lanes (the march changes only these fields)
            const int back = (int)(lane_rank(lb) * LPR);
            const float sd = __shfl(sg.sd, back), dist = __shfl(sg.dist, back), step = __shfl(sg.step, back);
            const float last = __shfl(sg.lastStep, back), d = __shfl(sg.d, back);
            const int iters = __shfl(sg.iters, back);
            if (lv) {
                st.sd = sd;
                st.dist = dist;
                st.step = step;
                st.lastStep = last;
                st.d = d;
                st.iters = iters;
            }
            // every ray's origin and direction again, as march_begin formed them (the pixel ray,
            // normalised): they are not held across the segments' march
            f3 p, dir;
            get_pixel_ray(cf, spx, spy, &p, &dir);
            st.p = p;
            st.dir = rtm::scale(dir, rtm::rcp(rtm::length(dir)));
        }
    };

    // ---- a batch of up to 64 queued hits: shading + first shadow step ----
    auto do_shade = [&]() {
        q_lock(&q.lock, lane);
        const uint32_t top = vload(q.h_top);
        const uint32_t take = top < 64u ? top : 64u;
        float4 r0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), r1 = r0, r2 = r0;
        if (lane < take) {
            const uint32_t ri = (top - take + lane) * HR;
            r0 = ld_rec(hq, ri);
            if constexpr (HR == 3u) {
                r1 = ld_rec(hq, ri + 1u);
                r2 = ld_rec(hq, ri + 2u);
            }
        }
        __builtin_amdgcn_s_waitcnt(0); // read before the slots can be reused
        if (lane == 0) q.h_top = top - take;
        q_unlock(&q.lock, lane);
        const uint32_t t = __float_as_uint(HR == 3u ? r2.w : r0.w);
        March<L, true> st;
        bool more = false;
        uint32_t aux = kAuxAO;
        uint32_t ao_aux = kAuxAO; // the hit's AO ray: counted (kAuxAO) or carrying its occluded pixel (fit)
        const bool valid = lane < take;
        // AO_SAMPLES >= 2: a counter slot per hit (LDS), popped from the free list (none left: kAuxAO)
        if (kAoSlots > 0u && k->ao_samples >= 2) {
            const uint64_t vb = __ballot(valid);
            if (vb) {
                q_lock(&q.lock, lane);
                const uint32_t top = vload(q.ao_top), n = (uint32_t)__popcll(vb), rank = lane_rank(vb);
                const uint32_t got = n < top ? n : top;
                if (valid && rank < got) ao_aux = kAuxAOSlot | (uint32_t)q.ao_free[top - 1u - rank];
                if (lane == 0) q.ao_top = top - got;
                q_unlock(&q.lock, lane);
            }
        }
        ShadeHit h;
        per_frame(valid, valid ? frame_of(m, t) : 0u, [&](uint32_t f) {
            Ctx cf = frame_ctx(c, ft, f);
            cf.nz.phase = RT_PHASE_SHADE;
            h = shade_hit<L>(cf, m, r0, r1, r2, t, t - f * m.frame_samples, st);
            c.nz.calls = cf.nz.calls;
            more = h.more;
            if (!more) {
                const float4 v = shade_finish(k, h.cb, h.fog, h.ray, st.d, st.f.w);
                if (m.fit) {
                    // the pixel is final now (no AO), or its unoccluded value is (ao_factor(0, 1) = 1) and
                    // the AO ray carries the occluded one (ao_factor(1, 1)); no sample, no k_finish
                    if (!(RT_DIAG_SKIP & 2)) {
                        const uint32_t tl = t - f * m.frame_samples; // (one sample per pixel)
                        gptr(ft->out8[f])[m.packed ? late(packed_index(tl)) : late(h.py) * W + h.px] = fit_pixel(v, 1.0f);
                    }
                    if (k->ao_samples) ao_aux = kAuxAOCand | (fit_pixel(v, ao_factor(1u, 1)) & 0xffffffu);
                } else if (m.fitm && aux_ao_slot(ao_aux)) {
                    // the colour the AO ray completing the count finishes with, and where: frame << 23 | pixel
                    const uint32_t tl = t - f * m.frame_samples;
                    cpl[late(ao_aux & 255u)] =
                        make_float4(v.x, v.y, v.z, __uint_as_float((f << 23) | (m.packed ? packed_index(tl) : h.py * W + h.px)));
                } else if (!(RT_DIAG_SKIP & 4)) {
                    sample_store(k, samples, t, v);
                }
                stat(BlockStats::SHADOW, (uint32_t)st.iters);
            }
            // the long shadows' finishing inputs: a fin pool slot each (this frame's lanes are the
            // active ones: the first of them takes the lock), fin[t] when the pool is empty
            const uint64_t mb = __ballot(more);
            if (mb) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(__ballot(1));
                q_lock(&q.lock, lane - lead);
                const uint32_t top = vload(q.f_top), n = (uint32_t)__popcll(mb), rank = lane_rank(mb);
                const uint32_t got = n < top ? n : top;
                if (more) aux = rank < got ? (uint32_t)q.fin_free[top - 1u - rank] : kAuxFinT;
                if (lane == lead) q.f_top = top - got;
                q_unlock(&q.lock, lane - lead);
                if (more && !(RT_DIAG_SKIP & 16)) fin_store<L>(aux == kAuxFinT ? fin + (size_t)FinRec<L>::N * t : finp + (size_t)FinRec<L>::N * aux, h);
            }
        });
        // fitm: the hits whose pixel the AO counter's completion does not store (a long shadow, or no slot)
        // are k_finish's.  Plain stores, no atomics (a device-scope atomic costs a 32-B HBM write on gfx950,
        // L2 or not: scripts/ubench_atomic.hip): the sample's aocc byte becomes kFinFlag and the unit's
        // hitmask word, zero from the unit, becomes nonzero (every writer stores the same value); a long
        // shadow's slot marks it (bit 10: its completion stores the flagged count).  (fit: no k_finish; a long
        // shadow and its AO ray race in long_finish, kRaceS / kRaceA)
        const bool kfin = valid && ((!RT_FIT_RACE && m.fit && k->ao_samples && more) ||
                                    (m.fitm && (more || !aux_ao_slot(ao_aux)))); // (fit: the race, long_finish)
        if (kfin) {
            reinterpret_cast<uint8_t*>(aocc)[late(t)] = (uint8_t)kFinFlag;
            hitmask[t >> 6] = 1ull;
        }
        if (m.fitm && more && aux_ao_slot(ao_aux))
            atomicOr(&q.ao_ctr[(ao_aux & 255u) >> 1], (1u << 10) << ((ao_aux & 1u) * 16u));
        if (__ballot(more)) {
            __builtin_amdgcn_s_waitcnt(0); // the fin record is in L2 before the ray is visible
            push_long(more, st, t, aux);
        }
        // AO extension: the hit's AO rays start as long rays (fit: after its unoccluded pixel is stored,
        // which an occluded AO ray overwrites)
        if (m.fit || m.fitm) __builtin_amdgcn_s_waitcnt(0);
#if RT_AO_GEN
        if (gen_on(k)) { // one generator record per hit (expanded at refill)
            push_recs(valid, [&](float4* r) { gen_pack(h, t, ao_aux, r); });
        } else
#endif
        for (int kk = 0; kk < k->ao_samples; ++kk) {
            March<L, true> ao;
            if (valid) ao_begin(c, h, (uint32_t)kk, ao);
            push_long(valid, ao, t, ao_aux);
        }
    };

    // ---- a task of the NEXT batch's camerarays prepass (FusedPrepass; camerarays.hlsl:12-21) ----
    // 8 rays, one 8-lane segment each (ray r on lanes 8r..8r+7), marched as k_camerarays_group marches
    // them: the octaves of each density sample spread over the segment (density_nomadplains_seg,
    // bit-identical to density_nomadplains), that frame's camerarays constants, frame 0's launch
    // constants.  The 8 results form one 128-B line of CameraResults, stored whole by one sc1
    // instruction; after the store is acknowledged the task adds 8 to ctl[1] (the next k_order polls it).
    // own (the gated launch, GatedPrepass): a task of THIS batch's prepass (pft = ft); after its line it
    // flags the task (sc1 store) and adds 8 to its frame's ray counter; the frame's last task derives the
    // frame's CellDistance (the API's array: units compute their own cells' brackets, gate_ready)
    auto do_prepass = [&](const FrameTable* __restrict__ pft, uint32_t qt, bool own) {
        if constexpr (L == RT_NOMADPLAINS) {
            constexpr uint32_t LPR = RT_PREPASS_LPR, RPW = 64u / LPR; // lanes per ray, rays per wave
            constexpr uint32_t WPF = RT_CAMERA_RES * RT_CAMERA_RES / RPW;   // waves per frame
            const uint32_t f = qt / WPF;
            const uint32_t ray0 = (qt - f * WPF) * RPW;
            const uint32_t ray = ray0 + late(lane) / LPR;
            const uint32_t lid = late(lane);
            const uint32_t j = lid & (LPR - 1u), base = lid & ~(LPR - 1u);
            Ctx cp = c;
            cp.k = pft->kcam[0];
            cp.kf = (KPtr)pft->kcam[f];
            cp.eye = rtm::mk(uniform_f(cp.kf->eye[0]), uniform_f(cp.kf->eye[1]), uniform_f(cp.kf->eye[2]));
            cp.sun = rtm::mk(uniform_f(cp.kf->sun[0]), uniform_f(cp.kf->sun[1]), uniform_f(cp.kf->sun[2]));
            const uint32_t tx = ray % RT_CAMERA_RES, ty = ray / RT_CAMERA_RES;
            const float r31 = rtm::rcp(31.0f);
            const uint32_t pxs = (uint32_t)(((float)tx * r31) * cp.k->screen[0]);
            const uint32_t pys = (uint32_t)(((float)ty * r31) * cp.k->screen[1]);
            f3 p, dir;
            get_pixel_ray(cp, (float)pxs, (float)pys, &p, &dir);
            March<L, false> st;
            march_begin(cp, st, p, RT_CAMERA_NEAR, 2.0f, dir);
            const SegOctaves<LPR> g = seg_octaves<LPR>(cp, j);
            __builtin_amdgcn_s_setprio(RT_FUSE_PRIO); // latency-bound: the next batch's k_order waits for these rays
            while (march_live<L, false, true>(cp, st, RT_CAMERA_FAR, 0)) {
                auto dens = [&](f3 q0) {
                    uint32_t used;
                    return density_nomadplains_seg<LPR, false>(cp, g, q0, j, base, &used);
                };
                march_step_with<L, false, true, decltype(dens), true>(cp, st, dens);
            }
            __builtin_amdgcn_s_setprio(0);
            RayResult rr = march_result(st);
            if (rr.density < 0.0f) rr.pd.w = RT_CAMERA_FAR;
            if (j == 0u) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                const v4f v = {rr.pd.x, rr.pd.y, rr.pd.z, rr.pd.w};
                float4* dst = pft->cam[f] + ray;
                asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(dst), "v"(v) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
            if (!own) {
                if (lane == 0) __hip_atomic_fetch_add(np.ctl + 1, RPW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            typedef uint32_t __attribute__((address_space(1))) guint;
            guint* gf = (guint*)(gp.gate + f * RT_GATE_WORDS);
            uint32_t old = 0;
            if (lane == 0) {
                const uint32_t task = ray0 / RT_FUSE_RAYS_PER_TASK; // = ray row * 4 + ray column / 8
                // a task's last wave (its add to the task's counter returned the other waves' rays) flags it;
                // the earlier waves' lines were acknowledged before their adds
                bool whole = true;
                if constexpr (RPW < RT_FUSE_RAYS_PER_TASK)
                    whole = __hip_atomic_fetch_add(gf + RT_GATE_TASKS + task, RPW, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT) == RT_FUSE_RAYS_PER_TASK - RPW;
                if (whole) {
                    __hip_atomic_fetch_or(gf + (task >> 5), 1u << (task & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    old = __hip_atomic_fetch_add(gf + RT_GATE_CTR, (uint32_t)RT_FUSE_RAYS_PER_TASK, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if ((uint32_t)__builtin_amdgcn_readfirstlane(old) == RT_CAMERA_RES * RT_CAMERA_RES - RT_FUSE_RAYS_PER_TASK) {
                // the frame's last task (its add returned last): every ray is in.  Its CellDistance (8-B sc1
                // stores), waited, then the cells flag: later units read their brackets from it (gate_cells)
                if (gp.debug & 2u) { // (RT_DEVICE_DEBUG_GATE_STRESS: late, ~200 us of the 100 MHz clock)
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    while (__builtin_amdgcn_s_memrealtime() - t0 < 20000ull) __builtin_amdgcn_s_sleep(8);
                }
                const float4* cam = pft->cam[f];
                typedef unsigned long long __attribute__((address_space(1))) gu64;
                gu64* cells = (gu64*)pft->cells[f];
                for (uint32_t c = late(lane); c < RT_CAMERA_RES * RT_CAMERA_RES; c += 64u) {
                    const float2 b = cell_bracket([&](int x, int y) { return cam_depth_sc1(cam, x, y); },
                                                  (int)(c % RT_CAMERA_RES), (int)(c / RT_CAMERA_RES));
                    __hip_atomic_store(cells + c, (unsigned long long)__float_as_uint(b.x) |
                                                      ((unsigned long long)__float_as_uint(b.y) << 32),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
                if (lane == 0) __hip_atomic_store(gf + RT_GATE_CTR + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    };

    // ---- the gated launch (GatedPrepass): which unit next? ----
    // Units are claimed by tile, in k_order's longest-first order, from the tiles whose prepass rays are in:
    // the scan starts at the first tile with units left (counters[RT_CTR_SCAN]), reads 64 order entries
    // and their claim counters (claims[i]: units of order entry i taken, atomic adds) per step, and takes the
    // first unit of the first READY tile with units left.  A tile is ready when every task (8 rays of a row)
    // holding a CameraResults ray its cells' setTargetDepths reads has set its bit in the frame's task mask
    // (rows cy0 - 2 .. cy1 + 2, columns cx0 - 2 .. cx1 + 2 of its pixels' cells; the cell index grows with
    // the pixel, so the corner pixels bound them).  So units run in the longest-first order among the ready
    // ones, on any block (no unit waits in a block that took it).  sc1 loads throughout (the hand-off: a
    // task wave stored its line sc1 and waited before its mask bit).
    typedef const uint32_t __attribute__((address_space(1))) gcuint;
    auto ld_sc1 = [&](const uint32_t* p) {
        return __hip_atomic_load((gcuint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // tile order entry e (frame << 24 | shard tile) against its frame's task mask w0..w3
    auto tile_ready = [&](uint32_t e, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) -> bool {
        const uint32_t f = e >> 24, first = m.frame_rot ? (m.tile_first + f) % m.tile_stride : m.tile_first;
        const uint32_t T = (e & 0xffffffu) * m.tile_stride + first;
        const uint32_t gx = (T % m.tiles32_x) * 32u, gy = (T / m.tiles32_x) * 32u;
        const uint32_t px0 = gx + m.off_x, py0 = gy + m.off_y;
        if (gx >= m.ext_x || gy >= m.ext_y || px0 >= W || py0 >= H) return true; // no pixel: nothing to wait for
        const uint32_t xe = m.off_x + m.ext_x < W ? m.off_x + m.ext_x : W, ye = m.off_y + m.ext_y < H ? m.off_y + m.ext_y : H;
        const uint32_t px1 = px0 + 31u < xe ? px0 + 31u : xe - 1u, py1 = py0 + 31u < ye ? py0 + 31u : ye - 1u;
        auto cell_of = [&](uint32_t p, float r) { return (int)rtm::floor(((float)p * r) * 32.0f); };
        const int cx0 = cell_of(px0, k->rcp_w) - 2, cx1 = cell_of(px1, k->rcp_w) + 2;
        const int cy0 = cell_of(py0, k->rcp_h) - 2, cy1 = cell_of(py1, k->rcp_h) + 2;
        const int xlo = cx0 < 0 ? 0 : cx0, xhi = cx1 > RT_CAMERA_RES - 1 ? RT_CAMERA_RES - 1 : cx1;
        const int ylo = cy0 < 0 ? 0 : cy0, yhi = cy1 > RT_CAMERA_RES - 1 ? RT_CAMERA_RES - 1 : cy1;
        // the row's tasks tlo .. thi as a 4-bit group (task = row * 4 + x / 8: bits 4 (row % 8) .. of word row / 8)
        const uint32_t g = ((2u << (xhi / RT_FUSE_RAYS_PER_TASK)) - 1u) & ~((1u << (xlo / RT_FUSE_RAYS_PER_TASK)) - 1u);
        bool ok = true;
        for (int r = ylo; r <= yhi; ++r) {
            const uint32_t w = (r >> 3) == 0 ? w0 : (r >> 3) == 1 ? w1 : (r >> 3) == 2 ? w2 : w3;
            ok = ok && ((w >> ((r & 7) * 4)) & g) == g;
        }
        return ok;
    };
    // one scan step per call: 64 order entries from the block's scan position q.gscan (the global head when
    // it is behind it); 1: a unit (f, u) claimed; 0: none ready in this step (the next call looks further, and
    // starts over at the head once past the end); -1: no unit left anywhere
    auto gated_fetch = [&](uint32_t* pf, uint32_t* pu) -> int {
        const uint32_t nt = n_total >> 4; // order entries (tiles) of the batch
        bool gate_all = vload(q.gate_all) != 0u;
        if (!gate_all) { // every frame's prepass done? (its ray counter; lanes < n_frames)
            const uint32_t gw = lane < m.n_frames ? ld_u32(gp.gate, late(lane * RT_GATE_WORDS + RT_GATE_CTR))
                                                  : (uint32_t)(RT_CAMERA_RES * RT_CAMERA_RES);
            gate_all = __ballot(gw < (uint32_t)(RT_CAMERA_RES * RT_CAMERA_RES)) == 0ull;
            if (gate_all && lane == 0) q.gate_all = 1u;
        }
        if (gate_all) {
            // every prepass ray is in: the units in order by the queue counter (one atomic per unit, as without
            // the gate), each claimed by its bit in its tile's word (claims[i], 16 units); a unit the scan took
            // while the prepass ran (its bit set) is skipped
            for (int tries = 0; tries < 16; ++tries) {
                const uint32_t qi = wave_fetch(&counters[RT_CTR_PRIMARY], lane);
                if (qi >= n_total) return -1;
                uint32_t old = 0u;
                if (lane == 0) old = atomicOr(gp.claims + late(qi >> 4), 1u << (qi & 15u));
                if (!((__builtin_amdgcn_readfirstlane(old) >> (qi & 15u)) & 1u)) {
                    const uint32_t e = __builtin_amdgcn_readfirstlane(order[qi >> 4]);
                    *pf = e >> 24;
                    *pu = (e & 0xffffffu) * 16u + (qi & 15u);
                    return 1;
                }
            }
            return 0;
        }
        // while the prepass runs: a scan step of 64 tiles from the block's position (the head when behind it)
        const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane(ld_sc1(counters + RT_CTR_SCAN));
        if (h >= nt) return -1;
        const uint32_t gs = vload(q.gscan);
        const uint32_t base = gs > h && gs < nt ? gs : h;
        const uint32_t i = late(base + lane); // (late: no per-lane scan address hoisted into the prologue)
        uint32_t e = 0u, c = 0xffffu;
        if (i < nt) { // buffer loads: uniform bases, one offset register
            e = ld_u32(order, i, false);
            c = ld_u32(gp.claims, i);
        }
        const bool left = (c & 0xffffu) != 0xffffu;
        const uint64_t lb = __ballot(left);
        if (base == h) { // the head moves past the tiles with no unit left
            const uint32_t nh = lb ? base + (uint32_t)__builtin_ctzll(lb) : base + 64u;
            if (nh > h && lane == 0) atomicMax(counters + RT_CTR_SCAN, nh);
        }
        if (lane == 0) q.gscan = base + 64u; // the block's next step (a hint: racing waves may repeat one)
        bool ready = left;
        if (left) { // the tile's frame's task mask (sc1 loads of its four words)
            const uint32_t gw = (e >> 24) * RT_GATE_WORDS;
            ready = tile_ready(e, ld_u32(gp.gate, gw), ld_u32(gp.gate, gw + 1u), ld_u32(gp.gate, gw + 2u),
                               ld_u32(gp.gate, gw + 3u));
        }
        // the wave's first try is the ready tile at or after its own slot in the step, so the waves scanning one
        // step spread their claims over its ready tiles (within a step the order is longest-first only roughly
        // anyway); the slot from the wave's hardware id, read when needed (no register held for it)
        const uint64_t rdy = __ballot(ready);
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint64_t from = rdy & (~0ull << ((hw ^ (hw >> 6) ^ (hw >> 12)) & 63u));
        for (uint64_t rb = from ? from : rdy; rb; rb &= rb - 1ull) {
            const uint32_t l = (uint32_t)__builtin_ctzll(rb);
            uint32_t cl = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)l) | 0xffff0000u;
            while (cl != 0xffffffffu) { // the tile's first unclaimed unit, by its bit
                const uint32_t kk = (uint32_t)__builtin_ctz(~cl);
                uint32_t old = 0u;
                if (lane == 0) old = atomicOr(gp.claims + late(base + l), 1u << kk);
                old = (uint32_t)__builtin_amdgcn_readfirstlane(old);
                if (!((old >> kk) & 1u)) {
                    const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)l);
                    *pf = el >> 24;
                    *pu = (el & 0xffffffu) * 16u + kk;
                    if (lane == 0) q.gscan = base; // (this step again next time: its tile may have units left)
                    return 1;
                }
                cl |= old;
            }
        }
        return 0;
    };

    // ---- one 8x8 primary unit ----
    auto do_unit = [&](uint32_t f, uint32_t u) {
        bool cells_in = true; // (the gated launch: the frame's CellDistance is stored, flagged by its last task)
        if constexpr (GATED) {
            cells_in = (vload(q.gate_cells) >> f) & 1u;
            if (!cells_in && ld_sc1(gp.gate + f * RT_GATE_WORDS + RT_GATE_CTR + 1) != 0u) {
                cells_in = true;
                if (lane == 0) atomicOr(&q.gate_cells, 1u << f);
            }
        }
        Ctx cf = frame_ctx(c, ft, f);
        cf.nz.phase = RT_PHASE_PRIMARY;
        uint32_t px, py;
        const bool valid = unit_pixel(m, f, u, lane, W, H, &px, &py);
        const float pxf = (float)px, pyf = (float)py;
        float plane_x = 0.0f;
        if (valid) {
            float spx = pxf * k->rcp_w, spy = pyf * k->rcp_h;
            const uint32_t cell = (uint32_t)rtm::fma(rtm::floor(spy * 32.0f), 32.0f, rtm::floor(spx * 32.0f));
            if (GATED && !cells_in) {
                // the gated launch before the frame's CellDistance is flagged: the cell's setTargetDepths from
                // its CameraResults (gate_ready passed)
                const float4* cam = ft->cam[f];
                plane_x = cell_bracket([&](int x, int y) { return cam_depth_sc1(cam, x, y); }, (int)(cell % RT_CAMERA_RES),
                                       (int)(cell / RT_CAMERA_RES)).x;
            } else if (GATED) { // flagged in this launch: an sc1 load of the bracket the frame's last task stored
                typedef const float __attribute__((address_space(1))) gcfloat;
                plane_x = __hip_atomic_load((gcfloat*)(ft->cells[f] + cell), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                plane_x = gptr(ft->cells[f])[cell].x;
            }
        }
        for (uint32_t a = 0; a < aa; ++a) {
            const uint32_t t = f * m.frame_samples + (u * 64u + lane) * aa + a;
            March<L, true> st;
            st.d = 0.0f;
            bool lv = false;
            if (valid) {
                f3 p, dir;
                get_pixel_ray(cf, pxf + k->aa_off[a][0], pyf + k->aa_off[a][1], &p, &dir);
                march_begin(cf, st, p, plane_x, 1.0f, dir);
                lv = true;
            }
            __builtin_amdgcn_s_setprio(0);
            for (uint32_t it = 0;; ++it) {
                lv = lv && march_live<L, true, false>(cf, st, RT_CAMERA_FAR, max_steps);
                const uint64_t lb = __ballot(lv);
                if (lb == 0ull) break;
                RT_DIAG_LIVE_HIST(if (lane == (uint32_t)__builtin_ctzll(__ballot(1))) atomicAdd(&g_live_hist[__popcll(lb)], 1ull);)
                RT_DIAG_PRIMARY_STEPS(if (lv) {
                    cf.nz.phase = RT_COUNT_PHASE;
                    count_noise(cf.nz);
                    cf.nz.phase = RT_PHASE_PRIMARY;
                })
                if constexpr (L == RT_NOMADPLAINS && kPrimarySeg > 0u && (!STATS || kStatsPrimarySeg)) {
                    if ((uint32_t)__popcll(lb) <= kPrimarySeg) {
                        primary_seg(cf, st, lv, lb, pxf + k->aa_off[a][0], pyf + k->aa_off[a][1]);
                        break;
                    }
                }
#if RT_FBM_EXIT
                if constexpr (L == RT_NOMADPLAINS) {
                    if (lv) { // exact unless the march provably continues after this sample (RT_FBM_EXIT)
                        const float ns = st.step * k->step_factor;
                        const bool allow = st.dist + ns < RT_CAMERA_FAR && ns > k->min_limit &&
                                           !(max_steps > 0 && st.iters + 1 >= max_steps);
                        march_step_with<L, true, false>(cf, st, [&](f3 q) { return density_nomadplains_x(cf, q, allow); });
                    }
                } else
#endif
                if (lv) march_step<L, true, false>(cf, st);
                if (it == 96u) __builtin_amdgcn_s_setprio(1);
                else if (it == 224u) __builtin_amdgcn_s_setprio(2);
                else if (it == 384u) __builtin_amdgcn_s_setprio(3);
            }
            __builtin_amdgcn_s_setprio(0);
            const bool hit = valid && st.d > 0.0f;
            WT(if (valid) wp_maxit = max(wp_maxit, (uint32_t)st.iters);)
            RayResult rr;
            if (valid) {
                rr = march_result(st);
                stat(BlockStats::PRIMARY, (uint32_t)st.iters);
                if (!hit) {
                    const float4 v = miss_sample(cf, pxf + k->aa_off[a][0], pyf + k->aa_off[a][1], rr.pd.w, rr.fc);
                    if (aa == 1u) { // the pixel is final (k_finish's sum of one sample times rcp(1) is v itself)
                        const uint32_t px8 = unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | 0xff000000u;
                        if (m.packed) { // a packed shard buffer (no float output then)
                            if (!(RT_DIAG_SKIP & 1)) gptr(ft->out8[f])[packed_index(late(u * 64u + lane))] = px8;
                        } else {
                            const size_t o = (size_t)py * W + px;
                            if (!(RT_DIAG_SKIP & 1)) gptr(ft->out8[f])[o] = px8;
                            if (float4* o32 = ft->out32[f]) gstore(o32 + o, make_float4(v.x, v.y, v.z, 1.0f));
                        }
                    } else {
                        samples[t] = v;
                    }
                }
            }
            const uint64_t hb = __ballot(hit);
            // k_finish skips the misses; with fit it finishes only the hits the shading marks
            if (lane == 0) hitmask[(f * m.n_units + u) * aa + a] = (m.fit || m.fitm) ? 0ull : hb;
            if (hb) {
                // the hits' records go on the block's hit stack in rank order (dense lines), stored
                // before the top publishes them.  The stack does not overflow: a wave starts a unit
                // only while fewer than 64 hits are queued, so at most 63 + 16 waves x 64 x aa are
                // (rt_spill_caps' hit_cap); a push past it is dropped and flagged (rt_device_check).
                const uint32_t n = (uint32_t)__popcll(hb), rank = lane_rank(hb);
                if (hit) stat(BlockStats::HITS, 1u);
                q_lock(&q.lock, lane);
                const uint32_t top = vload(q.h_top);
                const bool fits = (uint32_t)__builtin_amdgcn_readfirstlane(top) + n <= hit_cap;
                if (hit && fits) hit_store<L>(hq + (size_t)(top + rank) * HR, t, rr);
                __builtin_amdgcn_s_waitcnt(0);
                if (lane == 0) {
                    if (fits) q.h_top = top + n;
                    else q.overflow |= RT_FLAG_HIT_OVERFLOW;
                }
                q_unlock(&q.lock, lane);
            }
        }
        c.nz.calls = cf.nz.calls;
    };

    // First unit of every wave is dealt wave-slot-major (wave slot w takes the next order index of row
    // w, w * blocks + j, j counted in the order the blocks start): the costliest units (k_order puts
    // them first) land one per SIMD instead of filling the first few CUs' SIMDs four deep, which sets
    // the frame time when there are barely more units than waves (an 8-way shard has ~4k units for 4k
    // waves); and a block that starts late (its CU still held by the other batch's k_trace tail, a
    // copy or a collective kernel) takes the cheapest units of each row, not a fixed set of the costliest.
    const uint32_t n_static = gridDim.x * (blockDim.x >> 6);
    const uint32_t first_qi = first_unit_index(counters, lane); // scalar, formed before the loop
    bool first_unit = true;
    bool np_open = np.tasks != 0u; // the next batch's prepass tasks may remain (FusedPrepass)
    bool gp_open = GATED && gp.tasks != 0u; // this batch's own prepass tasks may remain (GatedPrepass)
#if RT_GATE_STATIC
    uint32_t gp_next = first_qi;
#endif
    if constexpr (GATED) {
        if (gp.debug & 1u) { // RT_DEVICE_DEBUG_GATE_STRESS: this CU's L1 holds the frames' previous CellDistance
            float acc = 0.0f;
            for (uint32_t f = 0; f < m.n_frames; ++f)
                for (uint32_t i = lane; i < RT_CAMERA_RES * RT_CAMERA_RES; i += 64u) acc += ft->cells[f][i].x;
            asm volatile("" : : "v"(acc));
        }
    }
    WT(wt[0] = __builtin_amdgcn_s_memrealtime();)
    for (;;) {
        if constexpr (L == RT_NOMADPLAINS) {
            // the gated launch: this batch's own prepass before anything else (every unit waits for some
            // of its rays).  Tasks are taken by resident waves, so every taken task finishes.
            if (GATED && gp_open) {
#if RT_GATE_STATIC
                // static: the wave's tasks are its first-unit index and every n_static-th after it, so the
                // first ones go to wave 0 of each block in the order the blocks start, then wave 1, ...: one
                // task wave per SIMD (the standalone prepass's shape) instead of the first blocks' 16 waves
                const uint32_t qt = gp_next;
                gp_next += n_static;
#else
                const uint32_t qt = wave_fetch(&counters[RT_CTR_GATE], lane);
#endif
                if (qt < gp.tasks * kPrepassSplit) {
                    WT(const unsigned long long tp = __builtin_amdgcn_s_memrealtime();)
                    do_prepass(ft, qt, true);
                    WT(const unsigned long long tq = __builtin_amdgcn_s_memrealtime(); wt[21] += tq - tp; wt[22] = tq;)
                    continue;
                }
                gp_open = false;
            }
            // the next batch's prepass first (after a wave's static first unit): its k_order waits for it.
            // A wave leaves only after it found no task left, so every task is taken by a resident wave.
            if (np_open && !first_unit) {
                const uint32_t qt = wave_fetch(np.ctl, lane);
                if (qt < np.tasks * kPrepassSplit) {
                    do_prepass(np.ft, qt, false);
                    continue;
                }
                np_open = false;
            }
        }
        const uint32_t lp = queued_long();
        const uint32_t hp = queued_hits();
        const bool drained = vload(q.drained) != 0u;
        WT(const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(); wt[12]++;
           wt[15] = t0; if (drained && wt[18] == 0) { wt[18] = t0; wt[19] = lp; wt[20] = hp; })
        // near the queue's end the long rays are taken from a smaller backlog (RT_NEAR_LONG_BATCH), so the
        // block's backlog at the drain -- what its post-drain tail marches -- is small
        const uint32_t lb_now = (RT_NEAR_UNITS > 0 && vload(q.near_end) != 0u) ? (uint32_t)RT_NEAR_LONG_BATCH : long_batch;
        if (lp >= lb_now || (drained && lp > 0u)) {
            // (A/B) near the queue's end the long-ray waves issue ahead of the unit waves (RT_LONG_PRIO)
            if (RT_LONG_PRIO > 0 && lb_now != long_batch) __builtin_amdgcn_s_setprio(RT_LONG_PRIO);
            if constexpr (L == RT_NOMADPLAINS && kSegLanes > 0u) {
                if (drained && (kSegDrainAll || lp <= kSegQueue)) { // (drain-all: do_shadow refills nothing now)
                    do_shadow_seg();
                    WT(const unsigned long long ds = __builtin_amdgcn_s_memrealtime() - t0; wt[4] += ds; wt[7]++;
                       wt[23] += ds; wt[24]++;)
                    continue;
                }
            }
            do_shadow();
            WT(const unsigned long long dl = __builtin_amdgcn_s_memrealtime() - t0; wt[4] += dl; wt[7]++; wt[27] += dl;)
            continue;
        }
        if (hp >= 64u || (drained && hp > 0u)) {
            if (lane == 0) atomicAdd(&q.active, 1u);
            do_shade();
            if (lane == 0) atomicSub(&q.active, 1u);
            WT(wt[3] += __builtin_amdgcn_s_memrealtime() - t0; wt[6]++;)
            continue;
        }
        if (GATED ? !drained : (!drained || first_unit)) {
            // (without the gated launch a wave's static first unit is taken even after the queue drained)
            if (lane == 0) atomicAdd(&q.active, 1u);
            bool run = false;
            uint32_t f = 0, u = 0;
            if constexpr (GATED) { // the gated launch: the first unit of a ready tile, longest-first
                const int got = __builtin_amdgcn_readfirstlane(gated_fetch(&f, &u)); // (wave-uniform)
                run = got > 0;
                if (got < 0) {
                    if (lane == 0) q.drained = 1u;
                } else if (got == 0 && RT_GATE_SLEEP) { // no ready tile in this step: yield the SIMD to the prepass
                    __builtin_amdgcn_s_sleep(RT_GATE_SLEEP);
                } // (0: no ready tile in this step; the next call looks further)
            } else {
                const uint32_t qi = first_unit ? first_qi : n_static + wave_fetch(&counters[RT_CTR_PRIMARY], lane);
                first_unit = false;
                if (RT_NEAR_UNITS > 0 && qi + (uint32_t)RT_NEAR_UNITS * n_static >= n_total && lane == 0) q.near_end = 1u;
                if (qi < n_total) {
                    // the batch's tiles longest-first across its frames: entry (frame << 24) | tile
                    const uint32_t e = __builtin_amdgcn_readfirstlane(order[qi >> 4]);
                    f = e >> 24;
                    u = (e & 0xffffffu) * 16u + (qi & 15u);
                    run = true;
                } else if (lane == 0) {
                    q.drained = 1u;
                }
            }
            WT(if (!run) wt[9] += __builtin_amdgcn_s_memrealtime() - t0;) // (a fetch that found no unit: idle)
            if (run) { // (do_unit inlined once; f and u are wave-uniform: say so, for the divergence analysis)
                do_unit((uint32_t)__builtin_amdgcn_readfirstlane(f), (uint32_t)__builtin_amdgcn_readfirstlane(u));
                WT(const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); wt[2] += t1 - t0; wt[5]++; wt[8] = t1;)
            }
            if (lane == 0) atomicSub(&q.active, 1u);
            continue;
        }
        // drained and nothing queued: leave once no wave of the block can still push
        if (vload(q.active) == 0u && queued_long() == 0u && queued_hits() == 0u) break;
        __builtin_amdgcn_s_sleep(2);
        WT(wt[9] += __builtin_amdgcn_s_memrealtime() - t0;)
    }
    // a dropped push (never, by rt_spill_caps' bound) becomes the device's sticky flag (rt_device_check)
    if (lane == 0) {
        const uint32_t ov = vload(q.overflow);
        if (ov) atomicOr(counters + RT_CTR_BYTES / 4, ov);
    }
    WT(wt[1] = __builtin_amdgcn_s_memrealtime();
       for (int o = 32; o >= 1; o >>= 1) {
           wl_rays += __shfl_xor(wl_rays, o, 64);
           wl_maxit = max(wl_maxit, (uint32_t)__shfl_xor(wl_maxit, o, 64));
           wp_maxit = max(wp_maxit, (uint32_t)__shfl_xor(wp_maxit, o, 64));
       }
       wt[13] = wl_rays; wt[14] = wl_maxit; wt[16] = wp_maxit;
       const uint32_t slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
       if (lane < RT_WT_FIELDS && slot < RT_WT_MAX_WAVES) {
           unsigned long long v = 0;
           for (int f = 0; f < RT_WT_FIELDS; ++f) v = (lane == (uint32_t)f) ? wt[f] : v;
           g_wave_trace[slot * RT_WT_FIELDS + lane] = v;
       })
    if constexpr (STATS) {
        // the block's last wave out adds its counters to the frame statistics
        uint32_t done = 0;
        if (lane == 0) done = atomicAdd(&s_st.done, 1u);
        if (__builtin_amdgcn_readfirstlane(done) == (blockDim.x >> 6) - 1u && lane == 0) {
            atomicAdd(&stats->primary_steps, vload(s_st.v[BlockStats::PRIMARY]));
            atomicAdd(&stats->shadow_steps, vload(s_st.v[BlockStats::SHADOW]));
            atomicAdd(&stats->ao_steps, vload(s_st.v[BlockStats::AO]));
            atomicAdd(&stats->hits, vload(s_st.v[BlockStats::HITS]));
            atomicAdd(&stats->noise_calls, vload(s_st.v[BlockStats::NOISE]));
            atomicAdd(&stats->noise_waves, vload(s_st.v[BlockStats::NOISE_WAVES]));
        }
    }
}

// tracescreen.hlsl:67-75: the sum of the saturated samples in AA order, / AA, UNORM8 store.  Misses
// were coloured by k_trace (with one sample per pixel their pixels are already final there, and the
// unit's hit ballot says which lanes remain), hits by the shading / long-ray paths; w marks a hit,
// whose AO factor applies.  Persistent over 8x8 units, strided statically (wave w takes units w,
// w + n_waves, ...): the per-unit work is so short that a shared queue atomic would serialise it.
__global__ void __launch_bounds__(1024) k_finish(const RtConsts* __restrict__ k, const FrameTable* __restrict__ ft,
                                                 UnitMap m, const uint64_t* __restrict__ hitmask,
                                                 const float4* __restrict__ samples, uint32_t* __restrict__ aocc)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t W = (uint32_t)k->width, H = (uint32_t)k->height, aa = (uint32_t)k->aa_samples;
    const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t total = m.n_units * m.n_frames;
    for (uint32_t g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < total; g += n_waves) {
        const uint32_t f = __builtin_amdgcn_readfirstlane(g / m.n_units), u = g - f * m.n_units;
        auto* out8 = gptr(ft->out8[f]);
        float4* out32 = ft->out32[f];
        uint32_t px, py;
        if (!unit_pixel(m, f, u, lane, W, H, &px, &py)) continue;
        // one sample per pixel: k_trace wrote the misses' pixels, only the hits remain (fit: only the
        // units whose hitmask word is nonzero, and in them the samples flagged kFinFlag)
        if (m.fit || m.fitm) {
            if (hitmask[f * m.n_units + u] == 0ull) continue;
            const uint32_t t = f * m.frame_samples + u * 64u + lane;
            if (!((aocc[t >> 2] >> ((t & 3u) * 8u)) & kFinFlag)) continue; // (its word is cleared by a flagged lane or is 0)
        } else if (aa == 1u && !((hitmask[f * m.n_units + u] >> lane) & 1ull)) {
            continue;
        }
        float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f;
        for (uint32_t a = 0; a < aa; ++a) {
            const uint32_t t = f * m.frame_samples + (u * 64u + lane) * aa + a;
            float4 v;
            if (aa == 1u) { // sample_store's colour-only record of a hit
                const float* c = reinterpret_cast<const float*>(samples) + 3u * t;
                v = make_float4(c[0], c[1], c[2], 1.0f);
            } else {
                v = samples[t];
            }
            if (v.w > 0.0f && k->ao_samples > 0) { // AO extension: ao multiplies the saturated sample
                const float ao = ao_factor(ao_occluded(aocc, t), k->ao_samples);
                v = make_float4(v.x * ao, v.y * ao, v.z * ao, v.w);
            }

            c0 = c0 + v.x;
            c1 = c1 + v.y;
            c2 = c2 + v.z;
        }
        // the next launch on these buffers counts from zero: every counted sample is read above, and
        // the words are cleared once all of them are (a word's other samples belong to this lane or to
        // lanes of this unit, whose reads in the same loop iterations precede these stores), so no
        // per-launch memset of the counts precedes k_trace
        if (k->ao_samples > 0) {
            const uint32_t t0 = f * m.frame_samples + (u * 64u + lane) * aa;
            for (uint32_t w = t0 >> 2; w <= (t0 + aa - 1u) >> 2; ++w) aocc[w] = 0u;
        }
        float ia = rtm::rcp((float)aa);
        c0 = c0 * ia;
        c1 = c1 * ia;
        c2 = c2 * ia;
        size_t o = out_index(m, u, lane, px, py, (uint32_t)k->width);
        if (!(RT_DIAG_SKIP & 64)) out8[o] = unorm8(c0) | (unorm8(c1) << 8) | (unorm8(c2) << 16) | 0xff000000u;
        if (out32) gstore(out32 + o, make_float4(c0, c1, c2, 1.0f));
    }
}

// Tile-cyclic shard transport: one 256-thread block per 32x32 tile.
// RecorderWinAPI::write's pixel conversion (RecorderWinAPI.cpp:244-253): the R8G8B8A8
// backbuffer DWORD dwc becomes dwc & 0xFF00 | (dwc & 0xFF) << 16 | (dwc & 0xFF0000) >> 16,
// i.e. bytes (B, G, R, 0) = MFVideoFormat_RGB32, row y at dst + y * pitch.  One v_perm_b32
// per pixel, 4 pixels (16 B) per thread: a pure HBM stream (read W*H*4 B, write W*H*4 B).
__global__ void __launch_bounds__(256) k_bgrx(const uint32_t* __restrict__ fb, uint32_t* __restrict__ dst, int w,
                                              int h, int pitch_words)
{
    const int quads = (w + 3) >> 2;
    const int y = blockIdx.y;
    for (int qx = blockIdx.x * blockDim.x + threadIdx.x; qx < quads; qx += gridDim.x * blockDim.x) {
        const int x = qx << 2;
        const uint32_t* src = fb + (size_t)y * w + x;
        uint32_t* out = dst + (size_t)y * pitch_words + x;
        // perm selector: result bytes (B, G, R, 0) from (R, G, B, A) = bytes 2, 1, 0 and constant 0 (0x0c)
        constexpr uint32_t sel = 0x0c000102u;
        if (x + 4 <= w && ((w & 3) == 0) && ((pitch_words & 3) == 0)) {
            const uint4 v = *reinterpret_cast<const uint4*>(src);
            uint4 o;
            o.x = __builtin_amdgcn_perm(0u, v.x, sel);
            o.y = __builtin_amdgcn_perm(0u, v.y, sel);
            o.z = __builtin_amdgcn_perm(0u, v.z, sel);
            o.w = __builtin_amdgcn_perm(0u, v.w, sel);
            *reinterpret_cast<uint4*>(out) = o;
        } else {
            for (int i = 0; i < 4 && x + i < w; ++i) out[i] = __builtin_amdgcn_perm(0u, src[i], sel);
        }
    }
}

// Shard transport: job blockIdx.y copies tile blockIdx.x of its shard (tile blockIdx.x * count +
// shard, row-major) between its framebuffer and its packed buffer (1024 RGBA8 pixels per tile,
// row-major in the tile).  Thread t moves pixels 4 (t & 7) .. +3 of tile row t >> 3: one 16-byte
// access each way when the row segment lies inside the frame and both pointers allow it.  Pixels
// outside the frame are neither read nor written.  A batch's pack or unpack (rank 0 unpacks
// (N-1) x B shards per batch) is one launch instead of one per frame and rank: those small
// launches queue behind the other batch's persistent k_trace and each costs a dispatch.
__global__ void __launch_bounds__(256) k_shard_copy(ShardJobs jobs, int w, int h, int count, int pack)
{
    const int job = blockIdx.y;
    const int tiles_x = (w + 31) / 32, total = tiles_x * ((h + 31) / 32);
    const int tile = (int)blockIdx.x * count + jobs.shard[job];
    if (tile >= total) return; // a shard smaller than the grid (ragged shards)
    const int r = (int)threadIdx.x >> 3, c = ((int)threadIdx.x & 7) * 4;
    const int x = (tile % tiles_x) * 32 + c, y = (tile / tiles_x) * 32 + r;
    if (y >= h || x >= w) return;
    uint32_t* fb = jobs.fb[job] + (size_t)y * w + x;
    uint32_t* pk = jobs.packed[job] + (size_t)blockIdx.x * 1024 + r * 32 + c;
    if (x + 3 < w && (((uintptr_t)fb | (uintptr_t)pk) & 15u) == 0) {
        if (pack) *reinterpret_cast<uint4*>(pk) = *reinterpret_cast<const uint4*>(fb);
        else *reinterpret_cast<uint4*>(fb) = *reinterpret_cast<const uint4*>(pk);
    } else {
        for (int i = 0; i < 4 && x + i < w; ++i) {
            if (pack) pk[i] = fb[i];
            else fb[i] = pk[i];
        }
    }
}

// ft == nullptr: one frame (a.consts -> out); else frames 0..n-1 of the table (blockIdx.y).
template <int L>
void launch_camerarays_l(const RtLaunch& a, float4* out, const FrameTable* ft, uint32_t n)
{
    if constexpr (L == RT_NOMADPLAINS) {
        // one LPR-lane group per ray.  A block holds the noise tables (one block per CU), so
        // a batch packs more rays per block to keep every frame's prepass in one dispatch
        // round: 8 rays of 32 lanes (256 threads) up to 2 frames, 16 up to 4, and beyond 64
        // rays of 8 lanes (512 threads, <= 256 blocks for <= 16 frames; 4 lanes up to 24 frames).  Fewer lanes per ray
        // lengthen a step (3 noise rounds instead of 1) but keep a 12-frame prepass in one
        // round: 1.4 -> 0.7 ms per batch, +1.8% at C3 (32 rays of 32 lanes took two rounds).
        auto go = [&](auto bs_tag, auto lpr_tag) {
            constexpr int BS = decltype(bs_tag)::value, LPR = decltype(lpr_tag)::value;
            dim3 grid(RT_CAMERA_RES * RT_CAMERA_RES / (BS / LPR), n), block(BS);
            if (a.stats)
                hipLaunchKernelGGL((k_camerarays_group<true, BS, LPR>), grid, block, 0, a.stream, a.consts, a.perm2d,
                                   a.grad, out, a.stats, ft);
            else
                hipLaunchKernelGGL((k_camerarays_group<false, BS, LPR>), grid, block, 0, a.stream, a.consts,
                                   a.perm2d, a.grad, out, a.stats, ft);
        };
        using C512 = std::integral_constant<int, 512>;
        using L32 = std::integral_constant<int, 32>;
        if (n <= 2) go(std::integral_constant<int, RT_PREPASS_BS1>{}, std::integral_constant<int, RT_PREPASS_LPR1>{});
        else if (n <= 4) go(C512{}, L32{});
        else if (n <= 16) go(C512{}, std::integral_constant<int, 8>{}); // 64 rays of 16 lanes per 1024 threads: same
        else go(C512{}, std::integral_constant<int, 4>{}); // > 16 frames: 128 rays of 4 lanes, <= 192 blocks for 24
        return;
    }
    dim3 grid(RT_CAMERA_RES * RT_CAMERA_RES / 64, n), block(64);
    if (a.stats)
        hipLaunchKernelGGL((k_camerarays<L, true>), grid, block, 0, a.stream, a.consts, a.perm2d, a.grad, out, a.stats,
                           ft);
    else
        hipLaunchKernelGGL((k_camerarays<L, false>), grid, block, 0, a.stream, a.consts, a.perm2d, a.grad, out, a.stats,
                           ft);
}

template <int L>
void launch_split_l(const RtLaunch& a, uint32_t ox, uint32_t oy, uint32_t ex, uint32_t ey, uint32_t first,
                    uint32_t stride)
{
    UnitMap m;
    uint32_t tiles_x = (ex + 31) / 32, tiles_y = (ey + 31) / 32, total = tiles_x * tiles_y;
    // a batch rotates the shards over its frames (frame f traces shard (first + f) % stride), so
    // each rank's share of a batch mixes the tile classes of every shard.  Measured at C3 with
    // 12-frame batches (one-GPU shard simulation): the slowest of 4 ranks
    // went from 4-7% above the mean to 3.49x/4 scaling; N=2 and N=8 within noise.  n_units is
    // the largest shard's; the trailing units of a smaller shard map past the tile range and
    // unit_pixel rejects every lane of them.
    const uint32_t rot = a.n_frames > 1u && stride > 1u ? 1u : 0u;
    if (!rot && first >= total) return;
    m.off_x = ox;
    m.off_y = oy;
    m.ext_x = ex;
    m.ext_y = ey;
    m.tiles32_x = tiles_x;
    m.tile_first = first;
    m.tile_stride = stride;
    m.n_units = ((total - (rot ? 0u : first) + stride - 1) / stride) * 16u; // rot: the largest shard
    m.frame_rot = rot;
    m.n_frames = a.n_frames;
    m.frame_samples = m.n_units * 64u * (uint32_t)a.aa;
    uint32_t blocks = (uint32_t)(a.num_cus > 0 ? a.num_cus : 256);
    uint32_t need = (m.n_units * m.n_frames + 15u) / 16u;
    uint32_t pblocks = need < blocks ? need : blocks;
    m.order_batch = RT_ORDER_BATCH >= 0 ? (uint32_t)RT_ORDER_BATCH
                                        : (uint32_t)(m.n_frames > 1u && m.n_units < kOrderBatchUnitsPerWave * pblocks * 16u);
    // k_finish holds no LDS: up to 2 blocks per CU
    uint32_t fblocks = need < 2u * blocks ? need : 2u * blocks;
    dim3 blk(1024);
    m.cells_from_cam = (uint32_t)a.cells_from_cam;
    m.fit = (uint32_t)a.fit;
    m.fitm = kAoSlots > 0u ? (uint32_t)a.fitm : 0u;
    m.packed = (uint32_t)a.packed;
    // k_order: setTargetDepths (cells_from_cam), the work counters' reset, the tile order
    // (fuse_next.ctl is zeroed even with no tasks: RT_DEVICE_DEBUG_WITHHOLD_FUSE's timeout test)
    hipLaunchKernelGGL(k_order, dim3(m.order_batch ? 1u : m.n_frames), blk, 0, a.stream, a.frames, m, a.order, a.queue,
                       a.wait_ctl, a.wait_total, a.fuse_next.ctl, a.host_flag, a.gated.tasks ? a.gated.gate : nullptr,
                       a.gated.claims);
    if (a.after_order) (void)hipEventRecord(a.after_order, a.stream);
    if (a.after_order_fuse) (void)hipEventRecord(a.after_order_fuse, a.stream);
    // primary + shading + long rays; what does not fit a CU's LDS rings goes to its spill stacks
    auto primary = [&](auto stats_tag) {
        constexpr bool S = decltype(stats_tag)::value;
        const RtConsts* k0 = a.frames_host.k[0];
        // the gated launch's own instantiation (nomadplains without STATS: the runtime never gates others)
        constexpr bool kCanGate = L == RT_NOMADPLAINS && !S;
        auto* kern = (kCanGate && a.gated.tasks) ? k_trace<L, S, kCanGate> : k_trace<L, S, false>;
        hipLaunchKernelGGL(kern, dim3(pblocks), dim3(TraceThreads<L>::value), 0, a.stream, k0, a.frames,
                           a.perm2d, a.grad, m,
                           a.order, a.hitmask, a.samples, a.fin, a.finpool, a.cpool, a.hitq, a.spill_long, a.hit_cap,
                           a.long_spill_cap, a.aocc, a.queue, a.stats, kLongBatch, kRefillIdle, kCompactLive,
                           a.small_rings ? 64u : kLongRing, a.small_rings ? 8u : kFinSlots, a.fuse_next, a.gated);
        // fit: every hit pixel is final in k_trace (with its AO ray, by the race of long_finish)
        if (!(m.fit && (RT_FIT_RACE || a.ao_samples == 0)))
            hipLaunchKernelGGL(k_finish, dim3(fblocks), blk, 0, a.stream, k0, a.frames, m, a.hitmask, a.samples, a.aocc);
    };
    if (a.stats) primary(std::true_type{});
    else primary(std::false_type{});
}

} // namespace

void rt_launch_camerarays(const RtLaunch& a, float4* out)
{
    switch (a.landscape) {
    case RT_TESTING: launch_camerarays_l<RT_TESTING>(a, out, nullptr, 1u); break;
    case RT_SIMPLE: launch_camerarays_l<RT_SIMPLE>(a, out, nullptr, 1u); break;
    case RT_GREENROCKS: launch_camerarays_l<RT_GREENROCKS>(a, out, nullptr, 1u); break;
    default: launch_camerarays_l<RT_NOMADPLAINS>(a, out, nullptr, 1u); break;
    }
}

void rt_launch_camerarays_batch(const RtLaunch& a)
{
    switch (a.landscape) {
    case RT_TESTING: launch_camerarays_l<RT_TESTING>(a, nullptr, a.frames, a.n_frames); break;
    case RT_SIMPLE: launch_camerarays_l<RT_SIMPLE>(a, nullptr, a.frames, a.n_frames); break;
    case RT_GREENROCKS: launch_camerarays_l<RT_GREENROCKS>(a, nullptr, a.frames, a.n_frames); break;
    default: launch_camerarays_l<RT_NOMADPLAINS>(a, nullptr, a.frames, a.n_frames); break;
    }
}

void rt_launch_tracescreen(const RtLaunch& a, uint32_t ox, uint32_t oy, uint32_t ex, uint32_t ey, uint32_t first,
                           uint32_t stride)
{
    if (ex == 0 || ey == 0 || stride == 0) return;
    switch (a.landscape) {
    case RT_TESTING: launch_split_l<RT_TESTING>(a, ox, oy, ex, ey, first, stride); break;
    case RT_SIMPLE: launch_split_l<RT_SIMPLE>(a, ox, oy, ex, ey, first, stride); break;
    case RT_GREENROCKS: launch_split_l<RT_GREENROCKS>(a, ox, oy, ex, ey, first, stride); break;
    default: launch_split_l<RT_NOMADPLAINS>(a, ox, oy, ex, ey, first, stride); break;
    }
}

void rt_launch_bgrx(hipStream_t s, const uint32_t* fb, uint32_t* dst, int w, int h, int pitch_words)
{
    const int quads = (w + 3) / 4;
    const int bx = (quads + 255) / 256;
    hipLaunchKernelGGL(k_bgrx, dim3(bx, h), dim3(256), 0, s, fb, dst, w, h, pitch_words);
}

void rt_launch_shard_copy(hipStream_t s, const ShardJobs& jobs, int n, int w, int h, int count, int pack)
{
    if (n <= 0 || n > RT_SHARD_JOBS) return;
    // shard 0 holds the most tiles: its count is the grid's x extent
    const size_t tiles = rt_shard_tiles(w, h, 0, count);
    if (tiles == 0) return;
    hipLaunchKernelGGL(k_shard_copy, dim3((unsigned)tiles, (unsigned)n), dim3(256), 0, s, jobs, w, h, count, pack);
}

// ---------------------------------------------------------------------------
// Diagnostics: device evaluation of the numeric primitives, noise3d and
// getDensity for the primitive-level parity tests (tests/test_gpu_parity.py).
namespace {

__global__ void k_debug_math(int op, const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y,
                             int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == 12) {
        // octave-count sweep: d2 = the float with bits bits(a[0]) + i; counts (in y[0..2] as
        // uint32) unflagged estimates that differ from np_octaves_exact, flagged lanes, and
        // how many of the swept d2 exist
        const float d2 = rtm::fbits(rtm::bits(a[0]) + (uint32_t)i);
        bool near;
        const int est = rts::np_octaves_estimate(d2, &near);
        uint32_t* cnt = reinterpret_cast<uint32_t*>(y);
        if (!near && est != rts::np_octaves_exact(d2)) atomicAdd(&cnt[0], 1u);
        const uint64_t bn = __ballot(near), ba = __ballot(true);
        if (__lane_id() == 0) {
            if (bn) atomicAdd(&cnt[1], (uint32_t)__popcll(bn));
            atomicAdd(&cnt[2], (uint32_t)__popcll(ba));
        }
        return;
    }
    float x = a[i], v = 0.0f;
    switch (op) {
    case 0: v = rtm::exp2(x); break;
    case 1: v = rtm::log2(x); break;
    case 2: v = rtm::exp(x); break;
    case 3: v = rtm::sin(x); break;
    case 4: v = rtm::cos(x); break;
    case 5: v = rtm::sqrt(x); break;
    case 6: v = rtm::rcp(x); break;
    case 7: v = rtm::rcp(rtm::sqrt(x)); break;
    case 8: v = rtm::pow(x, b[i]); break;
    case 9: v = rtm::max(x, b[i]); break;
    case 10: v = rtm::min(x, b[i]); break;
    case 11: v = rtm::pow_nonneg(x, b[i]); break;
    default: v = 0.0f; break;
    }
    y[i] = v;
}

template <int L>
__global__ void __launch_bounds__(256) k_debug_noise(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                                     const float4* __restrict__ grad, const float* __restrict__ xyz,
                                                     float* __restrict__ out, int n, int density)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kNoiseLdsWords];
    load_noise_lds(lds, perm2d, grad, k);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ctx c = make_ctx(k, lds);
    f3 p = rtm::mk(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    // density 2: noise3d_z0(x, y) (z ignored)
    if (density == 2) {
        out[i] = noise3d_z0(c.nz, p.x, p.y);
    } else {
        out[i] = density ? get_density<L>(c, p) : noise3d(c.nz, p.x, p.y, p.z);
    }
}

// sky.hlsl:26-36,83-137 for one view direction per thread: (mie, rayleigh, space)
__global__ void __launch_bounds__(256) k_debug_sky(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                                   const float4* __restrict__ grad, const float* __restrict__ dirs,
                                                   float* __restrict__ out, int n)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kNoiseLdsWords];
    load_noise_lds(lds, perm2d, grad, k);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ctx c = make_ctx(k, lds);
    const f3 d = rtm::mk(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
    const SkyColor sc = get_rayleigh_mie(c, d);
    const float space = get_space_color(c, d);
    float* o = out + 7 * i;
    o[0] = sc.mie.x;
    o[1] = sc.mie.y;
    o[2] = sc.mie.z;
    o[3] = sc.rayleigh.x;
    o[4] = sc.rayleigh.y;
    o[5] = sc.rayleigh.z;
    o[6] = space;
}

// scripts/batch_shard_sim.py's coupled transport model (diagnostics): one wave that stores the 100 MHz
// clock when it starts (stamp, if set), waits until base[0] + until_ticks (base set: a stamp of an earlier
// launch; a peer's side of a transfer becoming ready), then spins `ticks` more (the transfer), holding a CU
// like a collective's kernel.  Vector stores only.
__global__ void __launch_bounds__(64) k_debug_spin(const unsigned long long* base, unsigned long long until_ticks,
                                                  unsigned long long ticks, unsigned long long* stamp)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (stamp && threadIdx.x == 0) *stamp = t0;
    const unsigned long long ready = base ? base[0] + until_ticks : t0;
    const unsigned long long end = (ready > t0 ? ready : t0) + ticks;
    while (__builtin_amdgcn_s_memrealtime() < end) __builtin_amdgcn_s_sleep(16);
}

} // namespace

void rt_launch_debug_spin(hipStream_t s, const unsigned long long* base, unsigned long long until_ticks,
                          unsigned long long ticks, unsigned long long* stamp)
{
    hipLaunchKernelGGL(k_debug_spin, dim3(1), dim3(64), 0, s, base, until_ticks, ticks, stamp);
}

void rt_launch_debug_sky(const RtLaunch& a, const float* dirs, float* out, int n)
{
    hipLaunchKernelGGL(k_debug_sky, dim3((n + 255) / 256), dim3(256), 0, a.stream, a.consts, a.perm2d, a.grad, dirs, out, n);
}

void rt_launch_debug_math(hipStream_t s, int op, const float* a, const float* b, float* y, int n)
{
    hipLaunchKernelGGL(k_debug_math, dim3((n + 255) / 256), dim3(256), 0, s, op, a, b, y, n);
}

void rt_launch_debug_noise(const RtLaunch& a, const float* xyz, float* out, int n, int density)
{
    dim3 g((n + 255) / 256), b(256);
    switch (a.landscape) {
    case RT_TESTING: hipLaunchKernelGGL(k_debug_noise<RT_TESTING>, g, b, 0, a.stream, a.consts, a.perm2d, a.grad, xyz, out, n, density); break;
    case RT_SIMPLE: hipLaunchKernelGGL(k_debug_noise<RT_SIMPLE>, g, b, 0, a.stream, a.consts, a.perm2d, a.grad, xyz, out, n, density); break;
    case RT_GREENROCKS: hipLaunchKernelGGL(k_debug_noise<RT_GREENROCKS>, g, b, 0, a.stream, a.consts, a.perm2d, a.grad, xyz, out, n, density); break;
    default: hipLaunchKernelGGL(k_debug_noise<RT_NOMADPLAINS>, g, b, 0, a.stream, a.consts, a.perm2d, a.grad, xyz, out, n, density); break;
    }
}

#ifdef RT_LIVE_HIST
// diagnostic build: copies (and with reset != 0 clears) the live-lanes-per-primary-step histogram
extern "C" int rt_debug_live_hist(unsigned long long* out, int reset)
{
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_live_hist), 65 * 8) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long zero[65] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_live_hist), zero, 65 * 8) != hipSuccess) return -1;
    }
    return 65;
}
#endif

#ifdef RT_WAVE_TRACE
// copies the last k_trace launch's per-wave timeline (RT_WT_FIELDS u64 per wave slot)
extern "C" int rt_debug_wave_trace(unsigned long long* out, int max_waves)
{
    const int n = max_waves < RT_WT_MAX_WAVES ? max_waves : RT_WT_MAX_WAVES;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_trace), (size_t)n * RT_WT_FIELDS * 8) != hipSuccess) return -1;
    return RT_WT_FIELDS;
}
#endif
