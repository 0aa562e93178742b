// rt_kernels.hip -- HIP kernels for gfx950 (MI355X): camera prepass, cell
// depths, and the per-pixel screen trace.
//
//   k_camerarays   <- Media/common/shaders/camerarays.hlsl:12-21
//   k_cell_depths  <- Graphics/Terrain.cpp:356-439 (setTargetDepths, host code
//                     in the reference; on the device here so the frame needs
//                     no GPU->CPU->GPU round trip)
//   k_tracescreen  <- Media/common/shaders/tracescreen.hlsl:16-76
//
// Launch interface (rt_launch_*) is plain C++ used by rt_runtime.cpp.
#include <hip/hip_runtime.h>

#include "rt_kernels.h"
#include "rt_shader.h"

using namespace rts;
using rtm::f3;

namespace {

__device__ __forceinline__ Ctx make_ctx(const RtConsts* k, const uint32_t* perm2d, const uint8_t* codes2)
{
    Ctx c;
    c.nz.perm2d = perm2d;
    c.nz.codes2 = codes2;
    c.k = k;
    c.eye = rtm::mk(k->eye[0], k->eye[1], k->eye[2]);
    c.sun = rtm::mk(k->sun[0], k->sun[1], k->sun[2]);
    return c;
}

// ---------------------------------------------------------------------------
// camerarays.hlsl:12-21.  One thread per prepass cell (32x32).
template <int L, bool STATS>
__global__ void __launch_bounds__(64) k_camerarays(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                                   const uint8_t* __restrict__ codes2, float4* __restrict__ out,
                                                   RtStats* stats)
{
    __shared__ uint32_t s_perm[128 * 128];
    __shared__ uint8_t s_codes[128];
    for (int i = threadIdx.x; i < 128 * 128; i += blockDim.x) s_perm[i] = perm2d[i];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) s_codes[i] = codes2[i];
    __syncthreads();
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= RT_CAMERA_RES * RT_CAMERA_RES) return;
    Ctx c = make_ctx(k, s_perm, s_codes);
    int tx = i % RT_CAMERA_RES, ty = i / RT_CAMERA_RES;
    const float r31 = rtm::rcp(31.0f);
    uint32_t pxs = (uint32_t)(((float)tx * r31) * k->screen[0]);
    uint32_t pys = (uint32_t)(((float)ty * r31) * k->screen[1]);
    f3 p, dir;
    get_pixel_ray(c, (float)pxs, (float)pys, &p, &dir);
    RayResult rr = trace_ray<L, false, true>(c, p, RT_CAMERA_NEAR, RT_CAMERA_FAR, 2.0f, dir, 0);
    if (rr.density < 0.0f) rr.pd.w = RT_CAMERA_FAR;
    out[i] = make_float4(rr.pd.x, rr.pd.y, rr.pd.z, rr.pd.w);
    if constexpr (STATS) atomicAdd(&stats->prepass_steps, (unsigned long long)rr.steps);
}

// ---------------------------------------------------------------------------
// Terrain.cpp:356-439 with the host's std::min/std::max argument order.
__device__ __forceinline__ float cd_get_depth(const float* d, int x, int y)
{
    x = x < 0 ? 0 : (x >= RT_CAMERA_RES ? RT_CAMERA_RES - 1 : x);
    y = y < 0 ? 0 : (y >= RT_CAMERA_RES ? RT_CAMERA_RES - 1 : y);
    return d[y * RT_CAMERA_RES + x];
}
__device__ __forceinline__ float cd_interp(const float* d, int x, int y)
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

__global__ void __launch_bounds__(1024) k_cell_depths(const float4* __restrict__ cam, float2* __restrict__ cells)
{
    __shared__ float s_d[RT_CAMERA_RES * RT_CAMERA_RES];
    int i = threadIdx.x;
    s_d[i] = cam[i].w;
    __syncthreads();
    int xpos = i % RT_CAMERA_RES, ypos = i / RT_CAMERA_RES;
    float dmin = cd_interp(s_d, xpos, ypos);
    float dmax = dmin;
    for (int xp = -2; xp <= 2; ++xp) {
        for (int yp = -2; yp <= 2; ++yp) {
            float d = cd_interp(s_d, xpos + xp, ypos + yp);
            dmin = (dmin < d) ? dmin : d;
            dmax = (d < dmax) ? dmax : d;
        }
    }
    dmin = dmin * 0.96f - 0.01f;
    dmax = dmax * 1.22f + 0.4f;
    dmin = (RT_CAMERA_NEAR < dmin) ? dmin : RT_CAMERA_NEAR;
    dmax = (dmax < RT_CAMERA_FAR) ? dmax : RT_CAMERA_FAR;
    cells[i] = make_float2(dmin, dmax);
}

// ---------------------------------------------------------------------------
// tracescreen.hlsl:16-48 traceSample
template <int L>
__device__ __forceinline__ f3 trace_sample(const Ctx& c, f3 pp, f3 pdir, f3 pdn, float plane_x, float plane_y,
                                           float* psteps, float* ssteps, int* hit)
{
    RayResult rr = trace_ray<L, true, false>(c, pp, plane_x, plane_y, 1.0f, pdir, c.k->max_steps);
    *psteps += rr.steps;
    float skyAmount = rr.pd.w * 0.0005f;
    skyAmount = rtm::sat(skyAmount * skyAmount);
    SkyColor scat = get_rayleigh_mie(c, pdn);
    f3 color;
    if (rr.density > 0.0f) {
        *hit += 1;
        f3 n = get_normal<L>(c, rr.pd);
        f3 hp = rtm::mk(rr.pd.x, rr.pd.y, rr.pd.z);
        ShadePre sp = shade_pre<L>(c, hp, n, pdn, rr.pd.w);
        RayResult sr = trace_ray<L, true, true>(c, hp, 0.4f, 100.0f, sp.precision, c.sun, 0);
        *ssteps += sr.steps;
        color = shade_post(c, sp, sr.density, sr.fc.w);
        color = rtm::mk(rtm::lerp(color.x, rr.fc.x, rr.fc.w), rtm::lerp(color.y, rr.fc.y, rr.fc.w),
                        rtm::lerp(color.z, rr.fc.z, rr.fc.w));
        color = rtm::mk(rtm::lerp(color.x, scat.rayleigh.x, skyAmount), rtm::lerp(color.y, scat.rayleigh.y, skyAmount),
                        rtm::lerp(color.z, scat.rayleigh.z, skyAmount));
    } else {
        float space = get_space_color(c, pdn);
        f3 sky = rtm::mk((scat.mie.x + scat.rayleigh.x) + space, (scat.mie.y + scat.rayleigh.y) + space,
                         (scat.mie.z + scat.rayleigh.z) + space);
        color = rtm::mk(rtm::lerp(sky.x, rr.fc.x, rr.fc.w), rtm::lerp(sky.y, rr.fc.y, rr.fc.w),
                        rtm::lerp(sky.z, rr.fc.z, rr.fc.w));
        color = rtm::mk(rtm::lerp(color.x, sky.x, skyAmount), rtm::lerp(color.y, sky.y, skyAmount),
                        rtm::lerp(color.z, sky.z, skyAmount));
    }
    return color;
}

// tracescreen.hlsl:50-76.  Block = 64 threads = one wave = one 8x8 pixel tile
// of the dispatch region [off, off + extent).  LDS holds the 64 KiB lattice
// and the 128-byte gradient code table for the block's lifetime.
template <int L, bool STATS>
__global__ void __launch_bounds__(1024) k_tracescreen(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                                     const uint8_t* __restrict__ codes2,
                                                     const float2* __restrict__ cells, uint32_t* __restrict__ out8,
                                                     float4* __restrict__ out32, uint32_t off_x, uint32_t off_y,
                                                     uint32_t ext_x, uint32_t ext_y, uint32_t tiles_x,
                                                     uint32_t tile_first, uint32_t tile_stride, RtStats* stats)
{
    __shared__ uint32_t s_perm[128 * 128];
    __shared__ uint8_t s_codes[128];
    for (int i = threadIdx.x; i < 128 * 128; i += blockDim.x) s_perm[i] = perm2d[i];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) s_codes[i] = codes2[i];
    __syncthreads();

    // 1024-thread block = 16 waves = a 32x32 pixel tile, each wave an 8x8 sub-tile
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t lx = (uint32_t)((wave & 3) * 8 + (lane & 7));
    uint32_t ly = (uint32_t)((wave >> 2) * 8 + (lane >> 3));
    uint32_t tile = blockIdx.x * tile_stride + tile_first;
    uint32_t gx = (tile % tiles_x) * 32 + lx, gy = (tile / tiles_x) * 32 + ly;
    if (gx >= ext_x || gy >= ext_y) return;
    uint32_t px = gx + off_x, py = gy + off_y;
    if (px >= (uint32_t)k->width || py >= (uint32_t)k->height) return; // UAV writes outside texOut are dropped

    Ctx c = make_ctx(k, s_perm, s_codes);
    float pxf = (float)px, pyf = (float)py;
    float spx = pxf * k->rcp_w, spy = pyf * k->rcp_h;
    uint32_t cell = (uint32_t)rtm::fma(rtm::floor(spy * 32.0f), 32.0f, rtm::floor(spx * 32.0f));
    float plane_x = cells[cell].x, plane_y = RT_CAMERA_FAR;
    float col0 = 0.0f, col1 = 0.0f, col2 = 0.0f;
    float psteps = 0.0f, ssteps = 0.0f;
    int hit = 0;
    const int aa = k->aa_samples;
    for (int a = 0; a < aa; ++a) {
        f3 p, dir;
        get_pixel_ray(c, pxf + k->aa_off[a][0], pyf + k->aa_off[a][1], &p, &dir);
        f3 pdn = rtm::normalize(dir);
        f3 s = trace_sample<L>(c, p, dir, pdn, plane_x, plane_y, &psteps, &ssteps, &hit);
        col0 = col0 + rtm::sat(s.x);
        col1 = col1 + rtm::sat(s.y);
        col2 = col2 + rtm::sat(s.z);
    }
    float ia = rtm::rcp((float)aa);
    col0 = col0 * ia;
    col1 = col1 * ia;
    col2 = col2 * ia;
    size_t o = (size_t)py * (size_t)k->width + px;
    out8[o] = unorm8(col0) | (unorm8(col1) << 8) | (unorm8(col2) << 16) | 0xff000000u;
    if (out32) out32[o] = make_float4(col0, col1, col2, 1.0f);
    if constexpr (STATS) {
        atomicAdd(&stats->primary_steps, (unsigned long long)psteps);
        atomicAdd(&stats->shadow_steps, (unsigned long long)ssteps);
        atomicAdd(&stats->hits, (unsigned long long)hit);
    }
}

template <int L>
void launch_camerarays_l(const RtLaunch& a, float4* out)
{
    dim3 grid(RT_CAMERA_RES * RT_CAMERA_RES / 64), block(64);
    if (a.stats)
        hipLaunchKernelGGL((k_camerarays<L, true>), grid, block, 0, a.stream, a.consts, a.perm2d, a.codes2, out, a.stats);
    else
        hipLaunchKernelGGL((k_camerarays<L, false>), grid, block, 0, a.stream, a.consts, a.perm2d, a.codes2, out, a.stats);
}

template <int L>
void launch_tracescreen_l(const RtLaunch& a, const float2* cells, uint32_t* out8, float4* out32, uint32_t ox,
                          uint32_t oy, uint32_t ex, uint32_t ey, uint32_t first, uint32_t stride)
{
    uint32_t tiles_x = (ex + 31) / 32, tiles_y = (ey + 31) / 32, total = tiles_x * tiles_y;
    if (first >= total) return;
    uint32_t n = (total - first + stride - 1) / stride;
    dim3 grid(n), block(1024);
    if (a.stats)
        hipLaunchKernelGGL((k_tracescreen<L, true>), grid, block, 0, a.stream, a.consts, a.perm2d, a.codes2, cells, out8,
                           out32, ox, oy, ex, ey, tiles_x, first, stride, a.stats);
    else
        hipLaunchKernelGGL((k_tracescreen<L, false>), grid, block, 0, a.stream, a.consts, a.perm2d, a.codes2, cells,
                           out8, out32, ox, oy, ex, ey, tiles_x, first, stride, a.stats);
}

// Tile-cyclic shard transport: one 256-thread block per 32x32 tile.
__global__ void __launch_bounds__(256) k_shard_copy(uint32_t* __restrict__ fb, uint32_t* __restrict__ packed, int w,
                                                    int h, int rank, int count, int pack)
{
    int tiles_x = (w + 31) / 32;
    int k = blockIdx.x;
    int tile = k * count + rank;
    int tx0 = (tile % tiles_x) * 32, ty0 = (tile / tiles_x) * 32;
    for (int i = threadIdx.x; i < 1024; i += 256) {
        int x = tx0 + (i & 31), y = ty0 + (i >> 5);
        if (x >= w || y >= h) continue;
        size_t f = (size_t)y * w + x, p = (size_t)k * 1024 + i;
        if (pack) packed[p] = fb[f];
        else fb[f] = packed[p];
    }
}

} // namespace

void rt_launch_camerarays(const RtLaunch& a, float4* out)
{
    switch (a.landscape) {
    case RT_TESTING: launch_camerarays_l<RT_TESTING>(a, out); break;
    case RT_SIMPLE: launch_camerarays_l<RT_SIMPLE>(a, out); break;
    case RT_GREENROCKS: launch_camerarays_l<RT_GREENROCKS>(a, out); break;
    default: launch_camerarays_l<RT_NOMADPLAINS>(a, out); break;
    }
}

void rt_launch_cell_depths(hipStream_t s, const float4* cam, float2* cells)
{
    hipLaunchKernelGGL(k_cell_depths, dim3(1), dim3(1024), 0, s, cam, cells);
}

void rt_launch_tracescreen(const RtLaunch& a, const float2* cells, uint32_t* out8, float4* out32, uint32_t ox,
                           uint32_t oy, uint32_t ex, uint32_t ey, uint32_t first, uint32_t stride)
{
    if (ex == 0 || ey == 0 || stride == 0) return;
    switch (a.landscape) {
    case RT_TESTING: launch_tracescreen_l<RT_TESTING>(a, cells, out8, out32, ox, oy, ex, ey, first, stride); break;
    case RT_SIMPLE: launch_tracescreen_l<RT_SIMPLE>(a, cells, out8, out32, ox, oy, ex, ey, first, stride); break;
    case RT_GREENROCKS: launch_tracescreen_l<RT_GREENROCKS>(a, cells, out8, out32, ox, oy, ex, ey, first, stride); break;
    default: launch_tracescreen_l<RT_NOMADPLAINS>(a, cells, out8, out32, ox, oy, ex, ey, first, stride); break;
    }
}

void rt_launch_shard_copy(hipStream_t s, uint32_t* fb, uint32_t* packed, int w, int h, int rank, int count, int pack)
{
    size_t n = rt_shard_tiles(w, h, rank, count);
    if (n == 0) return;
    hipLaunchKernelGGL(k_shard_copy, dim3((unsigned)n), dim3(256), 0, s, fb, packed, w, h, rank, count, pack);
}
