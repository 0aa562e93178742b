// Microbenchmark of the nomadplains FBM body in isolation (rts::np_fbm and experimental variants),
// at k_trace's occupancy: one 1024-thread block per CU holding the same LDS noise image (perm2D,
// gxy/gz pairs, octave tables) padded to k_trace's 159 KiB.  Each lane marches a fixed ray of
// density samples (wave-coherent start distance, so the octave counts vary the way they do between
// neighbouring pixels); every variant must return the same bits as variant 0.
// Prints per variant: ms per launch, cycles per wave-octave on a SIMD (clock from s_memtime /
// s_memrealtime) and the lane utilisation of the octave loop.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//        -fno-fast-math scripts/ubench_fbm.hip -o scripts/_build/ubench_fbm
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../gpgpuraytrace_amd/csrc/rt_shader.h"

using namespace rts;
using rtm::f3;

constexpr int kPermWords = 128 * 128;
constexpr int kNpOct = RT_NP_OCTAVES + 3, kColOct = RT_COL_OCTAVES + 3;
constexpr int kOctWords = (kNpOct * 4 + kColOct * 2 + 3) / 4 * 4;
constexpr int kOctBase = (int)kLdsGz / 4 + (int)(kLdsGz - kLdsGxy) / 4;
constexpr int kNoiseLdsWords = kOctBase + kOctWords;
constexpr int kPadWords = (159392 / 4) - kNoiseLdsWords; // k_trace's LDS footprint

__device__ __forceinline__ void load_image(uint32_t* lds, const uint32_t* perm2d, const float4* grad, const RtConsts* k)
{
    float4* oct = reinterpret_cast<float4*>(lds + kOctBase);
    float2* colt = reinterpret_cast<float2*>(oct + kNpOct);
    const int i = threadIdx.x;
    if (i < kNpOct) {
        const int n = i <= RT_NP_OCTAVES ? i : RT_NP_OCTAVES;
        oct[i] = make_float4(k->np_scale[n], k->np_scale_y[n], k->np_rcp[n], 0.0f);
    }
    if (i < kColOct) {
        const int n = i <= RT_COL_OCTAVES ? i : RT_COL_OCTAVES;
        colt[i] = make_float2(k->col_scale[n], k->col_rcp[n]);
    }
    float4* gxy = reinterpret_cast<float4*>(lds + kLdsGxy / 4);
    float4* gz = reinterpret_cast<float4*>(lds + kLdsGz / 4);
    for (int j = threadIdx.x; j < 128 * 16; j += blockDim.x) {
        int e = j >> 4;
        float4 g0 = grad[e], g1 = grad[(e + 1) & 127];
        gxy[j] = make_float4(g0.x, g1.x, g0.y, g1.y);
        gz[j] = make_float4(g0.z, g1.z, 0.0f, 0.0f);
    }
    uint4* p = reinterpret_cast<uint4*>(lds);
    const uint4* src = reinterpret_cast<const uint4*>(perm2d);
    for (int j = threadIdx.x; j < kPermWords / 4; j += blockDim.x) p[j] = src[j];
    __syncthreads();
}

// the cell with a volatile texel read: keeps InstCombine from turning the pipeline's phi of two
// loads into one load of a phi (which moves the texel read back next to its use)
template <bool FAST>
__device__ __forceinline__ NoiseCell cell_v(const NoiseView& nz, float px, float py, float pz)
{
    NoiseCell c;
    const float fx = rtm::floor(px), fy = rtm::floor(py), fz = rtm::floor(pz);
    c.xy = v2(px, py) - v2(fx, fy);
    c.z = pz - fz;
    c.Z = layer_index<FAST>(fz);
    typedef __attribute__((address_space(3))) const volatile uint32_t lds_u32;
    c.t = *(lds_u32*)(nz.img + texel_offset<FAST>(fx, fy));
    return c;
}

// noise3d_lattice with the lerp tail in scalar ops (same fma chains): a packed FP32 result read by
// the next packed op costs an s_nop hazard slot on gfx950; scalar consumers do not
__device__ __forceinline__ float lattice_s(const NoiseView& nz, uint32_t t, uint32_t Z, float x, float y, float x1,
                                           float y1, float z, float ux, float uy, float uz)
{
    uint32_t w = (t + Z * 0x01010101u) & 0x7f7f7f7fu;
    auto gxy_at = [&](uint32_t sel) {
        return *reinterpret_cast<const float4*>(nz.img + __builtin_amdgcn_perm(w, nz.so16, sel));
    };
    auto gz_at = [&](uint32_t sel) {
        return *reinterpret_cast<const float2*>(nz.img + (kLdsGz - kLdsGxy) + __builtin_amdgcn_perm(w, nz.so16, sel));
    };
    const float4 a0 = gxy_at(0x0c020400u), a1 = gxy_at(0x0c020500u), b0 = gxy_at(0x0c020600u), b1 = gxy_at(0x0c020700u);
    const float2 za0 = gz_at(0x0c020400u), za1 = gz_at(0x0c020500u), zb0 = gz_at(0x0c020600u), zb1 = gz_at(0x0c020700u);
    const v2f zz = v2(z, z + -1.0f);
    const v2f g00 = gdot2(a0, za0, x, y, zz), g10 = gdot2(b0, zb0, x1, y, zz);
    const v2f g01 = gdot2(a1, za1, x, y1, zz), g11 = gdot2(b1, zb1, x1, y1, zz);
    const float lx00 = fma(ux, g10.x - g00.x, g00.x), lx01 = fma(ux, g10.y - g00.y, g00.y);
    const float lx10 = fma(ux, g11.x - g01.x, g01.x), lx11 = fma(ux, g11.y - g01.y, g01.y);
    const float l0 = fma(uy, lx10 - lx00, lx00), l1 = fma(uy, lx11 - lx01, lx01);
    return fma(uz, l1 - l0, l0);
}

template <bool FAST>
__device__ __forceinline__ float fbm_slerp(const Ctx& c, f3 q0, int n_oct)
{
    float s = 0.0f;
#pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES; ++N) {
        if (N > n_oct) break;
        const float4 oc = c.nz.oct[N];
        count_noise(c.nz);
        const NoiseCell ce = noise3d_cell<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x);
        const v2f uxy = fade2(ce.xy);
        const v2f xy1 = ce.xy + v2(-1.0f, -1.0f);
        s = fma(lattice_s(c.nz, ce.t, ce.Z, ce.xy.x, ce.xy.y, xy1.x, xy1.y, ce.z, uxy.x, uxy.y, fade(ce.z)), oc.z, s);
    }
    return s;
}

// ---- variants ------------------------------------------------------------------------------
// 0: rts::np_fbm (product)
// 1: octave N+1's cell (texel load) issued before octave N's lattice half
template <bool FAST>
__device__ __forceinline__ float fbm_pipe(const Ctx& c, f3 q0, int n_oct)
{
    float s = 0.0f;
    float4 oc = c.nz.oct[1];
    NoiseCell cur = cell_v<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x);
#pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES; ++N) {
        if (N > n_oct) break;
        const float4 on = c.nz.oct[N + 1];
        const NoiseCell nxt = cell_v<FAST>(c.nz, q0.x * on.x, q0.y * on.y, q0.z * on.x);
        count_noise(c.nz);
        s = fma(noise3d_finish(c.nz, cur), oc.z, s);
        cur = nxt;
        oc = on;
    }
    return s;
}

// 2: as 1, and the octave constants two octaves ahead (their LDS read leaves the critical path)
template <bool FAST>
__device__ __forceinline__ float fbm_pipe2(const Ctx& c, f3 q0, int n_oct)
{
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const volatile v4f lds_f4;
    float s = 0.0f;
    float4 oc = c.nz.oct[1], on = c.nz.oct[2];
    NoiseCell cur = cell_v<FAST>(c.nz, q0.x * oc.x, q0.y * oc.y, q0.z * oc.x);
#pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES; ++N) {
        if (N > n_oct) break;
        const v4f ov = *(lds_f4*)(c.nz.oct + N + 2);
        const float4 onn = make_float4(ov.x, ov.y, ov.z, ov.w);
        const NoiseCell nxt = cell_v<FAST>(c.nz, q0.x * on.x, q0.y * on.y, q0.z * on.x);
        count_noise(c.nz);
        s = fma(noise3d_finish(c.nz, cur), oc.z, s);
        cur = nxt;
        oc = on;
        on = onn;
    }
    return s;
}

// 3: octave pairs: octaves N and N+1 evaluated together (two independent dependency chains per
// lane), summed in octave order; a wave none of whose lanes needs N+1 evaluates N alone
template <bool FAST>
__device__ __forceinline__ float fbm_pairs(const Ctx& c, f3 q0, int n_oct)
{
    float s = 0.0f;
#pragma unroll 1
    for (int N = 1; N <= RT_NP_OCTAVES; N += 2) {
        if (N > n_oct) break;
        const float4 oa = c.nz.oct[N];
        if (__ballot(N + 1 <= n_oct)) {
            const float4 ob = c.nz.oct[N + 1];
            const NoiseCell ca = noise3d_cell<FAST>(c.nz, q0.x * oa.x, q0.y * oa.y, q0.z * oa.x);
            const NoiseCell cb = noise3d_cell<FAST>(c.nz, q0.x * ob.x, q0.y * ob.y, q0.z * ob.x);
            const float va = noise3d_finish(c.nz, ca), vb = noise3d_finish(c.nz, cb);
            count_noise(c.nz);
            s = fma(va, oa.z, s);
            if (N + 1 <= n_oct) {
                count_noise(c.nz);
                s = fma(vb, ob.z, s);
            }
        } else {
            count_noise(c.nz);
            s = fma(noise3d_finish(c.nz, noise3d_cell<FAST>(c.nz, q0.x * oa.x, q0.y * oa.y, q0.z * oa.x)), oa.z, s);
        }
    }
    return s;
}

template <int V>
__device__ __forceinline__ float fbm(const Ctx& c, f3 q0, int n)
{
    if constexpr (V == 4) return fbm_slerp<true>(c, q0, n);
    else if constexpr (V == 3) return fbm_pairs<true>(c, q0, n);
    if constexpr (V == 2) return fbm_pipe2<true>(c, q0, n);
    else if constexpr (V == 1) return fbm_pipe<true>(c, q0, n);
    else return np_fbm<true>(c, q0, n);
}

template <int V, bool COUNT>
__global__ void __launch_bounds__(1024) k_fbm(const RtConsts* __restrict__ k, const uint32_t* __restrict__ perm2d,
                                              const float4* __restrict__ grad, uint32_t* __restrict__ out,
                                              unsigned long long* __restrict__ cnt, unsigned long long* clk, int samples)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kNoiseLdsWords + kPadWords];
    load_image(lds, perm2d, grad, k);
    if (threadIdx.x == 0) lds[kNoiseLdsWords] = 0; // keep the pad
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    Ctx c;
    c.nz.img = reinterpret_cast<const char*>(lds);
    c.nz.oct = reinterpret_cast<const float4*>(lds + kOctBase);
    c.nz.colt = reinterpret_cast<const float2*>(c.nz.oct + kNpOct);
    c.nz.so16 = kLdsGxy | ((threadIdx.x & 15u) * 16u);
    c.nz.calls = 0;
    c.k = k;
    c.kf = k;
    c.eye = rtm::mk(0.0f, 100.0f, 0.0f);
    c.sun = rtm::mk(0.0f, 1.0f, 0.0f);
    const uint32_t lane = threadIdx.x & 63u, wave = blockIdx.x * 16u + (threadIdx.x >> 6);
    // a ray per lane inside an 8x8 pixel block's frustum; start distance per wave (1 .. ~2000)
    const float ax = ((float)(lane & 7u) - 3.5f) * 0.0015f + (float)(wave % 61u) * 0.01f;
    const float ay = ((float)(lane >> 3) - 3.5f) * 0.0015f - 0.05f - (float)(wave % 7u) * 0.01f;
    f3 dir = rtm::normalize(rtm::mk(ax, ay, 1.0f));
    // every wave marches the same 32 start distances (1 .. 1985) in a rotated order: equal work per
    // wave, so the persistent grid has no tail
    auto tstart = [&](int i) { return 1.0f + (float)(((uint32_t)(i >> 6) + wave) & 31u) * 64.0f; };
    float t = tstart(0);
    uint32_t acc = 0;
    for (int i = 0; i < samples; ++i) {
        const f3 p = rtm::mk(fma(dir.x, t, c.eye.x), fma(dir.y, t, c.eye.y), fma(dir.z, t, c.eye.z));
        const f3 q0 = rtm::scale(rtm::scale(p, 0.4f), 0.006f);
        const int n = np_octaves(c, p);
        const float s = fbm<V>(c, q0, n);
        acc = (acc * 0x9E3779B1u) ^ rtm::bits(s);
        t = (i & 63) == 63 ? tstart(i + 1) : t * 1.004f + 0.05f;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if constexpr (COUNT) {
        atomicAdd(&cnt[0], (unsigned long long)(c.nz.calls & 0xffffffffull));
        atomicAdd(&cnt[1], (unsigned long long)(c.nz.calls >> 32));
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

struct Dev {
    RtConsts* k;
    uint32_t* perm;
    float4* grad;
    uint32_t* out;
    unsigned long long* cnt;
    unsigned long long* clk;
};

template <int V>
void run(const Dev& d, int samples, std::vector<uint32_t>& ref)
{
    const int n = 256 * 1024;
    (void)hipMemset(d.cnt, 0, 16);
    hipLaunchKernelGGL((k_fbm<V, true>), dim3(256), dim3(1024), 0, 0, d.k, d.perm, d.grad, d.out, d.cnt, d.clk, samples);
    unsigned long long cnt[2];
    (void)hipMemcpy(cnt, d.cnt, 16, hipMemcpyDeviceToHost);
    std::vector<uint32_t> h(n);
    hipLaunchKernelGGL((k_fbm<V, false>), dim3(256), dim3(1024), 0, 0, d.k, d.perm, d.grad, d.out, d.cnt, d.clk, samples);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_fbm<V, false>), dim3(256), dim3(1024), 0, 0, d.k, d.perm, d.grad, d.out, d.cnt, d.clk,
                           samples);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    (void)hipMemcpy(h.data(), d.out, n * 4, hipMemcpyDeviceToHost);
    unsigned long long c[2];
    (void)hipMemcpy(c, d.clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
    const double cyc = ms * 1e-3 * ghz * 1e9 * 1024.0 / (double)cnt[1]; // SIMD-cycles per wave-octave
    bool same = true;
    if (ref.empty()) ref = h;
    else same = ref == h;
    printf("variant %d: %.3f ms, %.1f cycles per wave-noise per SIMD (clock %.2f GHz), lane util %.3f, %s\n", V, ms, cyc,
           ghz, (double)cnt[0] / (64.0 * (double)cnt[1]), same ? "bit-exact" : "MISMATCH");
}

int main(int argc, char** argv)
{
    const int samples = argc > 1 ? atoi(argv[1]) : 64;
    // tables: a seeded permutation, perm2D and gradients built like Noise.cpp (not the product seed)
    static const float g3[16][3] = {{1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1},
                                    {1, 0, -1}, {-1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1},
                                    {1, 1, 0}, {0, -1, 1}, {-1, 1, 0}, {0, -1, -1}};
    std::mt19937 rng(300);
    std::vector<int> P(128);
    for (int i = 0; i < 128; ++i) P[i] = i;
    for (int i = 0; i < 128; ++i) std::swap(P[i], P[rng() % 128]);
    std::vector<uint32_t> perm(128 * 128);
    for (int x = 0; x < 128; ++x)
        for (int y = 0; y < 128; ++y) {
            int A = P[x] + y, B = P[(x + 1) % 128] + y;
            perm[x + y * 128] = (uint32_t)P[A % 128] | (uint32_t)P[(A + 1) % 128] << 8 | (uint32_t)P[B % 128] << 16 |
                                (uint32_t)P[(B + 1) % 128] << 24;
        }
    std::vector<float> grad(128 * 4);
    for (int x = 0; x < 128; ++x)
        for (int j = 0; j < 3; ++j) grad[x * 4 + j] = g3[P[x] % 16][j];
    RtConsts k;
    memset(&k, 0, sizeof(k));
    for (int n = 1; n <= RT_NP_OCTAVES; ++n) {
        float S = rtm::pow(1.96f, (float)n);
        k.np_scale[n] = S;
        k.np_scale_y[n] = S * 0.35f;
        k.np_rcp[n] = rtm::rcp(S);
    }
    k.np_expo = 0.78f;
    Dev d;
    (void)hipMalloc(&d.k, sizeof(k));
    (void)hipMalloc(&d.perm, perm.size() * 4);
    (void)hipMalloc(&d.grad, grad.size() * 4);
    (void)hipMalloc(&d.out, 256 * 1024 * 4);
    (void)hipMalloc(&d.cnt, 16);
    (void)hipMalloc(&d.clk, 16);
    (void)hipMemcpy(d.k, &k, sizeof(k), hipMemcpyHostToDevice);
    (void)hipMemcpy(d.perm, perm.data(), perm.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d.grad, grad.data(), grad.size() * 4, hipMemcpyHostToDevice);
    std::vector<uint32_t> ref;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(d, samples, ref);
        run<1>(d, samples, ref);
        run<2>(d, samples, ref);
        run<3>(d, samples, ref);
        run<4>(d, samples, ref);
    }
    return 0;
}
