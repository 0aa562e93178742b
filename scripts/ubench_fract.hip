// Exhaustive check over every finite float x (both signs) of the gfx950 instructions a noise3d
// cell could use instead of floor / cvt / sub:
//   v_fract_f32(x)         vs  x - floor(x)                 (the oracle's fraction, rule R1)
//   v_cvt_flr_i32_f32(x)   vs  (int)floor(x)                 (lattice index, |x| < 2^31)
// and the issue cost of v_mad_u64_u32, v_perm_b32, v_cvt_i32_f32, v_floor_f32, v_fract_f32,
// v_cvt_flr_i32_f32 at 4 waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_fract.hip -o scripts/_build/ubench_fract
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_sweep(unsigned long long base, unsigned int* bad)
{
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned int bits = (unsigned int)i;
    const float x = __uint_as_float(bits);
    if (!(__builtin_fabsf(x) < __builtin_inff())) return;
    const float fl = __builtin_floorf(x);
    const float ref = x - fl;
    const float fr = __builtin_amdgcn_fractf(x);
    if (__float_as_uint(fr) != __float_as_uint(ref)) {
        const unsigned int n = atomicAdd(&bad[0], 1u);
        if (n < 8) bad[8 + n] = bits;
    }
    if (__builtin_fabsf(x) < 2147483520.0f) {
        int a;
        asm volatile("v_cvt_flr_i32_f32 %0, %1" : "=v"(a) : "v"(x));
        if (a != (int)fl) atomicAdd(&bad[1], 1u);
    }
}

template <int OP>
__global__ void __launch_bounds__(1024) k_cost(unsigned int* out, unsigned int s)
{
    unsigned int v[8];
    float f[8];
    for (int i = 0; i < 8; ++i) {
        v[i] = threadIdx.x * 7u + i;
        f[i] = (float)(threadIdx.x + i) * 0.37f;
    }
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) { // v_mad_u64_u32 (as noise3d's t + Z * 0x01010101)
                unsigned long long r;
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(v[i]), "s"(s), "v"((unsigned long long)v[i]) : "vcc");
                v[i] = (unsigned int)r;
            } else if constexpr (OP == 1) {
                v[i] = __builtin_amdgcn_perm(v[i], s, 0x0c0c0400u);
            } else if constexpr (OP == 2) {
                v[i] = (unsigned int)(int)f[i];
                f[i] = __uint_as_float(v[i] | 0x3f800000u);
            } else if constexpr (OP == 3) {
                f[i] = __builtin_floorf(f[i]) + 0.5f;
            } else if constexpr (OP == 4) {
                f[i] = __builtin_amdgcn_fractf(f[i] + 1.5f);
            } else if constexpr (OP == 5) {
                v[i] = v[i] * 0x01010101u;
            } else {
                f[i] = __builtin_fmaf(f[i], 1.0001f, 0.5f);
            }
        }
    }
    unsigned int acc = 0;
    for (int i = 0; i < 8; ++i) acc += v[i] + __float_as_uint(f[i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
void cost(const char* name, unsigned int* out)
{
    hipLaunchKernelGGL(k_cost<OP>, dim3(256), dim3(1024), 0, 0, out, 0x01010101u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_cost<OP>, dim3(256), dim3(1024), 0, 0, out, 0x01010101u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // 4 waves per SIMD, 4096 x 8 operations per wave
    const double ns = ms / 5 * 1e6 / (4096.0 * 8 * 4);
    printf("%-22s %.3f ns per op-group per SIMD (~%.2f cycles at 2.1 GHz; fma-only = reference)\n", name, ns, ns * 2.1);
}

int main()
{
    unsigned int* bad;
    hipMalloc(&bad, 64 * sizeof(unsigned int));
    hipMemset(bad, 0, 64 * sizeof(unsigned int));
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(k_sweep, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, bad);
    unsigned int h[16];
    hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    printf("v_fract_f32 != x - floor(x): %u inputs", h[0]);
    for (int i = 0; i < 8 && i < (int)h[0]; ++i) printf(" %08x", h[8 + i]);
    printf("\nv_cvt_flr_i32_f32 != (int)floor(x): %u inputs\n", h[1]);
    unsigned int* out;
    hipMalloc(&out, 256 * 1024 * sizeof(unsigned int));
    cost<6>("v_fma_f32", out);
    cost<0>("v_mad_u64_u32", out);
    cost<5>("v_mul_lo_u32", out);
    cost<1>("v_perm_b32", out);
    cost<2>("v_cvt_i32_f32 + v_or", out);
    cost<3>("v_floor_f32 + v_add", out);
    cost<4>("v_fract_f32 + v_add", out);
    return 0;
}
