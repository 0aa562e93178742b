// Microbenchmark: issue cost of v_fma_f32 vs v_pk_fma_f32 (and v_pk_mul / v_pk_add) on gfx950,
// 4 and 8 waves per SIMD, 8 independent accumulator chains per lane.  Prints ns per wave-instruction
// per SIMD and the implied cycles at the measured clock (s_memtime / s_memrealtime).
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu.hip -o /tmp/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int kIters = 4096;

template <int MODE>
__global__ void __launch_bounds__(1024) k_valu(float* out, float a, float b, unsigned long long* clk)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = (float)(threadIdx.x + i);
    for (int it = 0; it < kIters; ++it) {
        if constexpr (MODE == 0) { // 16 scalar FMAs
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], a, b);
        } else if constexpr (MODE == 1) { // 8 packed FMAs (same 16 FMAs)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                v2f v = {x[i], x[i + 1]};
                v2f aa = {a, a}, bb = {b, b};
                v = __builtin_elementwise_fma(v, aa, bb);
                x[i] = v.x;
                x[i + 1] = v.y;
            }
        } else if constexpr (MODE == 2) { // 16 scalar muls
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = x[i] * a;
        } else { // 8 packed muls
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                v2f v = {x[i], x[i + 1]};
                v2f aa = {a, a};
                v = v * aa;
                x[i] = v.x;
                x[i + 1] = v.y;
            }
        }
    }
    float s = 0.0f;
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int MODE>
void run(const char* name, int waves_per_simd, float* out, unsigned long long* clk)
{
    const int threads = waves_per_simd * 4 * 64; // per CU (one block per CU)
    dim3 grid(256), block(threads);
    hipLaunchKernelGGL(k_valu<MODE>, grid, block, 0, 0, out, 1.0001f, 0.5f, clk);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_valu<MODE>, grid, block, 0, 0, out, 1.0001f, 0.5f, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9; // memrealtime ticks at 100 MHz
    const int instrs = (MODE == 0 || MODE == 2) ? 16 : 8;
    const double wave_instrs_per_simd = (double)kIters * instrs * waves_per_simd;
    const double ns = ms / 5 * 1e6 / wave_instrs_per_simd;
    printf("%-10s waves/SIMD %d: %.3f ms/launch, %.3f ns per wave-instr per SIMD = %.2f cycles at %.2f GHz\n", name,
           waves_per_simd, ms / 5, ns, ns * ghz, ghz);
}

int main()
{
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 1024 * sizeof(float));
    hipMalloc(&clk, 16);
    for (int w : {1, 2, 4}) {
        run<0>("v_fma_f32", w, out, clk);
        run<1>("v_pk_fma", w, out, clk);
        run<2>("v_mul_f32", w, out, clk);
        run<3>("v_pk_mul", w, out, clk);
    }
    return 0;
}
