// Issue cost of single VALU instructions on gfx950 at 4 waves per SIMD (one 1024-thread block per
// CU, 256 CUs), 8 independent chains per lane, each instruction in inline asm so the compiler
// neither packs nor removes it.  Prints cycles per wave-instruction per SIMD at the clock measured
// with s_memtime / s_memrealtime.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_issue.hip -o scripts/_build/ubench_issue
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS(OP)                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { OP; }

template <int K>
__global__ void __launch_bounds__(1024) k_issue(unsigned int* out, unsigned long long* clk)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned int v[8], w[8];
    unsigned long long d[8];
    for (int i = 0; i < 8; ++i) {
        v[i] = threadIdx.x * 7u + (unsigned)i * 3u + 1u;
        w[i] = v[i] ^ 0x3f800000u;
        d[i] = v[i];
    }
    const unsigned int s = 0x01010101u;
    for (int it = 0; it < 2048; ++it) {
        if constexpr (K == 0) CHAINS(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 1) CHAINS(asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 2) CHAINS(asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 3) CHAINS(asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(d[i])))
        if constexpr (K == 4) CHAINS(asm volatile("v_floor_f32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 5) CHAINS(asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 6) CHAINS(asm volatile("v_cvt_flr_i32_f32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 7) CHAINS(asm volatile("v_fract_f32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 8) CHAINS(asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(w[i]), "s"(s)))
        if constexpr (K == 9) CHAINS(asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(d[i]) : "v"(v[i]), "s"(s) : "vcc"))
        if constexpr (K == 10) CHAINS(asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "s"(s), "v"(w[i])))
        if constexpr (K == 11) CHAINS(asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 12) CHAINS(asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 13) CHAINS(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 14) CHAINS(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 15) CHAINS(asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 16) CHAINS(asm volatile("v_bfe_u32 %0, %0, 8, 7" : "+v"(v[i])))
        if constexpr (K == 17) CHAINS(asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 18) CHAINS(asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 19) CHAINS(asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 20) CHAINS(asm volatile("v_exp_f32 %0, %0" : "+v"(v[i])))
        if constexpr (K == 21) CHAINS(asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(d[i])))
        if constexpr (K == 22) CHAINS(asm volatile("v_lshlrev_b32 %0, 2, %0" : "+v"(v[i])))
        if constexpr (K == 23) CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 24) CHAINS(asm volatile("v_fmamk_f32 %0, %0, 0x3f800001, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 25) CHAINS(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
    }
    unsigned int acc = 0;
    for (int i = 0; i < 8; ++i) acc += v[i] + (unsigned int)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int K>
void run(const char* name, unsigned int* out, unsigned long long* clk)
{
    hipLaunchKernelGGL(k_issue<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_issue<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
    const double per = ms / 5 * 1e-3 / (2048.0 * 8 * 4); // seconds per wave-instruction per SIMD
    printf("%-20s %.2f cycles per wave-instruction per SIMD (clock %.2f GHz)\n", name, per * ghz * 1e9, ghz);
}

int main()
{
    unsigned int* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, 256 * 1024 * sizeof(unsigned int));
    (void)hipMalloc(&clk, 16);
    run<0>("v_fma_f32", out, clk);
    run<1>("v_fmac_f32", out, clk);
    run<24>("v_fmamk_f32", out, clk);
    run<2>("v_add_f32", out, clk);
    run<13>("v_mul_f32", out, clk);
    run<14>("v_sub_f32", out, clk);
    run<3>("v_pk_fma_f32", out, clk);
    run<21>("v_pk_add_f32", out, clk);
    run<4>("v_floor_f32", out, clk);
    run<7>("v_fract_f32", out, clk);
    run<5>("v_cvt_i32_f32", out, clk);
    run<6>("v_cvt_flr_i32_f32", out, clk);
    run<17>("v_cvt_f32_i32", out, clk);
    run<8>("v_perm_b32", out, clk);
    run<9>("v_mad_u64_u32", out, clk);
    run<15>("v_mad_u32_u24", out, clk);
    run<25>("v_mul_lo_u32", out, clk);
    run<10>("v_and_or_b32", out, clk);
    run<11>("v_lshl_or_b32", out, clk);
    run<18>("v_or3_b32", out, clk);
    run<12>("v_and_b32", out, clk);
    run<19>("v_add_u32", out, clk);
    run<22>("v_lshlrev_b32", out, clk);
    run<16>("v_bfe_u32", out, clk);
    run<23>("v_cndmask_b32", out, clk);
    run<20>("v_exp_f32", out, clk);
    return 0;
}
