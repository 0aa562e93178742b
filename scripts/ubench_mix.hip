// Issue cost of MIXED and DEPENDENT VALU streams on gfx950 at 4 waves per SIMD (one 1024-thread
// block per CU), to calibrate the cost model of k_trace's noise body (scripts/valu_cost.py):
// the single-type rates of scripts/ubench_issue.hip, then dependency chains of 1..8, 2- and 4-cycle
// ops interleaved, and VALU streams with s_nop / SALU / ds_read / s_waitcnt in between.
// Prints cycles per VALU wave-instruction per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_mix.hip -o scripts/_build/ubench_mix
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 1024;

#define FMA(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(w[i]))
#define PK(i) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(d[i]))
#define FLOOR(i) asm volatile("v_floor_f32 %0, %0" : "+v"(v[i]))
#define PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(w[i]), "s"(s))

template <int K>
__global__ void __launch_bounds__(1024) k_mix(unsigned int* out, unsigned long long* clk)
{
    __shared__ unsigned int lds[1024];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float v[8], w[8];
    double d[8];
    for (int i = 0; i < 8; ++i) {
        v[i] = (float)(threadIdx.x * 7u + (unsigned)i * 3u + 1u) * 1e-9f;
        w[i] = 0.5f;
        d[i] = v[i];
    }
    const unsigned int s = 0x01010101u;
    unsigned int acc = 0, sa = 0;
    const unsigned int addr = (threadIdx.x & 255u) * 4u;
    for (int it = 0; it < kIters; ++it) {
        if constexpr (K == 0) { // 8 independent v_fma chains (16 VALU per iteration)
#pragma unroll
            for (int r = 0; r < 2; ++r) for (int i = 0; i < 8; ++i) FMA(i);
        } else if constexpr (K == 1) { // 4 chains
#pragma unroll
            for (int r = 0; r < 4; ++r) for (int i = 0; i < 4; ++i) FMA(i);
        } else if constexpr (K == 2) { // 2 chains
#pragma unroll
            for (int r = 0; r < 8; ++r) for (int i = 0; i < 2; ++i) FMA(i);
        } else if constexpr (K == 3) { // 1 chain
#pragma unroll
            for (int r = 0; r < 16; ++r) FMA(0);
        } else if constexpr (K == 4) { // 8 independent v_pk_fma chains (16 per iteration)
#pragma unroll
            for (int r = 0; r < 2; ++r) for (int i = 0; i < 8; ++i) PK(i);
        } else if constexpr (K == 5) { // 2 pk chains
#pragma unroll
            for (int r = 0; r < 8; ++r) for (int i = 0; i < 2; ++i) PK(i);
        } else if constexpr (K == 6) { // 1 pk chain
#pragma unroll
            for (int r = 0; r < 16; ++r) PK(0);
        } else if constexpr (K == 7) { // fma / pk_fma alternating, 8 chains each
#pragma unroll
            for (int i = 0; i < 8; ++i) { FMA(i); PK(i); }
        } else if constexpr (K == 8) { // fma + floor alternating
#pragma unroll
            for (int i = 0; i < 8; ++i) { FMA(i); FLOOR(i); }
        } else if constexpr (K == 9) { // fma + perm alternating (int and float chains)
#pragma unroll
            for (int i = 0; i < 8; ++i) { FMA(i); asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(acc) : "v"(addr), "s"(s)); }
        } else if constexpr (K == 10) { // 16 fma + 4 s_nop
#pragma unroll
            for (int r = 0; r < 2; ++r) for (int i = 0; i < 8; ++i) { FMA(i); if (i & 1) { } else if (i & 2) asm volatile("s_nop 0"); }
        } else if constexpr (K == 11) { // 16 fma + 8 SALU
#pragma unroll
            for (int r = 0; r < 2; ++r) for (int i = 0; i < 8; ++i) { FMA(i); if (i & 1) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sa)); }
        } else if constexpr (K == 12) { // 16 fma + 4 ds_read_b32 (waited at the end of the iteration)
            unsigned int x0, x1, x2, x3;
            asm volatile("ds_read_b32 %0, %1" : "=v"(x0) : "v"(addr));
            asm volatile("ds_read_b32 %0, %1 offset:1024" : "=v"(x1) : "v"(addr));
#pragma unroll
            for (int i = 0; i < 8; ++i) FMA(i);
            asm volatile("ds_read_b32 %0, %1 offset:2048" : "=v"(x2) : "v"(addr));
            asm volatile("ds_read_b32 %0, %1 offset:3072" : "=v"(x3) : "v"(addr));
#pragma unroll
            for (int i = 0; i < 8; ++i) FMA(i);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc += x0 ^ x1 ^ x2 ^ x3;
        } else if constexpr (K == 13) { // 16 fma + 2 ds_read_b128 + 2 ds_read_b64
            unsigned int x0, x1, x2, x3;
            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
            typedef unsigned int u2 __attribute__((ext_vector_type(2)));
            u4 a, b;
            u2 c, e;
            asm volatile("ds_read_b128 %0, %1" : "=v"(a) : "v"(addr * 4u & 0xff0u));
            asm volatile("ds_read_b64 %0, %1 offset:2048" : "=v"(c) : "v"(addr * 2u & 0x7f8u));
#pragma unroll
            for (int i = 0; i < 8; ++i) FMA(i);
            asm volatile("ds_read_b128 %0, %1" : "=v"(b) : "v"(addr * 4u & 0xff0u));
            asm volatile("ds_read_b64 %0, %1 offset:2048" : "=v"(e) : "v"(addr * 2u & 0x7f8u));
#pragma unroll
            for (int i = 0; i < 8; ++i) FMA(i);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            x0 = a.x ^ b.y; x1 = c.x ^ e.y; x2 = a.z ^ b.w; x3 = c.y;
            acc += x0 ^ x1 ^ x2 ^ x3;
        } else if constexpr (K == 14) { // 2 chains alternating fma / pk (dependent mixed)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                FMA(0); FMA(1);
                PK(0); PK(1);
            }
        }
    }
    for (int i = 0; i < 8; ++i) acc += __float_as_uint(v[i]) + (unsigned int)(unsigned long long)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + sa;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int K>
void run(const char* name, int valu_per_iter, unsigned int* out, unsigned long long* clk)
{
    hipLaunchKernelGGL(k_mix<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mix<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
    const double per = ms / 5 * 1e-3 / ((double)kIters * valu_per_iter * 4); // s per VALU wave-instr per SIMD
    printf("%-44s %.2f cycles per VALU wave-instruction per SIMD (clock %.2f GHz)\n", name, per * ghz * 1e9, ghz);
}

int main()
{
    unsigned int* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, 256 * 1024 * sizeof(unsigned int));
    (void)hipMalloc(&clk, 16);
    run<0>("fma, 8 independent chains", 16, out, clk);
    run<1>("fma, 4 chains", 16, out, clk);
    run<2>("fma, 2 chains", 16, out, clk);
    run<3>("fma, 1 chain", 16, out, clk);
    run<4>("pk_fma, 8 chains", 16, out, clk);
    run<5>("pk_fma, 2 chains", 16, out, clk);
    run<6>("pk_fma, 1 chain", 16, out, clk);
    run<7>("fma + pk_fma alternating (model 3)", 16, out, clk);
    run<8>("fma + floor alternating (model 3)", 16, out, clk);
    run<9>("fma + perm alternating (model 3)", 16, out, clk);
    run<10>("16 fma + 4 s_nop", 16, out, clk);
    run<11>("16 fma + 8 s_add", 16, out, clk);
    run<12>("16 fma + 4 ds_read_b32 + waitcnt", 16, out, clk);
    run<13>("16 fma + 2 b128 + 2 b64 + waitcnt", 16, out, clk);
    run<14>("2 chains fma,fma,pk,pk (model 3)", 16, out, clk);
    return 0;
}
