// Issue cost of SDWA (sub-dword addressing) forms on gfx950 next to the ops they could replace in
// the noise lattice's address arithmetic (v_perm_b32, v_and_or_b32), at 4 waves per SIMD (one
// 1024-thread block per CU, 256 CUs), 8 independent chains per lane, each instruction in inline asm.
// The preserve forms write one byte of the destination and keep the other three, so the
// destination is read as well as written.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_sdwa.hip -o scripts/_build/ubench_sdwa
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS(OP)                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { OP; }

template <int K>
__global__ void __launch_bounds__(1024) k_sdwa(unsigned int* out, unsigned long long* clk)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned int v[8], w[8];
    for (int i = 0; i < 8; ++i) {
        v[i] = threadIdx.x * 7u + (unsigned)i * 3u + 1u;
        w[i] = v[i] ^ 0x3f800000u;
    }
    const unsigned int s = 0x0c020400u, m = 127u;
    unsigned int mv = m;
    asm volatile("" : "+v"(mv));
    for (int it = 0; it < 2048; ++it) {
        if constexpr (K == 0) CHAINS(asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "v"(w[i]), "s"(s)))
        if constexpr (K == 1)
            CHAINS(asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2"
                                : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 2)
            CHAINS(asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 "
                                "src1_sel:DWORD" : "+v"(v[i]) : "v"(w[i]), "v"(mv)))
        if constexpr (K == 3)
            CHAINS(asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 "
                                "src1_sel:DWORD" : "+v"(v[i]) : "v"(w[i]), "s"(m)))
        if constexpr (K == 4)
            CHAINS(asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 "
                                "src1_sel:DWORD" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 5)
            CHAINS(asm volatile("v_and_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:DWORD "
                                "src1_sel:DWORD" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 6) CHAINS(asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "s"(s), "v"(w[i])))
        if constexpr (K == 7) CHAINS(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 8) CHAINS(asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 9)
            CHAINS(asm volatile("v_mul_f32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
                                "src1_sel:DWORD" : "+v"(v[i]) : "v"(w[i])))
        if constexpr (K == 10) CHAINS(asm volatile("v_mov_b32 %0, %1" : "=v"(v[i]) : "v"(w[i] + v[i])))
        if constexpr (K == 11) CHAINS(asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(v[i]) : "s"(s), "v"(w[i])))
    }
    unsigned int acc = 0;
    for (int i = 0; i < 8; ++i) acc += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int K>
void run(const char* name, unsigned int* out, unsigned long long* clk)
{
    hipLaunchKernelGGL(k_sdwa<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_sdwa<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
    const double per = ms / 5 * 1e-3 / (2048.0 * 8 * 4); // seconds per wave-instruction per SIMD
    printf("%-44s %.2f cycles per wave-instruction per SIMD (clock %.2f GHz)\n", name, per * ghz * 1e9, ghz);
}

int main()
{
    unsigned int* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, 256 * 1024 * sizeof(unsigned int));
    (void)hipMalloc(&clk, 16);
    run<0>("v_perm_b32", out, clk);
    run<1>("v_mov_b32_sdwa byte1<-byte2 preserve", out, clk);
    run<2>("v_and_b32_sdwa byte1<-byte2&v preserve", out, clk);
    run<3>("v_and_b32_sdwa byte1<-byte2&s preserve", out, clk);
    run<4>("v_add_u32_sdwa word0+dword", out, clk);
    run<5>("v_and_b32_sdwa ->word0 pad", out, clk);
    run<6>("v_and_or_b32", out, clk);
    run<7>("v_mul_u32_u24", out, clk);
    run<8>("v_and_b32", out, clk);
    run<9>("v_mul_f32_sdwa", out, clk);
    run<10>("v_mov_b32 (+ v_add_u32)", out, clk);
    run<11>("v_bfi_b32", out, clk);
    return 0;
}
